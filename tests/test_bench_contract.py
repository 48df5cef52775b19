"""CPU: the committed bench lines (profiles/) keep the bench.py contract
(DESIGN.md §5): metric / value / unit / steps fields, a roofline object whose
frac is achieved / peak, a cpu_baseline object, and the configs named by
BASELINE.json.  Also checks that bench.py's option parser knows every config
without touching a GPU."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROFILES = os.path.join(REPO, "profiles")

LINES = {
    "r01_fused_bench.json": "C3",
    "r01_c1_replay_bench.json": "C1",
    "r01_c2_replay_bench.json": "C2",
    "r01_c4_1gpu_bench.json": "C4",
    "r01_c5_sweep_bench.json": "C5",
    "r02_bench.json": "C3",
    "r02_c1_bench.json": "C1",
    "r02_c2_bench.json": "C2",
    "r02_c4_bench.json": "C4",
    "r02_c5_bench.json": "C5",
}


def _load(name):
    path = os.path.join(PROFILES, name)
    if not os.path.exists(path):
        pytest.skip(f"{name} not committed")
    with open(path) as f:
        return json.loads(f.readline())


@pytest.mark.parametrize("name,cfg", sorted(LINES.items()))
def test_bench_line_fields(name, cfg):
    d = _load(name)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["unit"] == "beam-cell updates/s" and d["higher_is_better"] is True
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["workload"].startswith(cfg)
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9
    cpu = d.get("cpu_baseline")
    if cpu is not None:
        assert cpu["kind"] in ("port", "reference") and cpu["cores"] >= 1 and cpu["sample"]


def test_headline_line_has_traffic_and_cpu_baseline():
    d = _load("r01_fused_bench.json")
    assert d["n_gpus"] == 1 and d["scaling"] == "weak"
    assert d["roofline"]["traffic"] and d["roofline"]["traffic"] > 0
    assert d["cpu_baseline"] and d["cpu_baseline"]["value"] > 0
    # the north-star targets (BASELINE.json): >= 1e10 updates/s, < 2 ms frontiers
    assert d["value"] >= 1e10 and d["frontier_ms"] < 2.0


def test_r02_headline_fields():
    """Round 2's C3 line: the frontier and atomic rooflines, the explored-map
    frontier pass, the host-input rate and the step cadence record."""
    d = _load("r02_bench.json")
    r = d["roofline"]
    assert r["traffic"] and r["traffic"] > 0
    fr = r["frontier"]
    assert fr["bound"] == "hbm" and abs(fr["frac"] - fr["achieved"] / fr["peak"]) < 1e-9
    at = r["atomics"]
    assert at["peak"] > 0 and 0 < at["frac"] <= 1.5
    assert d["frontier_ms_explored"] and d["frontier_ms_explored"] < 2.0
    assert d["value_host_inputs"] and d["value_host_inputs"] >= 1e10
    c = d["step_wall_us"]
    assert c["n"] == d["steps"] and c["p50"] <= c["p90"] <= c["max"]
    assert d["value"] >= 1e10 and d["frontier_ms"] < 2.0 and d["cpu_baseline"]["value"] > 0


def test_bench_spawned_ranks_fail_together():
    """`--gpus 2` without a launcher spawns two rank processes; here (no GPU)
    they fail at the device call, and bench.py must exit non-zero promptly
    rather than hang or report a line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1",
                          "--cpu-seconds", "0"], capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode != 0
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]


def test_bench_parser_knows_every_config():
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--help"],
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    for cfg in ("C1", "C2", "C3", "C4", "C5"):
        assert cfg in out.stdout


def test_r06_headline_fields():
    """Round 6's final C3 line: the measured traffic and the design's own byte
    model beside the SURVEY model's `frac`, and the two agree."""
    d = _load("r06_final_bench.json")
    r = d["roofline"]
    assert r["traffic"] and r["frac_traffic"] and r["frac_hbm_model"]
    assert r["frac_hbm_model"] < r["frac"]  # the SURVEY model counts LDS-resident counter bytes
    assert abs(r["frac_hbm_model"] - r["frac_traffic"]) < 0.1 * r["frac_traffic"]
    assert d["value"] >= 1e10 and d["frontier_ms"] < 2.0 and d["value_host_inputs"] >= 1e10


def test_hbm_model_applies_only_where_dense_items_dominate():
    sys.path.insert(0, REPO)
    import bench

    dense = bench.hbm_model({"active_tiles": 3000.0, "pieces": 600000.0, "sparse_items": 10.0}, 0.048, 5e6)
    assert dense["hbm_model_applies"] and 0 < dense["frac_hbm_model"] < 1
    sparse = bench.hbm_model({"active_tiles": 20000.0, "pieces": 45000.0, "sparse_items": 19000.0}, 0.09, 1e6)
    assert not sparse["hbm_model_applies"] and sparse["frac_hbm_model"] is None
    assert sparse["frac_hbm_touched"] > 0
