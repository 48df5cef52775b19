"""GPU: `bench.py --gpus N` started the way the driver starts `--gpus 1` (no
launcher, no WORLD_SIZE) spawns its own N rank processes and prints one JSON
line whose n_gpus / world size / per-rank records say so.  The box has one GPU
and RCCL needs one GPU per rank, so the ranks share cuda:0 over gloo
(--backend gloo --device-override 0): the same process layout, band handles
and device exchange (dm/sharded.py) as an RCCL run on a node.  The N = 1 leg
runs in-process (no spawn) and reports the same fields as before."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "3", "--warmup", "1", "--pool", "2", "--cpu-seconds", "0", "--no-explored",
         "--no-host-inputs", "--profile-steps", "2", "--grid", "4096", "--robots", "8", "--beams", "1024"]


def _run(args, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, "-u", os.path.join(REPO, "bench.py")] + args, env=env,
                         capture_output=True, text=True, timeout=timeout, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]  # ONE JSON line, from rank 0 only
    return json.loads(lines[0])


def test_bench_self_spawns_two_ranks():
    d = _run(["--gpus", "2", "--backend", "gloo", "--device-override", "0"] + SMALL)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["steps"] == 3
    r = d["ranks"]
    assert r["world_size"] == 2 and r["backend"] == "gloo"
    assert r["launcher"].startswith("bench.py --gpus N")
    assert len(r["ms_per_step"]) == 2 and all(t > 0 for t in r["ms_per_step"])
    # value = all ranks' updates / the slowest rank's timed region
    assert abs(d["ms_per_step"] - max(r["ms_per_step"])) < 1e-9
    assert abs(d["value"] - sum(r["updates"]) / (d["ms_per_step"] * 1e-3 * d["steps"])) < 1e-6 * d["value"]
    assert d["exchange_fallbacks"] == sum(r["exchange_fallbacks"])
    assert d["config"]["grid"] == [4096, 8192] and d["config"]["parallelism"] == "row-bands x2"
    # per-rank exchange phases (HIP events / libdm timers) and the bytes model
    x = r["exchange_ms_per_pass"]
    for k in ("halo", "export", "records_gather", "merge"):
        assert len(x[k]) == 2 and all(v == v and v >= 0 for v in x[k]), (k, x)
    assert x["passes_timed"] >= 2
    b = r["exchange_bytes_per_pass"]
    assert b["halo_row_bytes"] == 4096 and b["records_gathered_per_rank"] == 2 * b["record_bytes"]
    assert b["record_bytes"] == 64 + 8 * 4096 + 32 * b["rec_cap"]
    assert r["records_comm"] == "shared" and "neighbour bands" in d["exchange"]


def test_bench_one_gpu_runs_in_process():
    d = _run(["--gpus", "1"] + SMALL)
    assert d["n_gpus"] == 1 and d["ranks"] is None
    assert d["config"]["grid"] == [4096, 4096] and d["config"]["parallelism"] == "single GPU"
    assert d["value"] > 0 and d["roofline"]["frac"] > 0
