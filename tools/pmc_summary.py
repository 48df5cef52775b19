"""Summarise rocprofv3 --pmc passes (tools/pmc_passes.sh) per kernel.

HBM traffic per dispatch, following MI355X_MICROARCH.md §HBM: FETCH_SIZE /
WRITE_SIZE are in KiB and their byte factor depends on the access shape
(2.0 for 16-B-per-lane streaming reads; other widths "uncalibrated").  The
factors come from profiles/fetch_calibration.json (tools/fetch_calib.sh:
known byte counts in each shape libdm uses), mapped per kernel by KERNEL_SHAPE
below; a kernel with no calibrated shape uses the documented 2.0 / 1.0.
`traffic_raw_bytes` keeps the uncorrected counters.  Usage:
    python tools/pmc_summary.py gpurun_out/pmc profiles/pmc_latest.json WORKLOAD
The output holds one entry per workload (C3, C3-explored, ...) measured on
the same sources; a summary from other sources is replaced, not merged.
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from src_hash import src_hash  # noqa: E402


# the probe shape (tools/native/fetch_probe.hip) closest to each kernel's
# dominant HBM traffic
KERNEL_SHAPE = {
    "k_tile_accum": "probe_accum",       # L float4 + state char4 rows, loaded then stored
    "k_frontier_bits": "probe_bits",     # 1 KiB fmask record per listed tile, u64 per lane
    "k_frontier_tile": "probe_ld8",      # fbits words, u64 per lane
    "k_frontier_tile_big": "probe_ld8",
    "k_recount": "probe_ld4",
}
DEFAULT_FACTORS = (2.0, 1.0)  # MI355X_MICROARCH.md: 16-B streaming reads / stores


def factors(kernel, calib):
    shape = KERNEL_SHAPE.get(kernel)
    e = (calib or {}).get("shapes", {}).get(shape or "", {})
    f = e.get("fetch_factor", DEFAULT_FACTORS[0])
    w = e.get("write_factor", DEFAULT_FACTORS[1])
    return f, w, (shape if e else "documented 16-B streaming (2.0 / 1.0)")


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main(pmc_dir, out, workload):
    kern = collections.defaultdict(dict)
    for sub in sorted(os.listdir(pmc_dir)):
        f = os.path.join(pmc_dir, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for k, counters in load(f).items():
            for c, vals in counters.items():
                kern[k][c] = sum(vals) / len(vals)
    try:
        calib = json.load(open(os.path.join(os.path.dirname(os.path.abspath(out)), "fetch_calibration.json")))
    except (OSError, ValueError):
        calib = None
    h = src_hash()
    try:
        res = json.load(open(out))
        if res.get("src_hash") != h or "workloads" not in res:
            res = None
    except (OSError, ValueError):
        res = None
    res = res or {"src_hash": h, "workloads": {}}
    entry = {"kernels": {}}
    res["workloads"][workload] = entry
    for k, c in kern.items():
        e = dict(c)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            f, w, shape = factors(k, calib)
            e["traffic_bytes"] = (f * c["FETCH_SIZE"] + w * c["WRITE_SIZE"]) * 1024.0
            e["traffic_raw_bytes"] = (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
            e["traffic_factors"] = {"fetch": f, "write": w, "shape": shape}
        if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
            e["wait_frac"] = c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"]
            e["active_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0.0) / c["SQ_WAVE_CYCLES"]
        entry["kernels"][k] = e
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, e in sorted(entry["kernels"].items()):
        if "traffic_bytes" in e:
            print(f"{k:24s} traffic {e['traffic_bytes']/1e6:8.1f} MB  wait {e.get('wait_frac', 0):.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "C3")
