"""Summarise rocprofv3 --pmc passes (tools/pmc_passes.sh) per kernel.

HBM traffic per dispatch, following MI355X_MICROARCH.md §HBM:
  FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
  bytes of a wide (16 B/lane) coalesced read, so bytes = 2*FETCH_SIZE*1024 +
  WRITE_SIZE*1024 is an upper estimate for kernels with narrower reads
  (`traffic_lo` keeps FETCH_SIZE uncorrected).  Usage:
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
            e["traffic_bytes"] = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
            e["traffic_lo_bytes"] = (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
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
