"""Factors that turn rocprofv3's FETCH_SIZE / WRITE_SIZE (KiB) into bytes for
each access shape of tools/native/fetch_probe.hip: factor = known bytes /
(counter * 1024).  MI355X_MICROARCH.md §HBM documents 2.0 for 16-B-per-lane
streaming reads and 1.0 for 16-B streaming stores; the other shapes are what
this calibrates.  Usage: python tools/fetch_calib.py OUTDIR profiles/fetch_calibration.json"""
import collections
import csv
import glob
import json
import os
import sys


def counters(outdir):
    agg = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(outdir, "p*", "**", "run_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].strip()
            agg[name][r["Counter_Name"]] = float(r["Counter_Value"])
    return agg


def main(outdir, out):
    known = json.load(open(os.path.join(outdir, "known.json")))
    got = counters(outdir)
    res = {"source": "tools/native/fetch_probe.hip under rocprofv3 --pmc (tools/fetch_calib.sh)",
           "shapes": {}}
    for k, kb in known.items():
        c = got.get(k, {})
        e = {"known_read_bytes": kb["read"], "known_write_bytes": kb["write"],
             "FETCH_SIZE_KiB": c.get("FETCH_SIZE"), "WRITE_SIZE_KiB": c.get("WRITE_SIZE")}
        if kb["read"] and c.get("FETCH_SIZE"):
            e["fetch_factor"] = kb["read"] / (c["FETCH_SIZE"] * 1024.0)
        if kb["write"] and c.get("WRITE_SIZE"):
            e["write_factor"] = kb["write"] / (c["WRITE_SIZE"] * 1024.0)
        res["shapes"][k] = e
        print(f"{k:14s} fetch x{e.get('fetch_factor', float('nan')):6.3f}  write x{e.get('write_factor', float('nan')):6.3f}")
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
