"""Per-kernel issue / stall fractions from tools/pmc_stall.sh (quad-cycle
SQ counters per dispatch, averaged over the kernel's dispatches): each
counter / SQ_WAVE_CYCLES.  Usage: python tools/pmc_stall.py OUTDIR"""
import csv
import glob
import re
import sys
from collections import defaultdict

out = sys.argv[1]
rows = []
for path in glob.glob(f"{out}/p1/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(path)))
acc = defaultdict(lambda: defaultdict(float))
n = defaultdict(set)
for r in rows:
    m = re.search(r"(k_\w+)", r.get("Kernel_Name", ""))
    if not m:
        continue
    k = m.group(1)
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
names = ["SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA",
         "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"]
print(f"{'kernel':24s} {'disp':>4s} " + " ".join(f"{x[3:]:>15s}" for x in names))
for k in sorted(acc):
    wc = acc[k].get("SQ_WAVE_CYCLES", 0.0)
    if wc <= 0:
        continue
    print(f"{k:24s} {len(n[k]):4d} " + " ".join(f"{acc[k].get(x, 0.0) / wc:15.3f}" for x in names))
