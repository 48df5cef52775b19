"""Per-step kernel record of a bench run from a rocprofv3 kernel trace.

Steps are delimited by consecutive k_tile_accum starts (one accumulation per
step).  For the accumulations [first, last) it prints the start-to-start
period and every kernel's duration inside that period, so the steps right
after band.reset() (the driver's 5 warm-up + 20 timed steps) can be compared
with steady-state steps of the same trace.

Usage: python tools/step_kernels.py TRACE.csv [first] [last]
   bench.py --steps 20 --warmup 5: the counts loop runs 6 accumulations, so
   the warm-up steps are accumulations 6..10 and the timed steps 11..30.
"""
import csv
import re
import sys
from collections import defaultdict

path = sys.argv[1]
first = int(sys.argv[2]) if len(sys.argv) > 2 else 6
last = int(sys.argv[3]) if len(sys.argv) > 3 else 32
rows = []
for r in csv.DictReader(open(path)):
    m = re.search(r"(k_\w+|__amd\w+)", r["Kernel_Name"])
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:20]))
rows.sort()
acc = [r for r in rows if r[2] == "k_tile_accum"]
short = {"k_tile_accum": "acc", "k_beam_prep": "prep", "k_plan": "plan", "k_scatter": "scat",
         "k_frontier_bits": "bits", "k_frontier_tile_big": "big", "k_frontier_tile": "wave",
         "k_frontier_resolve": "res", "k_rank_sort": "sort", "k_list_tiles": "list",
         "k_fmask_items": "fmi", "k_integrate_reset": "rst", "k_seq_gate": "gate", "k_seq_signal": "sig"}
cols = ["acc", "prep", "plan", "scat", "bits", "big", "wave", "res", "sort", "list", "gate"]
print(f"{'step':>4} {'period':>7} " + " ".join(f"{c:>6}" for c in cols) + "  other")
for i in range(first, min(last, len(acc) - 1)):
    t0, t1 = acc[i][0], acc[i + 1][0]
    d = defaultdict(float)
    other = defaultdict(float)
    for s, e, n in rows:
        if t0 <= s < t1:
            k = short.get(n)
            if k in cols:
                d[k] += (e - s) / 1e3
            else:
                other[k or n] += (e - s) / 1e3
    print(f"{i:4d} {(t1 - t0) / 1e3:7.1f} " + " ".join(f"{d[c]:6.1f}" for c in cols) + "  " +
          " ".join(f"{k}={v:.1f}" for k, v in sorted(other.items()) if k not in ("rst", "sig")))
