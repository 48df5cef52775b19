"""Kernel timeline of a few consecutive steps from a rocprofv3 kernel trace
(pipelined bench: two streams).  Prints each kernel's start / end relative
to the step's first k_tile_accum start, and the period between consecutive
k_rank_sort ends.  Usage: python tools/timeline.py [trace.csv] [first_step]"""
import csv
import re
import statistics
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
first = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rows = []
for r in csv.DictReader(open(path)):
    m = re.search(r"(k_\w+|__amd\w+)", r["Kernel_Name"])
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:20]))
rows.sort()
accum = [i for i, r in enumerate(rows) if r[2] == "k_tile_accum"]
sorts = [r[1] for r in rows if r[2] == "k_rank_sort"]
periods = [b - a for a, b in zip(sorts, sorts[1:])]
print(f"rank_sort end-to-end period: median {statistics.median(periods) / 1e3:.1f} us "
      f"(min {min(periods) / 1e3:.1f}) over {len(periods)} steps")
for k in range(first, min(first + 2, len(accum) - 1)):
    t0 = rows[accum[k]][0]
    print(f"-- step from k_tile_accum #{k}")
    for s, e, name in rows[accum[k] - 6:accum[k + 1] + 1]:
        print(f"  {name:26s} {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f}  ({(e - s) / 1e3:5.1f})")

# main-stream gaps per step (pipelined region): rank_sort end -> next
# accumulation start, accumulation end -> bit rows start, bit rows end -> tile start
def gaps(a, b):
    out = []
    ends = [r for r in rows if r[2] == a]
    starts = [r for r in rows if r[2] == b]
    j = 0
    for s, e, _ in ends:
        while j < len(starts) and starts[j][0] < e:
            j += 1
        if j < len(starts):
            out.append((starts[j][0] - e) / 1e3)
    return out


for a, b in (("k_rank_sort", "k_tile_accum"), ("k_frontier_bits", "k_frontier_tile_big"),
             ("k_frontier_tile_big", "k_frontier_resolve"), ("k_frontier_resolve", "k_rank_sort"),
             ("k_tile_accum", "k_frontier_bits"), ("k_scatter", "k_tile_accum")):
    g = gaps(a, b)[5:30]
    if g:
        print(f"gap {a} -> {b}: median {statistics.median(g):.1f} us, min {min(g):.1f}")
