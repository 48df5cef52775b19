"""Per-call GPU timeline from a rocprofv3 kernel trace: for each integrate
call (k_integrate_reset .. the accumulation) and frontier call (k_frontier_bits
.. k_rank_sort), the span from the first kernel's start to the last kernel's
end, the summed kernel time, and the gaps between consecutive kernels.
Usage: python tools/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv"""
import csv
import re
import statistics
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv")):
    m = re.search(r"(k_\w+|__amd\w+)", r["Kernel_Name"])
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:20]))
rows.sort()
calls = {"integrate": ("k_integrate_reset", "k_tile_accum"), "frontier": ("k_frontier_bits", "k_rank_sort")}
for name, (first, last) in calls.items():
    spans, busy, gaps, prev_end = [], [], [], {}
    cur = None
    for s, e, k in rows:
        if k == first:
            cur = [s, e, e - s, []]
        elif cur is not None:
            cur[3].append(s - cur[1])
            cur[1] = e
            cur[2] += e - s
            if k == last:
                spans.append(cur[1] - cur[0])
                busy.append(cur[2])
                gaps.append(sum(cur[3]))
                cur = None
    if spans:
        print(f"{name:10s} calls={len(spans):3d} span_us={statistics.median(spans) / 1e3:7.1f} "
              f"kernels_us={statistics.median(busy) / 1e3:7.1f} gaps_us={statistics.median(gaps) / 1e3:6.1f}")
