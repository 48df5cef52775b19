"""Host API calls interleaved with kernel executions from one rocprofv3 run
with --hip-trace --kernel-trace (both in the same clock): prints a window of
the pipelined bench around k_tile_accum number N, relative to its start.
Usage: python tools/host_gpu_trace.py DIR [N] [count]"""
import csv
import re
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 70
cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 2
ev = []
for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
    m = re.search(r"(k_\w+|__amd\w+)", r["Kernel_Name"])
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + (m.group(1) if m else "?") +
               " q" + r.get("Queue_Id", "?")))
skip = {"hipGetLastError", "__hipPushCallConfiguration", "__hipPopCallConfiguration", "hipSetDevice"}
for r in csv.DictReader(open(f"{d}/run_hip_api_trace.csv")):
    if r["Function"] not in skip:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "   H " + r["Function"]))
ev.sort()
acc = [i for i, e in enumerate(ev) if e[2].startswith("K k_tile_accum")]
a, b = acc[n], acc[min(n + cnt, len(acc) - 1)]
t0 = ev[a][0]
for s, e, name in ev[a - 30:b + 1]:
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} ({(e - s) / 1e3:6.1f}) {name}")
per = [(ev[acc[i + 1]][0] - ev[acc[i]][0]) / 1e3 for i in range(len(acc) - 1)]
per.sort()
print("k_tile_accum start-to-start: median %.1f us" % per[len(per) // 2])
