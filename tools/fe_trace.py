"""Front-end placement in a pipelined C3 kernel trace (rocprofv3 --kernel-trace
CSV): per step k, relative to k_tile_accum(k)'s start, when the next batch's
front-end kernels (k_beam_prep / k_plan / k_scatter of batch k+1) start and
end, when k_tile_accum(k+1) starts, and which hardware queue each kernel ran
on.  Used to check whether a second front-end stream (DM_FE_STREAMS=2) lets
batch k+1's front-end start before batch k's accumulation, and what holds it.

Usage: python tools/fe_trace.py TRACE.csv [first_accum] [n_steps]"""
import csv
import re
import statistics
import sys

path = sys.argv[1]
first = int(sys.argv[2]) if len(sys.argv) > 2 else 40
n = int(sys.argv[3]) if len(sys.argv) > 3 else 12
rows = []
for r in csv.DictReader(open(path)):
    m = re.search(r"(k_\w+|__amd\w+)", r["Kernel_Name"])
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:20],
                 int(r["Queue_Id"])))
rows.sort()
by = {}
for s, e, name, q in rows:
    by.setdefault(name, []).append((s, e, q))
acc = by.get("k_tile_accum", [])
prep = by.get("k_beam_prep", [])
plan = by.get("k_plan", [])
scat = by.get("k_scatter", [])
queues = {name: sorted({q for _, _, q in v}) for name, v in by.items()}
print("queues per kernel:", queues)
# the i-th accumulation consumes the i-th front-end (every call runs all three)
m = min(len(acc), len(prep), len(plan), len(scat))
cols = ["prep(k+1)", "plan(k+1)", "scat(k+1)"]
stats = {c: [] for c in ["prep_start", "prep_end", "scat_end", "accum_next", "accum_len", "period"]}
print(f"{'k':>4} {'accum':>12} " + " ".join(f"{c:>16}" for c in cols) + f" {'accum(k+1)':>10}")
for k in range(first, min(first + n, m - 1)):
    t0, t1, q0 = acc[k]
    f = []
    for lst in (prep, plan, scat):
        s, e, q = lst[k + 1]
        f.append(f"{(s - t0) / 1e3:6.1f}-{(e - t0) / 1e3:6.1f}q{q}")
    an = acc[k + 1][0]
    print(f"{k:4d} {0:5.1f}-{(t1 - t0) / 1e3:5.1f}q{q0} " + " ".join(f"{x:>16}" for x in f) +
          f" {(an - t0) / 1e3:10.1f}")
for k in range(first, m - 1):
    t0, t1, _ = acc[k]
    stats["prep_start"].append((prep[k + 1][0] - t0) / 1e3)
    stats["prep_end"].append((prep[k + 1][1] - t0) / 1e3)
    stats["scat_end"].append((scat[k + 1][1] - t0) / 1e3)
    stats["accum_next"].append((acc[k + 1][0] - t0) / 1e3)
    stats["accum_len"].append((t1 - t0) / 1e3)
print("medians (us from k_tile_accum(k) start):",
      {k: round(statistics.median(v), 1) for k, v in stats.items() if v})
