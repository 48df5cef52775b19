"""Cadence of a long bench run in windows: reads a `bench.py --step-trace`
file (per-step host intervals, µs) and writes mean / p50 / p99 / max per
window of N steps (the drain interval at the end is left out).
    python tools/step_windows.py TRACE.json OUT.json [N=2000]"""
import json
import sys

import numpy as np

tr = json.load(open(sys.argv[1]))
n = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
us = np.asarray(tr["step_us"][:-1], float)
out = {"steps": int(us.size + 1), f"windows_of_{n}": []}
for w in range(us.size // n):
    x = us[w * n:(w + 1) * n]
    out[f"windows_of_{n}"].append({"window": w, "mean_us": round(float(x.mean()), 1),
                                   "p50": round(float(np.percentile(x, 50)), 1),
                                   "p99": round(float(np.percentile(x, 99)), 1), "max": round(float(x.max()), 1)})
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out[f"windows_of_{n}"]))
