"""Print a rocprofv3 kernel_stats.csv as a short table (kernel, calls, avg/min us, %)."""
import csv
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv"
for r in csv.DictReader(open(path)):
    m = re.search(r"(k_\w+|__amd\w+)", r["Name"])
    n = m.group(1) if m else r["Name"][:30]
    print(f"{n:32s} calls={r['Calls']:>5} avg_us={float(r['AverageNs']) / 1e3:8.2f} "
          f"min_us={float(r['MinNs']) / 1e3:8.2f} pct={float(r['Percentage']):5.1f}")
