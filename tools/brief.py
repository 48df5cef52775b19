"""Print the key numbers of a bench JSON line (gpurun_out/bench.log by default)."""
import json
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench.log"
d = json.loads([l for l in open(path) if l.startswith("{")][-1])
for k in ("value", "ms_per_step", "frontier_ms", "integrate_ms", "value_host_inputs", "frontier_ms_explored",
          "clusters"):
    print(f"{k:22s} {d.get(k)}")
r = d.get("roofline") or {}
print("tile_accum frac", r.get("frac"), "avg ms", r.get("avg_launch_ms"), "traffic", r.get("traffic"))
if r.get("atomics"):
    print("atomics frac", r["atomics"]["frac"])
fr = r.get("frontier") or {}
print("frontier device ms", fr.get("device_ms"), "frac", fr.get("frac"), "frac_traffic", fr.get("frac_traffic"))
print("kernels", {k: round(v * 1e3, 1) for k, v in d.get("kernel_avg_ms", {}).items()})
ex = d.get("frontier_explored")
if ex:
    print("explored", round(ex["frontier_ms"], 4), {k: round(v * 1e3, 1) for k, v in ex["roofline"]["kernels_ms"].items()},
          "frac", ex["roofline"]["frac"])
