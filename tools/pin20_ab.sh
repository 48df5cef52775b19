set -o pipefail
: > gpurun_out/pin20.log
for r in 1 2 3 4 5; do
  for m in off auto; do
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-explored --no-host-inputs --profile-steps 0 --pin-host $m > gpurun_out/pin20_tmp.log 2>&1 || { echo "$m failed"; tail -5 gpurun_out/pin20_tmp.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/pin20_tmp.log').read().strip().splitlines()[-1])
print('$m', round(d['value']/1e9, 1), round(d['step_wall_us']['p50'], 1), d['host_cpus'])" | tee -a gpurun_out/pin20.log
  done
done
