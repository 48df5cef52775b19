set -o pipefail
D=distributed-autonomous-exploration-and-mapping_amd/dm
: > gpurun_out/ord.log
for r in 1 2; do
  for spec in "eb2:libdm.so:--order eb --depth 2" "be1:libdm.so:--order be --depth 1" "eb1:libdm.so:--order eb --depth 1" "be2:libdm_rb3.so:--order be --depth 2" "eb3:libdm_rb3.so:--order eb --depth 3"; do
    tag=${spec%%:*}; rest=${spec#*:}; lib=${rest%%:*}; args=${rest#*:}
    DM_LIB=$PWD/$D/$lib timeout -k 10 120 python -u bench.py --steps 400 --warmup 40 --cpu-seconds 0 --profile-steps 0 --no-explored --no-host-inputs $args > gpurun_out/ord_tmp.out 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/ord_tmp.out; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/ord_tmp.out').read().strip().splitlines()[-1])
print('$tag', round(d['value']/1e9, 1), 'e9', round(d['ms_per_step']*1e3, 1), 'us/step', 'p50', round(d['step_wall_us']['p50'], 1))" | tee -a gpurun_out/ord.log
  done
done
