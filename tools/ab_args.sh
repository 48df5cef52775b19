#!/bin/bash
# C3 A/B of libdm variants with per-variant environment AND bench arguments
# (repo root, GPU box):
#   bash tools/ab_args.sh ROUNDS STEPS spec ...
#   spec = tag[:VAR=V,VAR2=W][@--arg,value,--arg2]   (tag: dm/libdm_<tag>.so, base = dm/libdm.so)
# One bench.py run per spec per round, alternating -> gpurun_out/ab_args.log
set -o pipefail
OUT=gpurun_out/ab_args.log
: > $OUT
R=$1; ST=$2; shift 2
D=distributed-autonomous-exploration-and-mapping_amd/dm
for r in $(seq $R); do
  for spec in "$@"; do
    head=${spec%%@*}; args=""; [ "$head" != "$spec" ] && args=${spec#*@}
    lt=${head%%:*}; envs=""; [ "$lt" != "$head" ] && envs=${head#*:}
    lib=$D/libdm_$lt.so; [ $lt = base ] && lib=$D/libdm.so
    env ${envs//,/ } DM_LIB=$PWD/$lib timeout -k 10 150 python -u bench.py --steps $ST --warmup 40 --cpu-seconds 0 \
      --profile-steps 10 --no-explored --no-host-inputs ${args//,/ } > gpurun_out/ab_args_tmp.log 2>&1 \
      || { echo "$spec failed"; tail -8 gpurun_out/ab_args_tmp.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab_args_tmp.log').read().strip().splitlines()[-1])
c=d.get('step_wall_us') or {}
print('$spec', round(d['value']/1e9, 1), 'e9', round(d['ms_per_step']*1e3, 1), 'us/step p50', round(c.get('p50', 0), 1), 'p90', round(c.get('p90', 0), 1), {k: round(v*1e3, 1) for k, v in d['kernel_avg_ms'].items()})
" | tee -a $OUT
  done
done
