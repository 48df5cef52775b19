#!/bin/bash
# Host-input (PCIe-inclusive) A/B on the GPU box (repo root): each tag is a
# library built with `make variant V=tag D=...` (dm/libdm_<tag>.so; "base" =
# dm/libdm.so).  One C3 bench run per tag and round, with value_host_inputs.
#   bash tools/h2d_ab.sh ROUNDS tag1 tag2[:VAR=V,VAR2=W] ...   -> gpurun_out/h2d_ab.log
set -o pipefail
OUT=gpurun_out/h2d_ab.log
: > $OUT
R=$1; shift
D=distributed-autonomous-exploration-and-mapping_amd/dm
for r in $(seq $R); do
  for spec in "$@"; do
    tag=$spec; lt=${spec%%:*}; envs=""; [ "$lt" != "$spec" ] && envs=${spec#*:}
    lib=$D/libdm_$lt.so; [ $lt = base ] && lib=$D/libdm.so
    env ${envs//,/ } DM_LIB=$PWD/$lib timeout -k 10 150 python -u bench.py --steps 400 --warmup 40 --cpu-seconds 0 --profile-steps 0 \
      --no-explored > gpurun_out/h2d_ab_tmp.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/h2d_ab_tmp.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/h2d_ab_tmp.log').read().strip().splitlines()[-1])
h=d['host_inputs']
print('$tag', 'device', round(d['value']/1e9, 1), 'e9', round(d['ms_per_step']*1e3, 1), 'us/step;',
      'host inputs', round(h['value']/1e9, 1), 'e9', round(h['ms_per_step']*1e3, 1), 'us/step')
" | tee -a $OUT
  done
done
