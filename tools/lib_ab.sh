#!/bin/bash
# libdm variant A/B on the GPU box (repo root): each tag is a library built
# with `make variant V=tag D=...` (dm/libdm_<tag>.so; "base" = dm/libdm.so).
#   bash tools/lib_ab.sh ROUNDS "C3|C5:SWEEP" tag1 tag2[:VAR=V,VAR2=W] ...
# Prints value / us per step (C3) or per-sweep-point ms (C5) -> gpurun_out/lib_ab.log
set -o pipefail
OUT=gpurun_out/lib_ab.log
: > $OUT
R=$1; W=$2; shift 2
D=distributed-autonomous-exploration-and-mapping_amd/dm
for r in $(seq $R); do
  for spec in "$@"; do
    tag=$spec; lt=${spec%%:*}; envs=""; [ "$lt" != "$spec" ] && envs=${spec#*:}
    lib=$D/libdm_$lt.so; [ $lt = base ] && lib=$D/libdm.so
    if [ "${W%%:*}" = C5 ]; then
      env ${envs//,/ } DM_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --config C5 --sweep ${W#C5:} --cpu-seconds 0 \
        > gpurun_out/lib_ab_tmp.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/lib_ab_tmp.log; exit 1; }
      python -c "
import json; d=json.loads(open('gpurun_out/lib_ab_tmp.log').read().strip().splitlines()[-1])
for p in d.get('sweep', []): print('$tag', 'beams', p.get('beams_per_scan'), 'ms/step', round(p.get('ms_per_step', 0), 3), 'int', round(p.get('integrate_ms', 0), 3), 'fr', round(p.get('frontier_ms', 0), 3), {k: round(v*1e3, 1) for k, v in (p.get('kernel_avg_ms') or {}).items()})
" | tee -a $OUT
    else
      env ${envs//,/ } DM_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --steps 400 --warmup 40 --cpu-seconds 0 --profile-steps 10 \
        --no-explored --no-host-inputs > gpurun_out/lib_ab_tmp.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/lib_ab_tmp.log; exit 1; }
      python -c "
import json; d=json.loads(open('gpurun_out/lib_ab_tmp.log').read().strip().splitlines()[-1])
print('$tag', round(d['value']/1e9, 1), 'e9', round(d['ms_per_step']*1e3, 1), 'us/step', {k: round(v*1e3, 1) for k, v in d['kernel_avg_ms'].items()})
" | tee -a $OUT
    fi
  done
done
