#!/bin/bash
# libdm variant A/B over the scan-replay / shared-map configs (GPU box, repo
# root): bash tools/cfg_ab.sh "C1 C4" spec ...  (spec = tag[:VAR=V,...][@--arg,value,...]; "base" =
# dm/libdm.so, else dm/libdm_<tag>.so; args go to bench.py); prints ms per step and kernel
# times -> gpurun_out/cfg_ab.log
set -o pipefail
OUT=gpurun_out/cfg_ab.log
: > $OUT
CFGS=$1; shift
D=distributed-autonomous-exploration-and-mapping_amd/dm
for c in $CFGS; do
  for spec in "$@"; do
    head=${spec%%@*}; args=""; [ "$head" != "$spec" ] && args=${spec#*@}
    t=${head%%:*}; envs=""; [ "$t" != "$head" ] && envs=${head#*:}
    lib=$D/libdm_$t.so; [ $t = base ] && lib=$D/libdm.so
    env ${envs//,/ } DM_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --config $c --cpu-seconds 0 ${args//,/ } \
      > gpurun_out/cfg_ab_tmp.log 2>&1 || { echo "$c $spec failed"; tail -5 gpurun_out/cfg_ab_tmp.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/cfg_ab_tmp.log').read().strip().splitlines()[-1])
print('$c', '$spec', round(d['ms_per_step']*1e3, 1), 'us/step', {k: round(v*1e3, 1) for k, v in (d.get('kernel_avg_ms') or {}).items()})
" | tee -a $OUT
  done
done
