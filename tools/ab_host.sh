#!/bin/bash
# A/B of the PCIe-inclusive rate (value_host_inputs) of libdm variants (GPU
# box, repo root): bash tools/ab_host.sh ROUNDS STEPS tag ... (base = dm/libdm.so)
set -o pipefail
OUT=gpurun_out/ab_host.log
: > $OUT
R=$1; ST=$2; shift 2
D=distributed-autonomous-exploration-and-mapping_amd/dm
for r in $(seq $R); do
  for t in "$@"; do
    lib=$D/libdm_$t.so; [ $t = base ] && lib=$D/libdm.so
    DM_LIB=$PWD/$lib timeout -k 10 150 python -u bench.py --steps $ST --warmup 40 --cpu-seconds 0 --profile-steps 2 \
      --no-explored > gpurun_out/ab_host_tmp.log 2>&1 || { echo "$t failed"; tail -5 gpurun_out/ab_host_tmp.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab_host_tmp.log').read().strip().splitlines()[-1])
print('$t', 'value', round(d['value']/1e9, 1), 'host_inputs', round(d['value_host_inputs']/1e9, 1), 'e9', 'host ms/step', round(d['host_inputs']['ms_per_step']*1e3, 1))
" | tee -a $OUT
  done
done
