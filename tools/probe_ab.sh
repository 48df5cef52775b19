#!/bin/bash
# explored-map frontier probe per library variant (GPU box, repo root):
#   bash tools/probe_ab.sh ROUNDS tag1 tag2 ...  -> gpurun_out/probe_ab.log
set -o pipefail
D=distributed-autonomous-exploration-and-mapping_amd/dm
: > gpurun_out/probe_ab.log
for r in $(seq $1); do
  for tag in "${@:2}"; do
    lib=$D/libdm_$tag.so; [ $tag = base ] && lib=$D/libdm.so
    DM_LIB=$PWD/$lib timeout -k 10 120 python -u tools/frontier_probe.py > gpurun_out/probe_tmp.out 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/probe_tmp.out; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/probe_tmp.out').read().strip().splitlines()[-1])
print('$tag', 'explored frontier ms', round(d['frontier_ms'], 4), {k: round(v*1e3, 1) for k, v in d['kernel_avg_ms'].items()})" | tee -a gpurun_out/probe_ab.log
  done
done
