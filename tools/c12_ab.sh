set -o pipefail
D=distributed-autonomous-exploration-and-mapping_amd/dm
: > gpurun_out/c12.log
for r in 1 2; do for tag in prev base; do for c in C1 C2; do
  lib=$D/libdm_$tag.so; [ $tag = base ] && lib=$D/libdm.so
  DM_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --config $c --cpu-seconds 0 > gpurun_out/c12_tmp.out 2>&1 || { echo fail; tail -3 gpurun_out/c12_tmp.out; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/c12_tmp.out').read().strip().splitlines()[-1])
print('$tag $c', 'ms/step %.4f'%d['ms_per_step'], {k: round(v*1e3,1) for k,v in d.get('kernel_avg_ms',{}).items()})" | tee -a gpurun_out/c12.log
done; done; done
