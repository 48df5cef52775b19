R=$PWD; OUT=$R/gpurun_out; D=$R/distributed-autonomous-exploration-and-mapping_amd/dm
cd /tmp && export TMPDIR=/tmp
for v in base fe2 fe2rb3; do
  lib=$D/libdm_$v.so; [ $v = base ] && lib=$D/libdm.so
  args=""; [ $v = fe2rb3 ] && args="--depth 3"
  DM_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr_$v -o run --output-format csv -- python3 $R/bench.py --steps 60 --warmup 20 --cpu-seconds 0 --no-explored --no-host-inputs --profile-steps 2 $args > $OUT/tr_$v.log 2>&1 || exit 1
done
