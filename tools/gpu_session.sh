#!/bin/bash
# One GPU-box session: parity tests -> bench (with CPU baseline) -> 2-rank
# sharded rehearsal (gloo, both ranks on GPU 0) -> rocprofv3 kernel stats ->
# PMC passes.  Stops at the first step that crashes, aborts or times out.
# Usage: bash tools/gpu_session.sh [tests|bench|shard|prof|pmc]...  (default: all)
set -o pipefail
R=$PWD
OUT=$R/gpurun_out
mkdir -p $OUT
steps="${@:-tests bench shard prof pmc}"
ok() { [ "$1" -eq 0 ]; }
for s in $steps; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
      rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed" $OUT/pytest_gpu.log | tail -6
      [ $rc -le 1 ] || exit $rc ;;
    bench)
      timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log; ok $rc || exit $rc ;;
    shard)
      timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --device-override 0 \
        --cpu-seconds 0 --pool 3 > $OUT/shard.log 2>&1
      rc=$?; echo "shard rc=$rc"; tail -1 $OUT/shard.log; ok $rc || exit $rc ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run \
        --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/prof.log 2>&1)
      rc=$?; echo "prof rc=$rc"; ok $rc || exit $rc ;;
    pmc)
      bash $R/tools/pmc_passes.sh gpurun_out/pmc; rc=$?; ok $rc || exit $rc ;;
  esac
done
