#!/bin/bash
# Kernel trace of the pipelined C5 step at one sweep point (GPU box, repo root):
#   bash tools/c5trace.sh BEAMS  -> gpurun_out/c5tr_BEAMS/run_kernel_trace.csv
R=$PWD; OUT=$R/gpurun_out; N=${1:-48}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/c5tr_$N -o run --output-format csv -- python3 $R/bench.py \
  --config C5 --sweep $N --steps 40 --warmup 10 --cpu-seconds 0 > $OUT/c5tr_$N.log 2>&1
