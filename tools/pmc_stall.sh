#!/bin/bash
# One PMC pass of issue / stall counters (SQ: 8 slots) over a short C3 bench
# run (steps back to back: rocprofv3 --pmc runs one dispatch at a time).
# Usage (GPU box, repo root): bash tools/pmc_stall.sh OUTDIR [DM_LIB=...]
# Summarise with: python tools/pmc_stall.py OUTDIR
set -o pipefail
R=$PWD
OUT=${1:-gpurun_out/pmc_stall}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM --kernel-trace \
  --output-format csv -d $R/$OUT/p1 -o run -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 \
  --profile-steps 0 --pool 3 --no-explored --no-host-inputs --no-overlap > $R/$OUT/p1.log 2>&1 \
  || { echo "pmc stall pass failed rc=$?"; exit 1; }
echo "pmc stall pass ok"
