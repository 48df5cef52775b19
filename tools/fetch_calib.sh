#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/native/
# fetch_probe.hip): two rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE
# cannot share one: 3 + 2 of the 4 TCC counters), then the factors.
# Usage on the GPU box, from the repo root:  bash tools/fetch_calib.sh [OUTDIR]
set -o pipefail
R=$PWD
OUT=${1:-gpurun_out/fetch_calib}
mkdir -p $R/$OUT
BIN=$R/tools/native/fetch_probe
[ -x $BIN ] || { echo "build $BIN first (make -C tools/native)"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 $BIN > $R/$OUT/known.json || { echo "probe failed"; exit 1; }
i=0
for group in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $group --kernel-trace --output-format csv -d $R/$OUT/p$i -o run \
    -- $BIN > $R/$OUT/p$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; exit 1; }
done
python3 $R/tools/fetch_calib.py $R/$OUT $R/profiles/fetch_calibration.json
