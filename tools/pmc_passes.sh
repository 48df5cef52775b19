#!/bin/bash
# PMC passes over one workload (one rocprofv3 --pmc run per counter group:
# rocprofv3 does not split counters over passes, MI355X_MICROARCH.md §PMC).
# Usage (on the GPU box, from the repo root):
#   bash tools/pmc_passes.sh OUTDIR [command...]
# default command: a short C3 bench run, steps back to back (--no-overlap):
# rocprofv3 --pmc runs one dispatch at a time, and the overlapped pipeline's
# cross-stream gates would wait for kernels queued behind them (DM_ERR_PIPELINE).
# Summarise with
#   python tools/pmc_summary.py OUTDIR profiles/pmc_latest.json WORKLOAD
set -o pipefail
R=$PWD
OUT=${1:-gpurun_out/pmc}
shift
CMD=("$@")
[ ${#CMD[@]} -eq 0 ] && CMD=(python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --profile-steps 0 --pool 3 \
                             --no-explored --no-host-inputs --no-overlap)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for group in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
             "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $group --kernel-trace --output-format csv -d $R/$OUT/p$i -o run \
    -- "${CMD[@]}" > $R/$OUT/p$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; exit 1; }
  echo "pmc pass $i ok"
done
