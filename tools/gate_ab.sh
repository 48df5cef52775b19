#!/bin/bash
# A/B of the cross-stream hand-offs (GPU box, repo root): C3 bench value with
# the seq gates (default), the front-end hand-off by an event wait
# (DM_FE_GATE=0), and both hand-offs by event waits (+ DM_PASS_GATE=0);
# two alternating rounds.  Output: gpurun_out/gate_ab.log
set -o pipefail
OUT=gpurun_out/gate_ab.log
: > $OUT
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 400 --warmup 40 --cpu-seconds 0 --profile-steps 0 \
    --no-explored --no-host-inputs > gpurun_out/ab_tmp.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/ab_tmp.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_tmp.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e9,1), 'e9', round(d['ms_per_step']*1e3,1), 'us/step', 'p50', round(d['step_wall_us']['p50'],1))" | tee -a $OUT
}
for r in 1 2; do
  run gates DM_FE_GATE=1 || exit 1
  run fe_event DM_FE_GATE=0 || exit 1
  run both_events DM_FE_GATE=0 DM_PASS_GATE=0 || exit 1
done
