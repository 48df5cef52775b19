#!/bin/bash
# Environment A/B of the C3 bench (GPU box, repo root), alternating rounds:
#   bash tools/ab.sh ROUNDS "tag:VAR=V,VAR2=V2" "tag2:VAR=W" ...
# Prints value, us/step and the host step cadence per run -> gpurun_out/ab.log
set -o pipefail
# per-tag extra bench.py arguments: BENCH_ARGS_<tag>="--depth 3" in the environment
declare -A BENCH_ARGS
for v in $(env | grep '^BENCH_ARGS_' | cut -d= -f1); do BENCH_ARGS[${v#BENCH_ARGS_}]="${!v}"; done
OUT=gpurun_out/ab.log
: > $OUT
R=$1; shift
for r in $(seq $R); do
  for v in "$@"; do
    tag=${v%%:*}; envs=${v#*:}
    env ${envs//,/ } timeout -k 10 120 python -u bench.py --steps 400 --warmup 40 --cpu-seconds 0 --profile-steps ${AB_PROFILE_STEPS:-0} \
      --no-explored --no-host-inputs ${BENCH_ARGS[$tag]} > gpurun_out/ab_tmp.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/ab_tmp.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_tmp.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e9,1), 'e9', round(d['ms_per_step']*1e3,1), 'us/step', 'p50', round(d['step_wall_us']['p50'],1), {k: round(v*1e3,1) for k, v in (d.get('kernel_avg_ms') or {}).items()})" | tee -a $OUT
  done
done
