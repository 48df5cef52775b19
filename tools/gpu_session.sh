#!/bin/bash
# One GPU-box session, steps run in order, stopping at the first step that
# crashes, aborts or times out (each step under its own time limit).
# Usage: bash tools/gpu_session.sh STEP...   (from the repo root)
#   tests         pytest -m gpu
#   tests:EXPR    pytest -m gpu -k EXPR
#   bench         python bench.py (the driver's command, with CPU baseline)
#   shard         2-rank sharded bench rehearsal (gloo, both ranks on GPU 0)
#   prof          rocprofv3 --kernel-trace --stats over a bench run
#   probe         rocprofv3 --kernel-trace --stats over tools/frontier_probe.py (explored map)
#   pmc           PMC passes over a short C3 bench -> profiles/pmc_latest.json [C3]
#   pmcx          PMC passes over the explored-map probe -> [C3-explored]
#   cfg:CN        bench.py --config CN
#   abfm          C3 A/B of fmask maintenance (tools/ab.sh -> ab.log)
#   timeline      per-workgroup accumulation timeline (tools/accum_timeline.py)
#   phase / phase5:N   phase build probe at C3 / C5 with N beams per scan
#   c5:SWEEP      bench.py --config C5 --sweep SWEEP
set -o pipefail
R=$PWD
OUT=$R/gpurun_out
mkdir -p $OUT
ok() { [ "$1" -eq 0 ]; }
for s in "$@"; do
  case $s in
    tests|tests:*)
      k=(); [ "$s" != tests ] && k=(-k "${s#tests:}")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v "${k[@]}" --timeout 400 --timeout-method thread \
        > $OUT/pytest_gpu.log 2>&1
      rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_gpu.log | tail -8
      ok $rc || exit $rc ;;
    bench)
      timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-600; ok $rc || exit $rc ;;
    rehearse:*)
      # N ranks of the multi-GPU bench on this one GPU (gloo, host-staged
      # exchange): the N > 1 line's fields, not xGMI timings
      n=${s#rehearse:}
      timeout -k 10 500 python -u bench.py --gpus $n --backend gloo --device-override 0 --steps 20 --warmup 5 \
        --cpu-seconds 0 --pool 3 --no-host-inputs > $OUT/rehearse_$n.log 2>&1
      rc=$?; echo "rehearse $n rc=$rc"; tail -1 $OUT/rehearse_$n.log | cut -c1-300; ok $rc || exit $rc ;;
    shard)
      timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --device-override 0 \
        --cpu-seconds 0 --pool 3 > $OUT/shard.log 2>&1
      rc=$?; echo "shard rc=$rc"; tail -1 $OUT/shard.log | cut -c1-300; ok $rc || exit $rc ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run \
        --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $OUT/prof.log 2>&1)
      rc=$?; echo "prof rc=$rc"; ok $rc || exit $rc ;;
    probe)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/probe -o run \
        --output-format csv -- python3 $R/tools/frontier_probe.py > $OUT/probe.log 2>&1)
      rc=$?; echo "probe rc=$rc"; tail -1 $OUT/probe.log | cut -c1-400; ok $rc || exit $rc ;;
    pmc)
      bash $R/tools/pmc_passes.sh gpurun_out/pmc; rc=$?; ok $rc || exit $rc
      python $R/tools/pmc_summary.py $OUT/pmc $R/profiles/pmc_latest.json C3 > $OUT/pmc_summary.log 2>&1 || exit 1
      cp $R/profiles/pmc_latest.json $OUT/pmc_latest.json ;;
    pmcx)
      bash $R/tools/pmc_passes.sh gpurun_out/pmcx python3 $R/tools/frontier_probe.py --passes 5; rc=$?; ok $rc || exit $rc
      python $R/tools/pmc_summary.py $OUT/pmcx $R/profiles/pmc_latest.json C3-explored > $OUT/pmcx_summary.log 2>&1 || exit 1
      cp $R/profiles/pmc_latest.json $OUT/pmc_latest.json ;;
    pmc5)
      # PMC passes per C5 sweep point -> profiles/pmc_latest.json [C5-N]
      for n in 12 48 192 768 4096; do
        bash $R/tools/pmc_passes.sh gpurun_out/pmc5_$n python3 $R/bench.py --config C5 --sweep $n --steps 5 \
          --warmup 2 --pool 2 --cpu-seconds 0 --no-overlap || exit 1
        python $R/tools/pmc_summary.py $OUT/pmc5_$n $R/profiles/pmc_latest.json C5-$n >> $OUT/pmc5_summary.log 2>&1 || exit 1
      done
      cp $R/profiles/pmc_latest.json $OUT/pmc_latest.json ;;
    abfm)
      # C3 A/B: fmask maintained or not (2 alternating rounds)
      timeout -k 10 600 bash $R/tools/ab.sh 2 "base:" "fmask:DM_FMASK=on"
      rc=$?; echo "abfm rc=$rc"; ok $rc || exit $rc ;;
    timeline)
      timeout -k 10 300 python -u $R/tools/accum_timeline.py 30 --json $OUT/accum_timeline.json \
        > $OUT/accum_timeline.log 2>&1
      rc=$?; echo "timeline rc=$rc"; ok $rc || exit $rc ;;
    phase5:*)
      timeout -k 10 300 python -u $R/tools/phase_probe.py c5 ${s#phase5:} > $OUT/phase_c5_${s#phase5:}.log 2>&1
      rc=$?; echo "phase5 rc=$rc"; ok $rc || exit $rc ;;
    phase)
      timeout -k 10 300 python -u $R/tools/phase_probe.py > $OUT/phase_c3.log 2>&1
      rc=$?; echo "phase rc=$rc"; ok $rc || exit $rc ;;
    c5:*)
      timeout -k 10 600 python -u bench.py --config C5 --sweep ${s#c5:} --cpu-seconds 0 > $OUT/bench_c5.log 2>&1
      rc=$?; echo "c5 rc=$rc"; tail -1 $OUT/bench_c5.log | cut -c1-300; ok $rc || exit $rc ;;
    driver)
      # the driver's exact command three times (step traces), a 200-step run,
      # and a kernel trace of the driver's command (per-step kernels after reset)
      for i in 1 2 3; do
        timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --step-trace $OUT/drv_trace_$i.json \
          > $OUT/drv_$i.log 2>&1
        rc=$?; echo "driver run $i rc=$rc"; ok $rc || exit $rc
      done
      timeout -k 10 400 python -u bench.py --gpus 1 --steps 200 --warmup 5 --cpu-seconds 0 \
        --step-trace $OUT/drv_trace_200.json > $OUT/drv_200.log 2>&1
      rc=$?; echo "200-step rc=$rc"; ok $rc || exit $rc
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/drvprof -o run \
        --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 \
        --no-explored --no-host-inputs > $OUT/drvprof.log 2>&1)
      rc=$?; echo "drvprof rc=$rc"; ok $rc || exit $rc ;;
    cfg:*)
      c=${s#cfg:}
      timeout -k 10 400 python -u bench.py --config $c --cpu-seconds 10 > $OUT/bench_$c.log 2>&1
      rc=$?; echo "$c rc=$rc"; tail -1 $OUT/bench_$c.log | cut -c1-300; ok $rc || exit $rc ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
