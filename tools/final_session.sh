set -o pipefail
bash tools/gpu_session.sh tests pmc || exit 1
python tools/pmc_summary.py gpurun_out/pmc profiles/pmc_latest.json > gpurun_out/pmc_summary.log 2>&1 || exit 1
cp profiles/pmc_latest.json gpurun_out/pmc_latest.json
bash tools/gpu_session.sh bench shard prof || exit 1
for c in C1 C2 C4 C5; do timeout -k 10 300 python -u bench.py --config $c --cpu-seconds 10 > gpurun_out/bench_$c.log 2>&1 || exit 1; echo "$c ok"; done
