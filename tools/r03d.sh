#!/usr/bin/env bash
# sort-stream A/B: shard probe schedules with the lane sort on its own stream (default) and not, then the
# headline bench both ways (verify leg only)
set -o pipefail
TAG=${1:-r03d}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
for SS in 1 0; do
  HIPBP_SORT_STREAM=$SS REPS=2 timeout -k 10 300 python tools/shard_probe.py 8192 ${PUSHES:-4096,2048} ${QMAX:-49152} > gpurun_out/shard_probe_${TAG}_ss$SS.txt 2>&1 || { cat gpurun_out/shard_probe_${TAG}_ss$SS.txt; exit 1; }
  echo "sort stream $SS"; grep push gpurun_out/shard_probe_${TAG}_ss$SS.txt
done
for SS in 1 0 1 0; do
  HIPBP_SORT_STREAM=$SS timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --no-ipa --no-prove --no-msm --no-host --no-check --no-h2d --no-shard > gpurun_out/bench_${TAG}_ss$SS.json 2> gpurun_out/bench_${TAG}_ss$SS.err || { tail -20 gpurun_out/bench_${TAG}_ss$SS.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_ss$SS.json')); print('bench sort stream $SS', round(d['value']))"
done
