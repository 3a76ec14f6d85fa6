#!/usr/bin/env bash
# GPU round trip (round 3): GPU test suite, the VALU issue-cost ubench, one full bench line.
#   tools/round3_check.sh <tag>   -> gpurun_out/{pytest,ubench_issue,bench}_<tag>.*
set -o pipefail
TAG=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
if [ "${SKIP_UBENCH:-0}" != 1 ]; then
  timeout -k 10 120 tools/ubench_issue > gpurun_out/ubench_issue_$TAG.json 2> gpurun_out/ubench_issue_$TAG.err || exit 1
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(round(d['value']), d['verify_check'], (d.get('with_h2d') or {}).get('value'))"
if [ "${SHARD_AB:-0}" = 1 ]; then   # configs[4] at N = 8: one rank's 8192-proof shard on one GPU
  for Q in 0 auto; do
    if [ $Q = auto ]; then unset HIPBP_QUAD; else export HIPBP_QUAD=$Q; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-ipa --no-prove --no-msm --no-host --no-check \
        --no-h2d --shard-total 8192 > gpurun_out/shard8k_${TAG}_q$Q.json 2> gpurun_out/shard8k_${TAG}_q$Q.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/shard8k_${TAG}_q$Q.json')); s=d['sharded_2p16']; print('quad=$Q', round(s['value']), round(s['ms'],2), s['verdicts_sha256'], round(d['value']))"
  done
  unset HIPBP_QUAD
fi
