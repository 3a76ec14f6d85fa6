#!/usr/bin/env bash
# round-3 HEAD check: full GPU suite, default bench line, configs[4] at N = 8 per rank (8192-proof shard)
set -o pipefail
TAG=${1:-r03zc}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(round(d['value']), d['repeats']['median'], d['sharded_2p16']['value'], d['verify_check']['matches_oracle_sample'])"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-ipa --no-prove --no-msm --no-host --no-check --no-h2d --no-repeats \
    --shard-total 8192 > gpurun_out/shard8k_$TAG.json 2> gpurun_out/shard8k_$TAG.err || { tail -30 gpurun_out/shard8k_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/shard8k_$TAG.json')); s=d['sharded_2p16']; print('shard 8192:', round(s['value']), round(s['ms'],2), s['verdicts_sha256'], s.get('passes_ms'))"
