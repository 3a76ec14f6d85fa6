#!/usr/bin/env bash
# round-3 final: full GPU suite, smoke, default bench line, configs[4] 8192 shard, headline profile
set -o pipefail
TAG=${1:-r03ze}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(round(d['value']), round(d['repeats']['median']), round(d['sharded_2p16']['value']), d['verify_check']['matches_oracle_sample'], round(d['msm']['value']/1e6,1), round(d['msm']['pippenger']['value']/1e6), round(d['ipa']['value']), round(d['prove']['value']))"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-ipa --no-prove --no-msm --no-host --no-check --no-h2d --no-repeats \
    --shard-total 8192 > gpurun_out/shard8k_$TAG.json 2> gpurun_out/shard8k_$TAG.err || { tail -30 gpurun_out/shard8k_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/shard8k_$TAG.json')); s=d['sharded_2p16']; print('shard 8192:', round(s['value']), round(s['value_min']), round(s['value_max']), round(s['ms'],2), s['verdicts_sha256'])"

