#!/usr/bin/env bash
# multirank rehearsal + configs[4] 8192 shard leg (median of 5 passes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "multirank or rccl" \
    > gpurun_out/pytest_r03zj.log 2>&1 || { tail -60 gpurun_out/pytest_r03zj.log; exit 1; }
tail -2 gpurun_out/pytest_r03zj.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-ipa --no-prove --no-msm --no-host --no-check --no-h2d --no-repeats \
    --shard-total 8192 > gpurun_out/shard8k_r03zj.json 2> gpurun_out/shard8k_r03zj.err || { tail -30 gpurun_out/shard8k_r03zj.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/shard8k_r03zj.json')); s=d['sharded_2p16']; print('shard 8192:', round(s['value']), round(s['value_min']), round(s['value_max']), s['passes_timed'], round(s['ms'],2), s['verdicts_sha256'])"
