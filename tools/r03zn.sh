#!/usr/bin/env bash
# same box: the shard probe, then bench.py's configs[4] leg at 8192, then the probe again
set -o pipefail
mkdir -p gpurun_out
REPS=5 timeout -k 10 300 python tools/shard_probe.py 8192 4096 16384:32768 > gpurun_out/shard_probe_r03zn_a.txt 2>&1 || exit 1
grep "push" gpurun_out/shard_probe_r03zn_a.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-ipa --no-prove --no-msm --no-host --no-check --no-h2d --no-repeats \
    --shard-total 8192 > gpurun_out/shard8k_r03zn.json 2> gpurun_out/shard8k_r03zn.err || { tail -30 gpurun_out/shard8k_r03zn.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/shard8k_r03zn.json')); s=d['sharded_2p16']; print('bench leg:', round(s['value']), round(s['value_min']), round(s['value_max']))"
REPS=5 timeout -k 10 300 python tools/shard_probe.py 8192 4096 16384:32768 > gpurun_out/shard_probe_r03zn_b.txt 2>&1 || exit 1
grep "push" gpurun_out/shard_probe_r03zn_b.txt
