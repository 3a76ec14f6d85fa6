#!/usr/bin/env bash
# split stage-2 product in the quad step + host-shard hook: parity tests, shard probe, shard bench leg
set -o pipefail
TAG=${1:-r03zd}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "quad or pipeline or oneshot or cuda_range or host_structs or pippenger or horner" \
    > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
REPS=5 timeout -k 10 300 python tools/shard_probe.py 8192 4096 16384:32768 > gpurun_out/shard_probe_$TAG.txt 2>&1 || { tail -20 gpurun_out/shard_probe_$TAG.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/shard_probe_$TAG.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-ipa --no-prove --no-msm --no-host --no-check --no-h2d --no-repeats \
    --shard-total 8192 > gpurun_out/shard8k_$TAG.json 2> gpurun_out/shard8k_$TAG.err || { tail -30 gpurun_out/shard8k_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/shard8k_$TAG.json')); s=d['sharded_2p16']; print('shard 8192:', round(s['value']), round(s['value_min']), round(s['value_max']), round(s['ms'],2), s['verdicts_sha256'])"
timeout -k 10 120 python tools/oneshot_probe.py > gpurun_out/oneshot_$TAG.txt 2>&1 || { tail -20 gpurun_out/oneshot_$TAG.txt; exit 1; }
tail -5 gpurun_out/oneshot_$TAG.txt
