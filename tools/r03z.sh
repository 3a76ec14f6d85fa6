#!/usr/bin/env bash
# quad-step A/B: quad parity tests, then the configs[4] rank shard (8192) schedules
set -o pipefail
TAG=${1:-r03z}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "quad or pipeline or oneshot or cuda_range" \
    > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
REPS=3 timeout -k 10 300 python tools/shard_probe.py 8192 4096 16384:32768 > gpurun_out/shard_probe_$TAG.txt 2>&1 || { tail -20 gpurun_out/shard_probe_$TAG.txt; exit 1; }
NP=3 REPS=3 timeout -k 10 300 python tools/shard_probe.py 8192 2731+2731+2730 16384:32768 >> gpurun_out/shard_probe_$TAG.txt 2>&1 || { tail -20 gpurun_out/shard_probe_$TAG.txt; exit 1; }
NP=4 REPS=3 timeout -k 10 300 python tools/shard_probe.py 8192 2048 16384:32768 >> gpurun_out/shard_probe_$TAG.txt 2>&1 || { tail -20 gpurun_out/shard_probe_$TAG.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/shard_probe_$TAG.txt
