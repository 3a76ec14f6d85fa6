#!/usr/bin/env bash
# quick GPU check after a kernel change: the GPU tests, then the shard probe
set -o pipefail
TAG=${1:-r03c}
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
REPS=2 timeout -k 10 300 python tools/shard_probe.py 8192 ${PUSHES:-1024,2048,4096} ${QMAX:-0,49152,131072,262144} > gpurun_out/shard_probe_$TAG.txt 2>&1 || { cat gpurun_out/shard_probe_$TAG.txt; exit 1; }
cat gpurun_out/shard_probe_$TAG.txt
