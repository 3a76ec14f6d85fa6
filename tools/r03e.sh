#!/usr/bin/env bash
# GPU tests + Pippenger probe (2^20, window 12: one stream, then two streams in flight, then batches of 4)
set -o pipefail
TAG=${1:-r03e}
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 200 python tools/pip_probe.py 20 12 12 2 4 > gpurun_out/pip_probe_$TAG.txt 2>&1 || { cat gpurun_out/pip_probe_$TAG.txt; exit 1; }
cat gpurun_out/pip_probe_$TAG.txt
