#!/usr/bin/env bash
set -o pipefail
TAG=${1:-r03g}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python tools/prove_pipe_probe.py 65536 2 4 22 > gpurun_out/prove_pipe_$TAG.txt 2>&1 || { cat gpurun_out/prove_pipe_$TAG.txt; exit 1; }
cat gpurun_out/prove_pipe_$TAG.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prove_trace_$TAG -o run -- python3 tools/prove_pipe_probe.py 65536 2 4 22 > /dev/null 2>&1 || exit 1
echo traced
