#!/usr/bin/env bash
set -o pipefail
TAG=${1:-r03h}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "prove or prover" --timeout 180 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for cfg in "1 2" "0 2" "1 3" "1 2"; do
  set -- $cfg
  HIPBP_PROVE_GATE=$1 timeout -k 10 200 python tools/prove_pipe_probe.py 65536 $2 6 22 > gpurun_out/prove_pipe_${TAG}_$1_$2.txt 2>&1 || { cat gpurun_out/prove_pipe_${TAG}_$1_$2.txt; exit 1; }
  echo "gate $1: $(tail -1 gpurun_out/prove_pipe_${TAG}_$1_$2.txt)"
done
