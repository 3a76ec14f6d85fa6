#!/usr/bin/env bash
# GPU round trip used while iterating: full GPU test suite, then bench A/B lines (+ optional PMC pass).
#   tools/gpu_check.sh <tag> [prefix bits ...]
set -o pipefail
TAG=${1:-chk}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
for K in "$@"; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu --no-ipa --no-prove --no-msm --prefix-bits $K > gpurun_out/ab_${TAG}_$K.json 2> gpurun_out/ab_${TAG}_$K.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_$K.json')); print($K, round(d['value']), round(d['roofline']['avg_launch_ms'],3))"
done
