#!/usr/bin/env bash
# fused add/sub block on the rare edges (field ops 8 / 9) + the field / drain-form tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "field or quad or sq_matches" \
    > gpurun_out/pytest_r03zh.log 2>&1 || { tail -60 gpurun_out/pytest_r03zh.log; exit 1; }
grep -E "addsub|passed|failed" gpurun_out/pytest_r03zh.log | tail -6
