#!/usr/bin/env bash
# mutation check of the fused add/sub block: a library built with sub's test 1 dropped from its
# rare-edge OR (ab/lib_mut1.so, made from a patched tools/gen_field_asm.py) must FAIL the edge test
set -o pipefail
mkdir -p gpurun_out
cp ab/lib_mut1.so cudabulletproof_amd/libcudabulletproof_hip.so
timeout -k 10 200 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -k "one_edge_lane_per_wave and addsub" \
    > gpurun_out/pytest_mut1.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_mut1.log | tail -4
[ $rc -ne 0 ] && echo "mutation caught (pytest rc=$rc)" || { echo "mutation NOT caught"; exit 1; }
