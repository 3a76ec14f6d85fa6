#!/usr/bin/env bash
# A/B of the drop-in first call between two prebuilt libraries ab/lib_old.so and ab/lib_new.so (GPU box):
# tests/dropin_latency.c, alternating, 4 runs each, n = $N (default 16) -> gpurun_out/ab_first/runs.jsonl
set -euo pipefail
mkdir -p gpurun_out/ab_first
python3 -c "import bench; bench.build_dropin_latency(); bench.dropin_proof_file('gpurun_out/ab_first/proof${N:-16}.bin', ${N:-16})"
LIB=cudabulletproof_amd/libcudabulletproof_hip.so
cp $LIB gpurun_out/ab_first/lib_orig.so
for i in 1 2 3 4; do
  for v in old new; do
    cp ab/lib_$v.so $LIB
    r=$(timeout -k 10 60 ./build/dropin_latency gpurun_out/ab_first/proof${N:-16}.bin ${WARM:-5})
    echo "{\"v\": \"$v\", \"n\": ${N:-16}, \"r\": $r}" >> gpurun_out/ab_first/runs.jsonl
  done
done
cp gpurun_out/ab_first/lib_orig.so $LIB
