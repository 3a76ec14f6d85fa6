#!/usr/bin/env bash
# Where the drop-in's first cuda_range_proof_verify call spends its time (run on the GPU box via
# gpurun): tests/dropin_latency.c on reference proof 0 of proofs_n16.npz, plain (its JSON line) and
# under rocprofv3 --hip-trace --kernel-trace (the HIP API calls and kernels of the first call).
#   bash tools/dropin_probe.sh <tag>  -> gpurun_out/dropin_<tag>/
set -euo pipefail
TAG=${1:-probe}
OUT=gpurun_out/dropin_$TAG
mkdir -p "$OUT"
python3 -c "import bench; bench.build_dropin_latency(); bench.dropin_proof_file('$OUT/proof16.bin', 16)"
for i in 1 2 3; do timeout -k 10 60 ./build/dropin_latency "$OUT/proof16.bin" 5 >> "$OUT/plain.jsonl"; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace" -o run -- ./build/dropin_latency "$OUT/proof16.bin" 3 > "$OUT/traced.jsonl" 2> "$OUT/trace.err"
