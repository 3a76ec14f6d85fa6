#!/usr/bin/env bash
# prover A/B: terms0 capped at 3 blocks per CU by a dynamic LDS pad (HIPBP_PROVE_T0_PAD) so the other
# stream's chain / rterms / commit kernels find a wave slot beside it, vs the default (4 blocks, no room)
set -o pipefail
TAG=${1:-r03r}
mkdir -p gpurun_out
for pad in 0 9216 10240 0; do
  HIPBP_PROVE_T0_PAD=$pad timeout -k 10 200 python tools/prove_pipe_probe.py 65536 2 6 22 > gpurun_out/prove_pad_${TAG}_$pad.txt 2>&1 || { cat gpurun_out/prove_pad_${TAG}_$pad.txt; exit 1; }
  echo "pad $pad: $(tail -1 gpurun_out/prove_pad_${TAG}_$pad.txt)"
done
