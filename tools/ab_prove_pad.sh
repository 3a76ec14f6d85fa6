#!/usr/bin/env bash
# prover A/B: terms0 capped at 3 blocks per CU by a dynamic LDS pad (HIPBP_PROVE_T0_PAD) so the other
# stream's chain / rterms / commit kernels find a wave slot beside it, with and without the terms0
# gate across streams (HIPBP_PROVE_GATE), vs the default (4 blocks, no gate)
set -o pipefail
TAG=${1:-r03s}
mkdir -p gpurun_out
for cfg in "0 0" "1 0" "1 10240" "1 9216" "1 12288" "0 0"; do
  set -- $cfg
  HIPBP_PROVE_GATE=$1 HIPBP_PROVE_T0_PAD=$2 timeout -k 10 200 python tools/prove_pipe_probe.py 65536 2 6 22 > gpurun_out/prove_pad_${TAG}_$1_$2.txt 2>&1 || { cat gpurun_out/prove_pad_${TAG}_$1_$2.txt; exit 1; }
  echo "gate $1 pad $2: $(tail -n 1 gpurun_out/prove_pad_${TAG}_$1_$2.txt)"
done
