#!/usr/bin/env bash
# Profile the GPU prover (hipbp_batch_generate_range_proof) with rocprofv3 on the GPU box.
#   tools/profile_prove.sh <tag>  -> gpurun_out/prof_<tag>_prove/{trace,pmc_busy,pmc_valu}/...
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}_prove
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RUN="python3 tools/prove_probe.py 16384 random"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $RUN > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc VALUBusy VALUUtilization --kernel-trace --output-format csv -d "$OUT/pmc_busy" -o run -- $RUN > "$OUT/busy.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_valu" -o run -- $RUN > "$OUT/valu.log" 2>&1
