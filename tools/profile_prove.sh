#!/usr/bin/env bash
# Profile the GPU prover (hipbp_batch_generate_range_proof) with rocprofv3 on the GPU box, at the
# bench's prove-leg configuration (B = 65536 64-bit proofs per batch, the bench's default K prefix tables, four
# streams; a 2-step verify leg runs first and its kernels are told apart by name).
#   tools/profile_prove.sh <tag>  -> gpurun_out/prof_<tag>_prove/{trace,pmc_busy,pmc_valu,pmc_fetch,pmc_write}/...
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}_prove
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RUN="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-ipa --no-msm --no-shard --no-host --no-check --no-h2d --no-repeats --table-legs= --prove-steps 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $RUN > "$OUT/bench_trace.json" 2> "$OUT/trace.log"
timeout -k 10 300 rocprofv3 --pmc VALUBusy VALUUtilization --kernel-trace --output-format csv -d "$OUT/pmc_busy" -o run -- $RUN > /dev/null 2> "$OUT/busy.log"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_valu" -o run -- $RUN > /dev/null 2> "$OUT/valu.log"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- $RUN > /dev/null 2> "$OUT/fetch.log"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- $RUN > /dev/null 2> "$OUT/write.log"
