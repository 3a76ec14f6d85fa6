#!/usr/bin/env bash
# Profile the batched verify with rocprofv3 on the GPU box (run from the repo root via gpurun).
#   tools/profile.sh <tag>    -> gpurun_out/prof_<tag>/{trace,pmc_fetch,pmc_write,pmc_valu}/...
# Kernel trace + stats in one run; PMC counters in their own runs (FETCH_SIZE and WRITE_SIZE
# do not fit one TCC pass on gfx950: MI355X_MICROARCH.md, rocprofv3 PMC slots).
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# the headline configuration (B = 1024, n = 64, the default K, two pipelines) and the default bench's
# own step and warm-up counts, so the trace's k_terms launches are the ones a default bench line times
# (the other legs off; the MSM leg at ${MSM_LOG2:-20} for its kernels' counters)
BENCH="python3 bench.py --no-cpu --no-ipa --no-prove --no-shard --no-host --no-check --no-h2d --no-repeats --table-legs= --msm-log2 ${MSM_LOG2:-20}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $BENCH > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- $BENCH > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- $BENCH > "$OUT/bench_write.json" 2> "$OUT/write.err"
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace --output-format csv -d "$OUT/pmc_valu" -o run -- $BENCH > "$OUT/bench_valu.json" 2> "$OUT/valu.err"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_cyc" -o run -- $BENCH > "$OUT/bench_cyc.json" 2> "$OUT/cyc.err"
timeout -k 10 400 rocprofv3 --pmc VALUBusy VALUUtilization --kernel-trace --output-format csv -d "$OUT/pmc_busy" -o run -- $BENCH > "$OUT/bench_busy.json" 2> "$OUT/busy.err"
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU2 --kernel-trace --output-format csv -d "$OUT/pmc_mix" -o run -- $BENCH > "$OUT/bench_mix.json" 2> "$OUT/mix.err"
ls -R "$OUT" > "$OUT/listing.txt"
