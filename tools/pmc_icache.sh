#!/usr/bin/env bash
# Instruction-fetch counters of the verify tick (k_terms): I-cache hits/misses and wave cycles
# waiting for instructions.  tools/pmc_icache.sh <tag> [extra bench args]
set -euo pipefail
TAG=${1:-ic}; shift || true
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BENCH="python3 bench.py --steps 6 --warmup 2 --no-cpu --no-ipa --no-prove --no-msm $*"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --kernel-trace --output-format csv -d "$OUT/ic" -o run -- $BENCH > "$OUT/ic.json" 2> "$OUT/ic.err"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d "$OUT/wait" -o run -- $BENCH > "$OUT/wait.json" 2> "$OUT/wait.err"
