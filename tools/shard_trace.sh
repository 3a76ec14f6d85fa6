#!/usr/bin/env bash
# Kernel trace of the configs[4] rank shard (8192 proofs, one 4096 push per pipeline): the
# timeline of its ticks per stream, for the drain analysis (tools/shard_timeline.py).
set -euo pipefail
TAG=${1:-r03n}
OUT=gpurun_out/shard_trace_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
REPS=1 RR=${RR:-0} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- \
    python3 tools/shard_probe.py 8192 ${PUSHES:-4096} ${QMAX:-16384:32768} > "$OUT/probe.txt" 2> "$OUT/probe.err"
cat "$OUT/probe.txt"
