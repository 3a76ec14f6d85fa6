#!/usr/bin/env bash
# Kernel trace of bench.py's configs[4] leg at one rank's 8192-proof shard (the default schedule:
# split stage 0, two pushes of 4096); tools/shard_timeline.py <tag> prints its last pass.
set -euo pipefail
TAG=${1:-r04}
OUT=gpurun_out/shard_trace_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- python3 bench.py --no-cpu --no-ipa \
    --no-msm --no-host --no-prove --no-h2d --no-repeats --no-check --steps 2 --shard-total 8192 > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 tools/shard_timeline.py "$TAG" > "$OUT/timeline.txt"
