#!/usr/bin/env bash
# rocprofv3 kernel trace of the Pippenger MSM alone (tools/pip_probe.py: 2^20 config-3 points,
# window 12, 12 MSMs over 2 streams) -> gpurun_out/prof_<tag>_pip/
set -euo pipefail
TAG=${1:-r02}
OUT=gpurun_out/prof_${TAG}_pip
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 tools/pip_probe.py 20 12 12 2 > "$OUT/probe.txt" 2> "$OUT/trace.err"
ls -R "$OUT" > "$OUT/listing.txt"
