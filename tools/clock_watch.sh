#!/usr/bin/env bash
# Shader clock and socket power while the headline runs (GPU box, via gpurun): bench.py's headline
# alone for a long region, rocm-smi sampled every 0.5 s (read-only queries) into
# gpurun_out/clock_<tag>/smi.jsonl; the bench line into bench.json.
#   bash tools/clock_watch.sh <tag> [steps]
set -euo pipefail
TAG=${1:-cw}
STEPS=${2:-2000}
OUT=gpurun_out/clock_$TAG
mkdir -p "$OUT"
timeout -k 10 400 python3 bench.py --steps "$STEPS" --warmup 5 --no-cpu --no-ipa --no-msm --no-prove --no-shard \
    --no-host --no-h2d --no-check --table-legs= > "$OUT/bench.json" 2> "$OUT/bench.err" &
BPID=$!
while kill -0 "$BPID" 2> /dev/null; do
    { printf '{"t": %s, "smi": ' "$(date +%s.%N)"; timeout 10 rocm-smi -c -P --json 2> /dev/null | tr -d '\n' || printf 'null'; printf '}\n'; } >> "$OUT/smi.jsonl"
    sleep 0.5
done
wait "$BPID"
