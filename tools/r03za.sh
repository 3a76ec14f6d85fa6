#!/usr/bin/env bash
# kernel trace of the configs[4] rank shard at HEAD + its timeline
set -o pipefail
TAG=${1:-r03za}
bash tools/shard_trace.sh $TAG || exit 1
python tools/shard_timeline.py $TAG > gpurun_out/shard_timeline_$TAG.txt 2>&1 || exit 1
cat gpurun_out/shard_timeline_$TAG.txt
