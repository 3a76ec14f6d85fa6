#!/usr/bin/env bash
# configs[4] rank shard: unequal pipeline shares and a high-priority second pipeline
set -o pipefail
TAG=${1:-r03zb}
mkdir -p gpurun_out
REPS=5 timeout -k 10 300 python tools/shard_probe.py 8192 4096,4352+3840,4608+3584 16384:32768 > gpurun_out/shard_probe_$TAG.txt 2>&1 || { tail -20 gpurun_out/shard_probe_$TAG.txt; exit 1; }
PRIO=1 REPS=5 timeout -k 10 300 python tools/shard_probe.py 8192 4096,4352+3840 16384:32768 >> gpurun_out/shard_probe_$TAG.txt 2>&1 || { tail -20 gpurun_out/shard_probe_$TAG.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/shard_probe_$TAG.txt
