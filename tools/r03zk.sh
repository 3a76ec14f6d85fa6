#!/usr/bin/env bash
# drain bounds re-checked after the operand-form quad / pair steps (quad:pair max items)
set -o pipefail
mkdir -p gpurun_out
REPS=5 timeout -k 10 400 python tools/shard_probe.py 8192 4096 16384:32768,16384:65536,32768:65536,8192:32768 > gpurun_out/shard_probe_r03zk.txt 2>&1 || { tail -20 gpurun_out/shard_probe_r03zk.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/shard_probe_r03zk.txt
