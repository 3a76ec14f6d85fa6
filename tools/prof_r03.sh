#!/usr/bin/env bash
# Round-3 profiling call: the headline configuration's PMC passes (tools/profile.sh), the
# Pippenger's (tools/profile_pip.sh), and the VALU roof of k_terms' own instruction mix
# (tools/ubench_step with a rocprofv3 SQ_INSTS_VALU pass).
set -o pipefail
TAG=${1:-r03b}
mkdir -p gpurun_out
tools/profile.sh $TAG || exit 1
echo "profile.sh done"
tools/profile_pip.sh $TAG || exit 1
echo "profile_pip.sh done"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 tools/ubench_step > gpurun_out/ubench_step_$TAG.json 2> gpurun_out/ubench_step_$TAG.err || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/ubench_step_pmc_$TAG -o run -- tools/ubench_step > /dev/null 2> gpurun_out/ubench_step_pmc_$TAG.err || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/ubench_issue_pmc_$TAG -o run -- tools/ubench_issue > /dev/null 2> gpurun_out/ubench_issue_pmc_$TAG.err || exit 1
cat gpurun_out/ubench_step_$TAG.json
REPS=2 timeout -k 10 300 python tools/shard_probe.py 8192 4096,8192 16384,32768,49152,65536,98304 > gpurun_out/shard_probe_$TAG.txt 2>&1 || exit 1
cat gpurun_out/shard_probe_$TAG.txt
REPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/shard_trace_$TAG -o run -- python3 tools/shard_probe.py 8192 4096 49152 > /dev/null 2>&1 || exit 1
