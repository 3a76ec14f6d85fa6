#!/usr/bin/env bash
# A/B of environment switches on the GPU box, alternating, twice:
#   tools/ab_env.sh "<bench args>" "HIPBP_PROVE_SORT=0" "HIPBP_PROVE_SORT=1"
set -e
mkdir -p gpurun_out/ab
ARGS=$1; shift
for rep in 1 2; do
i=0
for cfg in "$@"; do
env $cfg timeout -k 10 200 python bench.py $ARGS > gpurun_out/ab/env${i}_r$rep.json 2>/dev/null
i=$((i+1))
done
done
echo ok
