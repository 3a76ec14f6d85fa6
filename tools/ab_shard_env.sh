#!/usr/bin/env bash
# A/B of environment settings on the configs[4] 8192-proof shard (bench.py's leg, median of 5 each run).
#   ENVS="HIPBP_ROW_MAX_ITEMS=2048 HIPBP_ROW_MAX_ITEMS=8192" bash tools/ab_shard_env.sh
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for kv in $ENVS; do
  env $kv timeout -k 10 300 python -u bench.py --no-cpu --no-ipa --no-msm --no-host --no-prove --no-h2d \
      --no-repeats --no-check --steps 2 --shard-total 8192 > gpurun_out/abse.json 2> gpurun_out/abse.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abse.json'))['sharded_2p16'];print('$kv',round(d['value']),round(d['value_min']),round(d['value_max']),d['verdicts_sha256'])"
done; done
