#!/usr/bin/env bash
# A/B: prove leg (B = 65536, 8 batches) with terms0 serialised across streams (HIPBP_PROVE_GATE=1) at
# 2..4 caller streams: each stream's latency-bound tail then has the other streams' terms0 to run under.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for cfg in ${CONFIGS:-2:0 3:1 4:1 3:0 4:0}; do
  IFS=: read ns gate <<< "$cfg"
  HIPBP_PROVE_GATE=$gate timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-ipa --no-msm --no-shard \
      --no-host --no-check --no-h2d --no-repeats --prove-steps ${STEPS:-8} --prove-streams $ns > gpurun_out/abpg.json \
      2> gpurun_out/abpg.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abpg.json'))['prove'];print('streams:gate $cfg',round(d['value']),round(d['ms_per_batch'],2),d['deterministic_across_streams'])"
done; done
