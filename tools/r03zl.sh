#!/usr/bin/env bash
# configs[4] 8192 shard leg: the headline's streams vs fresh streams, alternated (the
# BENCH_SHARD_STREAMS toggle it used was removed after the A/B: profiles/shard/shard8k_streams_r03zl.txt)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for m in reuse fresh; do
  BENCH_SHARD_STREAMS=$m timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-ipa --no-prove --no-msm --no-host --no-check --no-h2d --no-repeats \
    --shard-total 8192 > gpurun_out/shard8k_r03zl_${m}_$rep.json 2> gpurun_out/shard8k_r03zl_${m}_$rep.err || { tail -30 gpurun_out/shard8k_r03zl_${m}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/shard8k_r03zl_${m}_$rep.json')); s=d['sharded_2p16']; print('$m', $rep, round(s['value']), round(s['value_min']), round(s['value_max']))"
done; done
