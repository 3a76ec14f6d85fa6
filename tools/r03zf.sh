#!/usr/bin/env bash
# H2D leg (one copy per step, issued two steps ahead) x3
set -o pipefail
mkdir -p gpurun_out
for A in 2 4 6; do rep=$A; export BENCH_H2D_AHEAD=$A;
  timeout -k 10 200 python bench.py --no-cpu --no-prove --no-ipa --no-msm --no-host --no-shard --no-check --no-repeats --steps 50 \
      > gpurun_out/h2d_r03zf_$rep.json 2> gpurun_out/h2d_r03zf_$rep.err || { tail -20 gpurun_out/h2d_r03zf_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/h2d_r03zf_$rep.json')); print($rep, round(d['value']), round(d['with_h2d']['value']), d['with_h2d'].get('copy_ahead_steps'))"
done
