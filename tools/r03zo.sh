#!/usr/bin/env bash
# sustained headline at HEAD: 2000 timed ticks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 2000 --warmup 5 --no-cpu --no-ipa --no-prove --no-msm --no-host --no-shard --no-h2d --no-repeats \
    > gpurun_out/bench_r03zo_sustained_2000ticks.json 2> gpurun_out/bench_r03zo.err || { tail -30 gpurun_out/bench_r03zo.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r03zo_sustained_2000ticks.json')); print(round(d['value']), round(d['ms_per_step'],3), d['verify_check']['matches_oracle_sample'])"
