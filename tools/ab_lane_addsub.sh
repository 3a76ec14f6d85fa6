#!/usr/bin/env bash
# A/B on one box: lane point ops with (fused) and without (base) fe_addsub, headline + H2D leg, alternated 3x
set -o pipefail
mkdir -p gpurun_out/ab
LIB=cudabulletproof_amd/libcudabulletproof_hip.so
for rep in 1 2 3; do
  for name in base fused; do
    cp ab/lib_$name.so $LIB
    timeout -k 10 200 python bench.py --no-cpu --no-prove --no-ipa --no-msm --no-host --no-shard --no-check --steps 50 \
        > gpurun_out/ab/${name}_r$rep.json 2> gpurun_out/ab/${name}_r$rep.err || { tail -20 gpurun_out/ab/${name}_r$rep.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab/${name}_r$rep.json')); print('$name', $rep, round(d['value']), round(d['repeats']['median']), round(d['with_h2d']['value']))"
  done
done
cp ab/lib_fused.so $LIB
