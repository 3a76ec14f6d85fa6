#!/usr/bin/env bash
# GPU-box half of an A/B of prebuilt libraries: ab/lib_<name>.so (built here, e.g.
#   HIPBP_EXTRA_CFLAGS="-DBP_TERMS_OCC=3" python -c "import cudabulletproof_amd as b; b.build(force=True)"
# then copied to ab/lib_<name>.so), each swapped in as the product library and benched twice,
# alternating.   AB="base occ3" bash tools/ab_run.sh
set -e
LIB=cudabulletproof_amd/libcudabulletproof_hip.so
mkdir -p gpurun_out
for rep in 1 2; do for v in $AB; do
  cp ab/lib_$v.so $LIB
  timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu --no-ipa --no-prove --no-shard --no-host --no-msm > gpurun_out/ab_$v.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', round(d['value']))"
done; done
cp ab/lib_base.so $LIB
