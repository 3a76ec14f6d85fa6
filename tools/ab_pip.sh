#!/usr/bin/env bash
# GPU-box half of a Pippenger A/B of prebuilt libraries ab/lib_<name>.so (see tools/ab_run.sh):
# each swapped in as the product library, tools/pip_probe.py 20 12 12 2 twice, alternating.
#   AB="base s16_8" bash tools/ab_pip.sh
set -e
LIB=cudabulletproof_amd/libcudabulletproof_hip.so
mkdir -p gpurun_out
for rep in 1 2; do for v in $AB; do
  cp ab/lib_$v.so $LIB
  echo "== $v"
  timeout -k 10 120 python tools/pip_probe.py 20 12 12 2
done; done
cp ab/lib_base.so $LIB
