#!/usr/bin/env bash
# A/B of prebuilt libraries on the GPU box: ab/lib_<name>.so copied in as the product library
# (the box's copy of the tree only), each configuration run alternately, twice.
#   tools/ab_libs.sh "base:1 new:0 new:1"     (name:HIPBP_LANE_SORT)
set -e
mkdir -p gpurun_out/ab
LIB=cudabulletproof_amd/libcudabulletproof_hip.so
for rep in 1 2; do
for cfg in $1; do
name=${cfg%%:*}; ls=${cfg##*:}
cp ab/lib_$name.so $LIB
HIPBP_LANE_SORT=$ls timeout -k 10 150 python bench.py --no-cpu --no-prove --no-ipa --steps 20 > gpurun_out/ab/${name}_s${ls}_r$rep.json 2>/dev/null
done
done
echo ok
