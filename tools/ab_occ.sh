#!/usr/bin/env bash
# k_terms occupancy A/B: the default build (128 VGPRs, 4 blocks per CU, no VGPRs left for other
# kernels' waves) vs a 96-VGPR build (ab/lib_wpe5.so, -DBP_TERMS_WPE=5), each with and without a
# dynamic LDS pad that caps k_terms at 4 blocks per CU (HIPBP_TERMS_LDS_PAD): headline verify bench
# and the configs[4] rank-shard probe per variant.
set -o pipefail
TAG=${1:-r03o}
mkdir -p gpurun_out
LIB=cudabulletproof_amd/libcudabulletproof_hip.so
cp $LIB /tmp/lib_default.so
run() {  # name lib pad
  cp "$2" $LIB
  HIPBP_TERMS_LDS_PAD=$3 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu --no-ipa --no-prove --no-msm \
      --no-host --no-check --no-h2d --no-shard > gpurun_out/ab_${TAG}_$1.json 2> gpurun_out/ab_${TAG}_$1.err || { tail -20 gpurun_out/ab_${TAG}_$1.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_${TAG}_$1.json')); print('$1 bench', round(d['value']), 'k_terms ms', round(d['roofline']['avg_launch_ms'], 3))"
  HIPBP_TERMS_LDS_PAD=$3 REPS=3 timeout -k 10 200 python tools/shard_probe.py 8192 4096 49152,16384:32768,24576:49152 > gpurun_out/ab_${TAG}_$1_shard.txt 2>&1 || { tail -20 gpurun_out/ab_${TAG}_$1_shard.txt; return 1; }
  echo "$1 $(grep push gpurun_out/ab_${TAG}_$1_shard.txt)"
}
run v0 /tmp/lib_default.so 0 && run v1 ab/lib_wpe5.so 0 && run v1pad ab/lib_wpe5.so 4096 && run v0b /tmp/lib_default.so 0
rc=$?
cp /tmp/lib_default.so $LIB
exit $rc
