set -e
mkdir -p gpurun_out/ab
for rep in 1 2; do
for cfg in "64 1" "0 1" "0 0" "64 0"; do
set -- $cfg
HIPBP_LANE_TREE_MAX=$1 HIPBP_CHAINS_FIRST=$2 timeout -k 10 120 python bench.py --no-cpu --no-prove --no-msm --no-ipa --steps 20 > gpurun_out/ab/lt$1_cf$2_r$rep.json 2>/dev/null
done
done
echo ok
