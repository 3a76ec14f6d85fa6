# A/B of the MSM lane ordering (HIPBP_MSM_SORT: 0 off, 1 longest first, 2 shortest first)
set -e
mkdir -p gpurun_out/abm
for rep in 1 2; do
for m in 0 1 2; do
HIPBP_MSM_SORT=$m timeout -k 10 120 python bench.py --no-cpu --no-prove --no-ipa --steps 2 > gpurun_out/abm/s${m}_r${rep}.json 2>/dev/null
done
done
echo ok
