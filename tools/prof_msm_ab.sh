# PMC A/B of the MSM lane ordering: VALU instructions, waves and cycles of k_msm_points
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_msm_ab
mkdir -p $OUT
for m in 0 1; do
HIPBP_MSM_SORT=$m timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/s$m -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-ipa --no-prove --msm-log2 20 > $OUT/s$m.json 2> $OUT/s$m.err
done
echo ok
