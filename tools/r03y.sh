set -o pipefail
mkdir -p gpurun_out
SKIP_UBENCH=1 bash tools/round3_check.sh r03y || exit 1
REPS=3 timeout -k 10 400 python tools/shard_probe.py 8192 4096,4096+3072+1024,3072+3072+1024+1024,2048 16384:32768 > gpurun_out/shard_probe_r03y.txt 2>&1 || { tail -20 gpurun_out/shard_probe_r03y.txt; exit 1; }
tail -30 gpurun_out/shard_probe_r03y.txt
