set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "prefix or two_streams or overwritten" > gpurun_out/pytest_prefix.log 2>&1 || { tail -30 gpurun_out/pytest_prefix.log; exit 1; }
tail -2 gpurun_out/pytest_prefix.log
for K in 0 16 20 22; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu --no-ipa --no-prove --no-msm --prefix-bits $K > gpurun_out/ab_prefix_$K.json 2> gpurun_out/ab_prefix_$K.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_prefix_$K.json')); print($K, round(d['value']), d['config']['prefix_tables'], round(d['roofline']['avg_launch_ms'],3))"
done
