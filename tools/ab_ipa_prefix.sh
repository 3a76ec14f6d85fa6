set -eo pipefail
mkdir -p gpurun_out/ipa_ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "gens_inner_product or msm_batch_gens or msm_batch" --timeout 200 --timeout-method thread 2>&1 | tail -2
for rep in 1 2; do for b in 0 14; do
timeout -k 10 200 python bench.py --steps 2 --warmup 1 --prefix-bits 0 --no-cpu --no-msm --no-prove --no-shard --no-host --ipa-steps 8 --ipa-prefix-bits $b > gpurun_out/ipa_ab/b${b}_r$rep.json 2>/dev/null
python -c "import json,sys;d=json.load(open('gpurun_out/ipa_ab/b${b}_r$rep.json'))['ipa'];print($b,round(d['value']),round(d['value_P_given']),d['prefix_tables'],d['P_tables_equal_plain'])"
done; done
