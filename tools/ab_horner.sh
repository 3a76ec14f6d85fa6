#!/usr/bin/env bash
# Horner A/B: ge_op16 rows (h1, the default) vs operand-form lane quads with squared doublings (h2);
# each library's Pippenger GPU tests (digests vs the oracle), then tools/pip_probe.py alternated
set -o pipefail
mkdir -p gpurun_out/abh
LIB=cudabulletproof_amd/libcudabulletproof_hip.so
cp ab/lib_h2.so $LIB
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pippenger or horner or fullsize" \
    > gpurun_out/abh/pytest_h2.log 2>&1 || { tail -40 gpurun_out/abh/pytest_h2.log; exit 1; }
tail -1 gpurun_out/abh/pytest_h2.log
for rep in 1 2; do for v in h1 h2; do
  cp ab/lib_$v.so $LIB
  timeout -k 10 120 python tools/pip_probe.py 20 12 12 2 > gpurun_out/abh/probe_${v}_$rep.txt 2>&1 || { tail -20 gpurun_out/abh/probe_${v}_$rep.txt; exit 1; }
  echo "$v $rep: $(grep -v amdgpu.ids gpurun_out/abh/probe_${v}_$rep.txt | tr '\n' ' ')"
done; done
for v in h1 h2; do
  cp ab/lib_$v.so $LIB
  timeout -k 10 120 python tools/pip_shard_probe.py > gpurun_out/abh/shard_${v}.txt 2>&1 || { tail -20 gpurun_out/abh/shard_${v}.txt; exit 1; }
  echo "$v shard: $(grep -E "msm_pippenger|horner|N=8" gpurun_out/abh/shard_${v}.txt | tr "\n" " ")"
done
