#!/usr/bin/env bash
# A/B: the headline (configs[1], B = 1024 per step) over 2..4 pipelines (bench.py --pipes), two runs each.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for np in ${PIPES:-2 3 4}; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-ipa --no-msm --no-shard --no-host --no-prove --no-h2d --no-check \
      --pipes $np > gpurun_out/abpp.json 2> gpurun_out/abpp.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abpp.json'));r=d['repeats'];print('pipes',$np,round(d['value']),'repeats median',round(r['median']))"
done; done
