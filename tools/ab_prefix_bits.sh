#!/usr/bin/env bash
# A/B: prefix-table width K (bench.py --prefix-bits) for the headline and the prove leg, two runs each.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for k in ${KS:-22 23}; do
  timeout -k 10 400 python -u bench.py --no-cpu --no-ipa --no-msm --no-shard --no-host --no-h2d --no-check \
      --prefix-bits $k > gpurun_out/abk.json 2> gpurun_out/abk.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/abk.json'));print('K',$k,round(d['value']),'repeats',round(d['repeats']['median']),'prove',round(d['prove']['value']))"
done; done
