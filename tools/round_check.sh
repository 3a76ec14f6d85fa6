#!/usr/bin/env bash
# Round-end check on the GPU box: full GPU test suite, smoke(), the default bench line.
#   tools/round_check.sh <tag>  -> gpurun_out/pytest_<tag>.log, gpurun_out/bench_<tag>.json
set -o pipefail
TAG=${1:-chk}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
python - "$TAG" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/bench_{sys.argv[1]}.json"))
print(round(d["value"]), round(d["valu_roofline"]["frac"], 3), "msm", round(d["msm"]["value"] / 1e6, 1),
      "pip", round(d["msm"]["pippenger"]["value"] / 1e6, 1), "ipa", round(d["ipa"]["value"]), "prove",
      round(d["prove"]["value"]), "shard", round(d["sharded_2p16"]["value"]), "host", round(d["host_api"]["value"]),
      "cpu", round(d["cpu_baseline"]["value"], 1))
PY
