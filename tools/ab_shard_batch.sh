mkdir -p gpurun_out
# configs[4] push-batch A/B on one GPU: CFGS="total:push ..." (default: the round-2 sweep)
for cfg in ${CFGS:-8192:1024 8192:2048 8192:4096 16384:4096 65536:1024 65536:2048 65536:4096}; do
  cfg=${cfg/:/ }
  set -- $cfg
  timeout -k 10 200 python bench.py --shard-total $1 --shard-batch $2 --no-ipa --no-prove --no-msm --no-host --no-cpu --steps 10 > gpurun_out/sh_$1_$2.json 2>gpurun_out/sh_$1_$2.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/sh_$1_$2.json'))['sharded_2p16']; print($1, $2, round(d['value']), round(d['ms'],1), d['verdicts_sha256'], d['passes'])"
done
