#!/bin/bash
# A/B of the one-rank data-parallel graph bench under env settings
set -o pipefail
OUT=gpurun_out/${1:-distab}; shift; mkdir -p $OUT
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg UMAMD_DIST=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29540+i)) bench.py --gpus 1 --no-cpu-baseline --no-roofline --steps 30 > $OUT/ab_$i.json 2> $OUT/ab_$i.err || { echo "FAILED $cfg"; tail -5 $OUT/ab_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" $OUT/ab_$i.json "$cfg"
done
