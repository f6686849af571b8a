#!/bin/bash
# the data-parallel captured path on a one-rank RCCL group (UMAMD_DIST=1):
# bucketed overlapped gradient all-reduce vs one all-reduce at the end, vs dp1
set -o pipefail
OUT=gpurun_out/${1:-dist1}
mkdir -p $OUT
FAST="--no-cpu-baseline --no-loss-delta --loader-steps 0 --fp32-steps 0 --eager-steps 0 --no-roofline --steps 30"
timeout -k 10 300 python -u bench.py $FAST > $OUT/dp1.json 2> $OUT/dp1.err || { echo DP1 FAILED; tail -20 $OUT/dp1.err; exit 1; }
echo "dp1 $(python3 -c "import json;d=json.load(open('$OUT/dp1.json'));print(d['value'],d['config']['parallelism'])")"
for MB in 16 0; do
  UMAMD_DIST=1 UMAMD_GRAD_BUCKET_MB=$MB timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py $FAST > $OUT/dist_mb$MB.json 2> $OUT/dist_mb$MB.err || { echo "DIST $MB FAILED"; tail -20 $OUT/dist_mb$MB.err; exit 1; }
  echo "dist1 bucket_mb=$MB $(python3 -c "import json;d=json.load(open('$OUT/dist_mb$MB.json'));print(d['value'],d['config']['parallelism'],d['config']['launch'])")"
done
