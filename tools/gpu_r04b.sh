#!/bin/bash
# dp1+SyncBN (one-rank RCCL group, UMAMD_DIST=1) variants: own RCCL
# communicators vs the process group, bucket sizes
set -o pipefail
OUT=gpurun_out/${1:-r04p}
mkdir -p $OUT
export TMPDIR=/tmp
FAST="--no-cpu-baseline --no-loss-delta --loader-steps 0 --fp32-steps 0 --eager-steps 0 --no-roofline --steps 30"
i=0
for arm in "" "UMAMD_OWN_RCCL=0" "UMAMD_GRAD_BUCKET_MB=0" "UMAMD_OWN_RCCL=0 UMAMD_GRAD_BUCKET_MB=0"; do
  i=$((i+1))
  env $arm UMAMD_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29530+i)) bench.py $FAST > $OUT/a$i.json 2> $OUT/a$i.err || { echo "ARM [$arm] FAILED"; tail -20 $OUT/a$i.err; exit 1; }
  echo "[$arm] $(python3 -c "import json;d=json.load(open('$OUT/a$i.json'));print(d['value'],d['ms_per_step'],d['config']['launch'])")"
done
