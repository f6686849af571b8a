#!/bin/bash
# bench arms (env settings), each run twice interleaved: tools/gpu_arms.sh TAG "ENV1" "ENV2" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
FAST="--no-cpu-baseline --no-loss-delta --loader-steps 0 --fp32-steps 0 --eager-steps 0 --no-roofline --steps 30"
for rep in 1 2; do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 300 python -u bench.py $FAST > $OUT/a$i.$rep.json 2> $OUT/a$i.$rep.err || { echo "BENCH [$E] FAILED"; tail -20 $OUT/a$i.$rep.err; exit 1; }
    echo "arm$i.$rep [$E] $(python3 -c "import json;d=json.load(open('$OUT/a$i.$rep.json'));print(d['value'],d['ms_per_step'])")"
  done
done
