#!/bin/bash
# A/B of env knobs on the bench step: tools/gpu_ab.sh TAG "ENV_A" "ENV_B" [pytest -k expr]
# each arm: bench (no CPU baseline / loss delta / loader / fp32 / eager legs), twice, interleaved
set -o pipefail
TAG=$1; A=$2; B=$3; K=${4:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1 \
    || { echo TESTS FAILED; grep -E "FAILED|Error" $OUT/tests.log | head; tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
FAST="--no-cpu-baseline --no-loss-delta --loader-steps 0 --fp32-steps 0 --eager-steps 0 --no-roofline --steps 30"
for rep in 1 2; do
  for arm in A B; do
    E=$A; [ $arm = B ] && E=$B
    env $E timeout -k 10 300 python -u bench.py $FAST > $OUT/$arm$rep.json 2> $OUT/$arm$rep.err || { echo "BENCH $arm FAILED"; tail -20 $OUT/$arm$rep.err; exit 1; }
    echo "$arm$rep [$E] $(python3 -c "import json;d=json.load(open('$OUT/$arm$rep.json'));print(d['value'],d['ms_per_step'])")"
  done
done
