#!/bin/bash
# GPU tests (optionally a -k subset) + the fast bench line twice: tools/gpu_tb.sh TAG [pytest -k expr]
set -o pipefail
TAG=$1; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${KA[@]}" > $OUT/tests.log 2>&1 \
  || { echo TESTS FAILED; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
FAST="--no-cpu-baseline --no-loss-delta --loader-steps 0 --fp32-steps 0 --eager-steps 0 --no-roofline --steps 30"
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py $FAST > $OUT/b$rep.json 2> $OUT/b$rep.err || { echo "BENCH FAILED"; tail -20 $OUT/b$rep.err; exit 1; }
  echo "b$rep $(python3 -c "import json;d=json.load(open('$OUT/b$rep.json'));print(d['value'],d['ms_per_step'])")"
done
