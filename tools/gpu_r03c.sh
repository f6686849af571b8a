#!/bin/bash
# full GPU suite then an A/B of one knob
set -o pipefail
OUT=gpurun_out/${1:-r03c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 \
  || { echo TESTS FAILED; grep -E "FAILED|Error" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
tools/gpu_ab.sh ${1:-r03c}_ab "$2" "$3"
