#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 \
  || { echo TESTS FAILED; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
tools/gpu_arms.sh r03o_arms "UMAMD_X=0" "UMAMD_GRAD_SLOTS=0"
