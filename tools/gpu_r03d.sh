#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 \
  || { echo TESTS FAILED; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
tools/gpu_ab.sh r03d_ab "UMAMD_STAGE_FN=1" "UMAMD_STAGE_FN=0"
tools/gpu_ab.sh r03d_ab2 "UMAMD_STAGE_FN=1 UMAMD_WGRAD_OVERLAP=0" "UMAMD_STAGE_FN=0 UMAMD_WGRAD_OVERLAP=0"
