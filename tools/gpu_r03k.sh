#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "decoder or graph or wgrad or model or merge or conv" > $OUT/tests.log 2>&1 \
  || { echo TESTS FAILED; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
tools/gpu_arms.sh r03k_arms "UMAMD_X=0" "UMAMD_MWG_BATCH=0" "UMAMD_FUSED_MERGE=0" "UMAMD_WRED_BATCH=1"
