#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "reflect or halo or decoder or conv or model_forward or train_step" > $OUT/tests.log 2>&1 \
  || { echo TESTS FAILED; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
tools/gpu_arms.sh r03m_arms "UMAMD_X=0" "UMAMD_IG_PAD_DGRAD=2"
