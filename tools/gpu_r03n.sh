#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 300 --timeout-method thread -k "halo or reflect or conv_bn_elu" > $OUT/tests.log 2>&1 \
  || { echo TESTS FAILED; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
tools/gpu_arms.sh r03n_arms "UMAMD_X=0" "UMAMD_HALO_PF2=1"
