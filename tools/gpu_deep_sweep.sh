#!/bin/bash
# GEMM knob sweep: focused conv tests, whole-step A/B, per-conv table
set -o pipefail
OUT=gpurun_out/${1:-cls1}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -x -k "stride2 or tappack or dgrad or conv_bn_elu or conv_first" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/sweep.sh ${1:-cls1} "UMAMD_IG_CLS4=0" "UMAMD_IG_CLS4=1" "UMAMD_IG_CLS4=0" "UMAMD_IG_CLS4=1" || exit 1
UMAMD_IG_CLS4=1 timeout -k 10 200 python -u tools/conv_table.py --top 100 > $OUT/table.txt 2>&1 || exit 1
