#!/bin/bash
# GEMM knob sweep: focused conv tests, whole-step A/B, per-conv tables
set -o pipefail
OUT=gpurun_out/${1:-deep2}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -x -k "glds_stage or dgrad or conv_bn_elu" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/sweep.sh ${1:-deep2} "UMAMD_IG_XCD_COL=0" "UMAMD_IG_XCD_COL=1" "UMAMD_IG_XCD_COL=0" "UMAMD_IG_XCD_COL=1" "UMAMD_IG_XCD_COL=1 UMAMD_IG_GLDS_DEEP=3" || exit 1
UMAMD_IG_XCD_COL=0 timeout -k 10 200 python -u tools/conv_table.py --top 80 > $OUT/table_x0.txt 2>&1 || exit 1
UMAMD_IG_XCD_COL=1 timeout -k 10 200 python -u tools/conv_table.py --top 80 > $OUT/table_x1.txt 2>&1 || exit 1
