#!/bin/bash
# head kernel micro-benchmark under each variant knob, then the head tests
set -o pipefail
OUT=gpurun_out/${1:-hm}; mkdir -p $OUT
for v in ${ARMS:-"dh_fwd=0" "dh_fwd=3" "dh_fwd=4" "dh_fwd=5"}; do
  echo "== $v" | tee -a $OUT/micro.txt
  UMAMD_TUNING=$v timeout -k 10 120 python -u tools/head_micro.py 100 2>&1 | tee -a $OUT/micro.txt || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -x -k "disp_head" --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
