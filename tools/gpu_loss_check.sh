#!/bin/bash
# loss tests + per-seed bf16 test, bench + step table, VALU PMC of the loss entries
set -o pipefail
TAG=${1:-loss}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_loss_stack.py tests/test_gpu_model.py -v -s -x -k "loss or bf16" --timeout 280 --timeout-method thread > $OUT/t.log 2>&1 || { echo TESTS FAILED; grep -E "seed|RMS|envelope|FAILED|Error|assert" $OUT/t.log | tail -30; exit 1; }
grep -E "seed |RMS|envelope|passed|failed" $OUT/t.log | tail -30
bash tools/gpu_step_prof.sh $TAG/s disp_head_onepass > $OUT/step.log 2>&1 || { echo STEP FAILED; tail -20 $OUT/step.log; exit 1; }
cut -c1-200 $OUT/s/bench.json; head -1 $OUT/s/prof/step_kernels.txt; grep loss_ $OUT/s/prof/step_kernels.txt
bash tools/gpu_pmc_valu.sh $TAG/valu
