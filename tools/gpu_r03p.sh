#!/bin/bash
# full GPU suite, knob arms, up2 micro, replayed-step trace (idle gaps)
set -o pipefail
T=${1:-r03p}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 \
  || { echo TESTS FAILED; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python -u tools/up2_micro.py > $OUT/up2_micro.txt 2>&1 || { echo UP2 FAILED; tail $OUT/up2_micro.txt; exit 1; }
cat $OUT/up2_micro.txt
tools/gpu_arms.sh ${T}_arms "UMAMD_X=0" "UMAMD_UP2_VALU=0"
tools/prof_step.sh ${T}_prof --loader-steps 0 --fp32-steps 0 --no-loss-delta --eager-steps 0 --no-roofline || { echo PROF FAILED; exit 1; }
head -3 gpurun_out/${T}_prof/step_kernels.txt
head -25 gpurun_out/${T}_prof/gaps.txt
