#!/bin/bash
# full GPU suite, default bench line, rocprof step table of the HEAD build
set -o pipefail
OUT=gpurun_out/${1:-r03e}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 \
  || { echo TESTS FAILED; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
tools/prof_step.sh ${1:-r03e}_prof --loader-steps 0 --fp32-steps 0 --no-loss-delta
head -40 gpurun_out/${1:-r03e}_prof/step_kernels.txt
timeout -k 10 120 python -u tools/gemm_ceiling.py > gpurun_out/${1:-r03e}/gemm_ceiling.txt 2>&1 || { echo CEILING FAILED; tail -20 gpurun_out/${1:-r03e}/gemm_ceiling.txt; exit 1; }
cat gpurun_out/${1:-r03e}/gemm_ceiling.txt
tools/gpu_trace_table.sh ${1:-r03e}_trace
