#!/bin/bash
# full GPU suite, bench line, gloo 2-rank rehearsal, counter passes
set -o pipefail
OUT=gpurun_out/${1:-r03b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -s > $OUT/tests.log 2>&1 \
  || { echo TESTS FAILED; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
UMAMD_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 2 --no-roofline > $OUT/bench_gloo2.json 2> $OUT/bench_gloo2.err || { echo GLOO2 FAILED; tail -30 $OUT/bench_gloo2.err; exit 1; }
cat $OUT/bench_gloo2.json
tools/gpu_pmc_counters.sh ${1:-r03b}_pmc
