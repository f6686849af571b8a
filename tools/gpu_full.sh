#!/bin/bash
# the round-end sequence on one box: full -m gpu suite, smoke, default bench line
# usage: tools/gpu_full.sh TAG
set -o pipefail
TAG=${1:-full}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
