#!/bin/bash
# One GPU call: selected op tests, per-conv table, bench (no CPU baseline).
# usage: tools/gpu_quick.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-quick}
K=${2:-"reflect or conv_bn_elu or dgrad"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -x -k "$K" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python -u tools/conv_table.py --top 200 > $OUT/table.txt 2>&1 || { echo TABLE FAILED; tail -20 $OUT/table.txt; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
