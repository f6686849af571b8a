#!/bin/bash
# Overlap A/B + focused tests: tools/gpu_ab.sh TAG "ENV1" "ENV2" ...
set -o pipefail
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
bash tools/sweep.sh $TAG "$@"
