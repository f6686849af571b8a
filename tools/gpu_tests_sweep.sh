#!/bin/bash
# Full GPU tests, then a throughput sweep: tools/gpu_tests_sweep.sh TAG "ENV1" ...
set -o pipefail
TAG=${1:-ts}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/sweep.sh $TAG "$@"
