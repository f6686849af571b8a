#!/bin/bash
# One GPU call: gpu tests, full bench line, rocprof kernel stats of a short bench.
# usage: tools/gpu_round.sh TAG [tests|notests]
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
fi
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-roofline > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { echo PROF FAILED; tail -30 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/$OUT/prof -name "*kernel_stats.csv"
