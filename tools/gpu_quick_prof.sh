#!/bin/bash
# focused GPU tests (-k expression), bench without the CPU baseline, and a
# rocprofv3 kernel-stats pass: tools/gpu_quick_prof.sh TAG "pytest -k expr"
set -o pipefail
TAG=${1:-qp}; K=${2:-"decoder or concat or up2"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "$K" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline --steps 30 > $OUT/bench$i.json 2> $OUT/bench$i.err || { echo BENCH FAILED; tail -30 $OUT/bench$i.err; exit 1; }; cut -c1-200 $OUT/bench$i.json; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-roofline > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { echo PROF FAILED; tail -30 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
