#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run, and the per-step kernel
# table of one replayed step: tools/prof_step.sh OUT [bench args...]
set -o pipefail
OUT=$1; shift
mkdir -p gpurun_out/$OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --no-cpu-baseline "$@" > $GRAFT_REPO_ROOT/gpurun_out/$OUT/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/$OUT/bench.err || exit $?
cd $GRAFT_REPO_ROOT
trace=$(find gpurun_out/$OUT/prof -name '*kernel_trace.csv' | head -1)
stats=$(find gpurun_out/$OUT/prof -name '*kernel_stats.csv' | head -1)
cp $stats gpurun_out/$OUT/kernel_stats.csv
python3 tools/step_stats.py $trace 200 > gpurun_out/$OUT/step_kernels.txt
python3 tools/step_launches.py $trace > gpurun_out/$OUT/step_launches.txt 2>&1 || true
python3 tools/trace_gaps.py $trace 25 > gpurun_out/$OUT/gaps.txt 2>&1 || true
rm -f $trace
