#!/bin/bash
# rocprofv3 kernel trace of the captured bench step only (no eager / loader /
# fp32 legs): tools/gpu_prof.sh TAG [extra bench args]
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
FAST="--no-cpu-baseline --no-loss-delta --loader-steps 0 --fp32-steps 0 --eager-steps 0 --no-roofline --steps 5 --warmup 3"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py $FAST "$@" > $OUT/prof.log 2>&1 || { echo PROF FAILED; tail -30 $OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/step_stats.py $OUT/prof/run_kernel_trace.csv 300 > $OUT/step_kernels.txt && python3 tools/step_launches.py $OUT/prof/run_kernel_trace.csv > $OUT/step_launches.txt && head -40 $OUT/step_kernels.txt
