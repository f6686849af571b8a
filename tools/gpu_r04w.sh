#!/bin/bash
# round-end evidence of the HEAD build: the default bench line, the rocprofv3
# kernel-trace --stats summary of the same command, the HBM traffic passes of
# the dominant entry and the counter passes.  usage: tools/gpu_r04w.sh TAG
set -o pipefail
T=${1:-r04w}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
tools/gpu_pmc.sh ${T}_pmc um_conv2d_dgrad || { echo PMC FAILED; exit 1; }
cat gpurun_out/${T}_pmc/pmc_traffic.json | head -30
cp gpurun_out/${T}_pmc/pmc_traffic.json profiles/pmc_traffic.json  # the bench line cites it
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/$OUT/bench_under_rocprof.json 2> $GRAFT_REPO_ROOT/$OUT/bench_under_rocprof.err) || { echo ROCPROF FAILED; tail -20 $OUT/bench_under_rocprof.err; exit 1; }
stats=$(find $OUT/prof -name '*kernel_stats.csv' | head -1)
cp $stats $OUT/kernel_stats.csv
find $OUT/prof -name '*kernel_trace.csv' -delete
head -25 $OUT/kernel_stats.csv | cut -c1-160
tools/gpu_pmc_counters.sh ${T}_cnt || { echo COUNTERS FAILED; exit 1; }
echo done
