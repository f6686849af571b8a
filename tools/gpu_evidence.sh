#!/bin/bash
# Round-end evidence on one box, in order: PMC traffic of the dominant entry
# and the loss VALU counters (copied into profiles/ so the bench line on this
# library reports them), the full -m gpu suite, smoke, the default bench line,
# rocprofv3 kernel stats of the bench command and the replayed-step table.
# usage: tools/gpu_evidence.sh TAG [ENTRY]
set -o pipefail
TAG=${1:-ev}; ENTRY=${2:-um_conv2d_wgrad}
OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/gpu_pmc.sh $TAG/pmc $ENTRY > $OUT/pmc.log 2>&1 || { echo PMC FAILED; tail -20 $OUT/pmc.log; exit 1; }
cp $OUT/pmc/pmc_traffic.json profiles/pmc_traffic.json
bash tools/gpu_pmc_valu.sh $TAG/valu > $OUT/valu.log 2>&1 || { echo VALU FAILED; tail -20 $OUT/valu.log; exit 1; }
cp $OUT/valu/pmc_loss_valu.json profiles/pmc_loss_valu.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cut -c1-200 $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/bprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/bench_prof.json 2> $GRAFT_REPO_ROOT/$OUT/bench_prof.err || { echo BENCH PROF FAILED; exit 1; }
cd $GRAFT_REPO_ROOT
cp $(find $OUT/bprof -name '*kernel_stats.csv' | head -1) $OUT/bench_kernel_stats.csv
rm -f $(find $OUT/bprof -name '*kernel_trace.csv')
bash tools/prof_step.sh $TAG/step --no-loss-delta --loader-steps 0 --fp32-steps 0 --eager-steps 0 --no-roofline > $OUT/step.log 2>&1 || { echo STEP FAILED; exit 1; }
head -1 $OUT/step/step_kernels.txt
