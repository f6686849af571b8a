#!/bin/bash
# One GPU call: selected op tests, default bench line, and the rocprofv3
# step table of a replayed step (tools/prof_step.sh).
# usage: tools/gpu_step_prof.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-step}; K=${2:-disp_head}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -v -x -k "$K" --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { echo TESTS FAILED; tail -40 $OUT/t.log; exit 1; }
tail -3 $OUT/t.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-loss-delta > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
bash tools/prof_step.sh $TAG/prof --no-loss-delta --loader-steps 0 --fp32-steps 0 --eager-steps 0 --no-roofline && head -40 $OUT/prof/step_kernels.txt
