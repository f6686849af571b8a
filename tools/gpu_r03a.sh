#!/bin/bash
# round-3 first call: new parity tests, graph/ddp tests, bench (loss delta +
# CPU sweep), gloo 2-rank bench rehearsal, counter list
set -o pipefail
OUT=gpurun_out/r03a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "counter list failed"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity_c2.py tests/test_gpu_graph.py tests/test_gpu_imageprep.py \
  "tests/test_gpu_model.py::test_nodes10_train_step_matches_oracle" -m gpu -s > $OUT/tests.log 2>&1 \
  || { echo TESTS FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
UMAMD_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 2 --no-roofline > $OUT/bench_gloo2.json 2> $OUT/bench_gloo2.err || { echo GLOO2 FAILED; tail -30 $OUT/bench_gloo2.err; exit 1; }
cat $OUT/bench_gloo2.json
