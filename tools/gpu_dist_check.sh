#!/bin/bash
# full GPU tests, single-GPU bench, and the data-parallel graph path on a
# one-rank RCCL group (UMAMD_DIST=1 keeps the SyncBN all-reduces at world 1)
set -o pipefail
OUT=gpurun_out/${1:-dist}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cut -c1-220 $OUT/bench.json
UMAMD_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --no-cpu-baseline --no-roofline > $OUT/bench_dist1.json 2> $OUT/bench_dist1.err || { echo DIST BENCH FAILED; tail -30 $OUT/bench_dist1.err; exit 1; }
cat $OUT/bench_dist1.json | cut -c1-220
