#!/bin/bash
# round-4: smoke(), the default bench line, then dp1 vs dp1+SyncBN on a
# one-rank RCCL group (UMAMD_DIST=1), twice interleaved
set -o pipefail
OUT=gpurun_out/${1:-r04o}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', d['value'], d['ms_per_step'], d.get('leg_errors'))"
FAST="--no-cpu-baseline --no-loss-delta --loader-steps 0 --fp32-steps 0 --eager-steps 0 --no-roofline --steps 30"
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py $FAST > $OUT/dp1.$rep.json 2> $OUT/dp1.$rep.err || { echo DP1 FAILED; tail -20 $OUT/dp1.$rep.err; exit 1; }
  echo "dp1 $(python3 -c "import json;d=json.load(open('$OUT/dp1.$rep.json'));print(d['value'],d['ms_per_step'],d['config']['parallelism'])")"
  UMAMD_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29520+rep)) bench.py $FAST > $OUT/sync.$rep.json 2> $OUT/sync.$rep.err || { echo "SYNC FAILED"; tail -20 $OUT/sync.$rep.err; exit 1; }
  echo "dp1+syncbn $(python3 -c "import json;d=json.load(open('$OUT/sync.$rep.json'));print(d['value'],d['ms_per_step'],d['config']['parallelism'])")"
done
