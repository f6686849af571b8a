#!/bin/bash
# one marked eager bench step under rocprofv3 --kernel-trace: per-launch table
# (entry, shape args, kernels, duration) of the conv/BN/loss entries
set -o pipefail
TAG=${1:-trace}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/pmc_counters.py run --labels $OUT/labels.json > $OUT/trace.log 2>&1 || { echo "TRACE FAILED"; tail -20 $OUT/trace.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/pmc_counters.py parse $OUT/trace --labels $OUT/labels.json --out $OUT/table.json
