#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs) over one marked eager
# step; bytes per launch of ENTRY -> profiles/pmc_traffic.json.
# usage: tools/gpu_pmc.sh TAG [ENTRY]
set -o pipefail
TAG=${1:-pmc}
ENTRY=${2:-um_conv2d_dgrad}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/$C -o run -- python3 $GRAFT_REPO_ROOT/tools/pmc_traffic.py run --entry $ENTRY > $OUT/$C.log 2>&1 || { echo "PMC $C FAILED"; tail -20 $OUT/$C.log; exit 1; }
  tail -1 $OUT/$C.log
done
cd $GRAFT_REPO_ROOT && python3 tools/pmc_traffic.py parse $OUT/FETCH_SIZE $OUT/WRITE_SIZE --entry $ENTRY --tag $TAG --out $OUT/pmc_traffic.json
