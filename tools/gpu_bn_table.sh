#!/bin/bash
# per-launch bandwidth of the BN passes of one eager step: tools/gpu_bn_table.sh TAG
set -o pipefail
TAG=${1:-bnt}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
E=um_bn_elu_fwd_slots,um_bn_elu_bwd_reduce_slots,um_bn_elu_bwd_apply_slots
cd /tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/pmc_counters.py run --entries $E --labels $OUT/labels.json > $OUT/trace.log 2>&1 || { echo "TRACE FAILED"; tail -20 $OUT/trace.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/bn_table.py $OUT/trace $OUT/labels.json > $OUT/table.txt && rm -rf $OUT/trace && tail -4 $OUT/table.txt
