#!/bin/bash
# SQ_INSTS_VALU (VALU wave-instructions) per launch of the loss entries, one
# --pmc pass each over one marked eager step -> OUT/pmc_loss_valu.json
# usage: tools/gpu_pmc_valu.sh TAG [ENTRY ...]
set -o pipefail
TAG=${1:-valu}; shift
ENTRIES=${@:-um_loss_fwd um_loss_bwd}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for E in $ENTRIES; do
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU --kernel-trace --output-format csv -d $OUT/$E -o run -- python3 $GRAFT_REPO_ROOT/tools/pmc_traffic.py run --entry $E > $OUT/$E.log 2>&1 || { echo "PMC $E FAILED"; tail -20 $OUT/$E.log; exit 1; }
  (cd $GRAFT_REPO_ROOT && python3 tools/pmc_traffic.py parse1 $OUT/$E --counter SQ_INSTS_VALU --entry $E --tag $TAG --out $OUT/pmc_loss_valu.json) || exit 1
done
