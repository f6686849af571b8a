#!/bin/bash
# rocprofv3 counter passes over one marked eager bench step (tools/pmc_counters.py):
# a kernel-trace-only pass (durations) + 3 PMC passes (MFMA, VALU/LDS, occupancy/stalls),
# each its own run under a hard time limit.  usage: tools/gpu_pmc_counters.sh TAG
set -o pipefail
TAG=${1:-pmcc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
R="python3 $GRAFT_REPO_ROOT/tools/pmc_counters.py run --labels $OUT/labels.json"
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- $R > $OUT/trace.log 2>&1 || { echo "TRACE FAILED"; tail -20 $OUT/trace.log; exit 1; }
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P3="SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- $R > $OUT/p$i.log 2>&1 || { echo "PASS $i FAILED"; tail -20 $OUT/p$i.log; exit 1; }
  tail -1 $OUT/p$i.log
done
cd $GRAFT_REPO_ROOT && python3 tools/pmc_counters.py parse $OUT/trace $OUT/p1 $OUT/p2 $OUT/p3 --labels $OUT/labels.json --out $OUT/counters.json
