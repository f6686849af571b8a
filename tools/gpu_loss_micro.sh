#!/bin/bash
# loss micro-benchmark + kernel trace + PMC passes (one counter group per pass)
set -o pipefail
OUT=gpurun_out/${1:-lm}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/loss_micro.py > $OUT/micro.txt 2>&1 || { cat $OUT/micro.txt; exit 1; }
cat $OUT/micro.txt
R=$GRAFT_REPO_ROOT/$OUT
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt -o kt -- python3 $GRAFT_REPO_ROOT/tools/loss_micro.py --reps 5 > $R/kt.log 2>&1 || exit 1
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" \
           "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $R/pmc$i -o p -- python3 $GRAFT_REPO_ROOT/tools/loss_micro.py --reps 2 > $R/pmc$i.log 2>&1 || echo "pmc pass $i failed"
done
