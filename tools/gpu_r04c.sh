#!/bin/bash
# VALU heads + f16 pre-BN y: kernel tests, precision arms, throughput A/B
set -o pipefail
OUT=gpurun_out/${1:-r04r}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "disp_head or y16 or conv_bn_elu_slots or decoder_stage" > $OUT/ops.log 2>&1; tail -1 $OUT/ops.log; grep -E "^FAILED|^E  " $OUT/ops.log | head -12
timeout -k 10 400 python -u tools/bf16_arms.py "" "UMAMD_Y_F16=1" "UMAMD_VALU_HEAD=0" > $OUT/arms.txt 2>&1 || { echo ARMS FAILED; tail -20 $OUT/arms.txt; exit 1; }
grep -v Warn $OUT/arms.txt
FAST="--no-cpu-baseline --no-loss-delta --loader-steps 0 --fp32-steps 0 --eager-steps 0 --no-roofline --steps 30"
for rep in 1 2; do
  for arm in "" "UMAMD_VALU_HEAD=0" "UMAMD_Y_F16=1"; do
    env $arm timeout -k 10 300 python -u bench.py $FAST > $OUT/b.json 2> $OUT/b.err || { echo "BENCH [$arm] FAILED"; tail -20 $OUT/b.err; exit 1; }
    echo "[$arm] $(python3 -c "import json;d=json.load(open('$OUT/b.json'));print(d['value'],d['ms_per_step'])")"
  done
done
