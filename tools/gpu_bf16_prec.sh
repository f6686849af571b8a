#!/bin/bash
# bf16 vs fp32 forward errors with the pre-BN y in bf16 (UMAMD_Y_ACT=1, the
# default) and in f32 (UMAMD_Y_ACT=0): prints of the two precision tests
set -o pipefail
OUT=gpurun_out/${1:-r03prec}
mkdir -p $OUT
export TMPDIR=/tmp
for Y in 1 0; do
  UMAMD_Y_ACT=$Y timeout -k 10 300 python -u -m pytest -q -s --timeout 240 --timeout-method thread \
    tests/test_gpu_model.py::test_model_forward_bf16 tests/test_gpu_debug_bf16.py > $OUT/y$Y.log 2>&1 \
    || { echo "Y_ACT=$Y FAILED"; tail -20 $OUT/y$Y.log; exit 1; }
  echo "== UMAMD_Y_ACT=$Y"; grep -E "bf16 vs fp32|NODES|passed" $OUT/y$Y.log | cut -c1-400
done
