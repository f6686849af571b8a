#!/bin/bash
# VALU heads: kernel tests, then a rocprof step table (per-kernel times)
set -o pipefail
OUT=gpurun_out/${1:-r04s}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "disp_head or y16" > $OUT/ops.log 2>&1; tail -1 $OUT/ops.log; grep -E "^FAILED|^E  " $OUT/ops.log | head -12
bash tools/prof_step.sh ${1:-r04s}_prof --no-loss-delta --loader-steps 0 --fp32-steps 0 --eager-steps 0 || { echo PROF FAILED; exit 1; }
grep -iE "head|igemm_kernel<__hip_bfloat16, 32, 256, 16|halo_conv_kernel<3, 16|sigmoid|kernels " gpurun_out/${1:-r04s}_prof/step_kernels.txt | head -20
python3 -c "import json;d=json.load(open('gpurun_out/${1:-r04s}_prof/bench.json'));print(d['value']);print(json.dumps(d['roofline'].get('disp_heads'))[:1500])"
