#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/t1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity_c2.py tests/test_gpu_graph.py -m gpu > gpurun_out/t1/tests.log 2>&1; echo "rc=$?"
grep -E "PASSED|FAILED|Fatal|passed|failed" gpurun_out/t1/tests.log | tail -20
