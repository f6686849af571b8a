#!/bin/bash
# one test under an env setting: tools/gpu_t2.sh "ENV=..." test_id
set -o pipefail
mkdir -p gpurun_out/t2
env $1 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s "$2" -m gpu > gpurun_out/t2/tests.log 2>&1; rc=$?
echo "rc=$rc"
grep -E "PASSED|FAILED|Fatal|passed|failed" gpurun_out/t2/tests.log | tail -5
