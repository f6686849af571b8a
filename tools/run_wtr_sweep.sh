set -o pipefail
mkdir -p gpurun_out
for t in 64 128; do
  UMAMD_WTR_TBK=$t timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k wgrad > gpurun_out/wtr_test_$t.log 2>&1 || exit 1
done
bash tools/sweep.sh wtr "UMAMD_WTR_TBK=32" "UMAMD_WTR_TBK=64" "UMAMD_WTR_TBK=128" "UMAMD_WTR_TBK=64 UMAMD_WSPLIT_BLOCKS=384" "UMAMD_WTR_TBK=128 UMAMD_WSPLIT_BLOCKS=384" "UMAMD_WTR_TBK=128 UMAMD_WSPLIT_BLOCKS=256" "UMAMD_WTR_TBK=64 UMAMD_WSPLIT_BLOCKS=512"
