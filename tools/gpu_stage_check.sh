mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_stg.log 2>&1 || exit 1
for shape in "8 256 512 72 32 1 1" "8 128 256 160 64 1 1" "8 64 128 320 128 1 1"; do
  echo "== $shape" >> gpurun_out/stg_micro.txt
  timeout -k 10 60 python -u tools/conv_micro.py $shape --only fwd >> gpurun_out/stg_micro.txt 2>&1 || exit 1
  timeout -k 10 60 python -u tools/conv_micro.py $shape --only dgrad >> gpurun_out/stg_micro.txt 2>&1 || exit 1
done
bash tools/sweep.sh stg "UMAMD_X=2"
