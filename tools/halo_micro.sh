#!/bin/bash
# halo conv micro A/B: knob settings x high-resolution shapes (fwd + dgrad):
#   tools/halo_micro.sh OUT "ENV1" "ENV2" ...
set -o pipefail
OUT=$1; shift
mkdir -p gpurun_out/$OUT
for shape in "8 256 512 32 32 3 1" "8 256 512 48 32 3 1 --reflect" "8 128 256 64 64 3 1" "8 128 256 32 32 7 1" "8 64 128 64 64 5 1" "8 128 256 88 64 3 1 --reflect"; do
  for cfg in "$@"; do
    echo "== $cfg | $shape" >> gpurun_out/$OUT/micro.txt
    env $cfg timeout -k 10 60 python -u tools/conv_micro.py $shape --only fwd >> gpurun_out/$OUT/micro.txt 2>&1 || exit 1
    env $cfg timeout -k 10 60 python -u tools/conv_micro.py $shape --only dgrad >> gpurun_out/$OUT/micro.txt 2>&1 || exit 1
  done
done
cat gpurun_out/$OUT/micro.txt
