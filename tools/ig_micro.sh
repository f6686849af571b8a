#!/bin/bash
# igemm micro sweep: knob settings x deep-layer shapes (fwd + dgrad):
#   tools/ig_micro.sh OUT "ENV1" "ENV2" ...
set -o pipefail
OUT=$1; shift
mkdir -p gpurun_out/$OUT
for cfg in "$@"; do
  for shape in "8 16 32 256 256 3 1" "8 8 16 512 512 3 1" "8 32 64 128 128 3 1" "8 64 128 64 64 3 1"; do
    echo "== $cfg | $shape" >> gpurun_out/$OUT/micro.txt
    env $cfg timeout -k 10 60 python -u tools/conv_micro.py $shape --only fwd >> gpurun_out/$OUT/micro.txt 2>&1 || exit 1
    env $cfg timeout -k 10 60 python -u tools/conv_micro.py $shape --only dgrad >> gpurun_out/$OUT/micro.txt 2>&1 || exit 1
  done
done
