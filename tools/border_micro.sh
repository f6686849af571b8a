#!/bin/bash
# reflect data gradient (split form: zero-pad pass + border fold) micro A/B:
#   tools/border_micro.sh OUT "ENV1" "ENV2" ...
set -o pipefail
OUT=$1; shift
mkdir -p gpurun_out/$OUT
for shape in "8 256 512 48 32 3 1 --reflect" "8 256 512 32 8 3 1 --reflect" "8 128 256 64 8 3 1 --reflect" "8 128 256 88 64 3 1 --reflect" "8 64 128 64 64 3 1 --reflect"; do
  for cfg in "$@"; do
    echo "== $cfg | $shape" >> gpurun_out/$OUT/micro.txt
    env $cfg timeout -k 10 60 python -u tools/conv_micro.py $shape --only dgrad 2>&1 | grep -v amdgpu.ids >> gpurun_out/$OUT/micro.txt || exit 1
  done
done
cat gpurun_out/$OUT/micro.txt
