#!/bin/bash
# reflect-pad data gradient per strategy (UMAMD_TUNING arms) on the decoder shapes
# usage: tools/gpu_refl_micro.sh TAG "ARM1" "ARM2" ...
set -o pipefail
TAG=$1; shift
for arm in "$@"; do
  for shape in "8 256 512 48 32 3 1" "8 128 256 64 32 3 1" "8 128 256 88 64 3 1" "8 256 512 32 8 3 1" "8 64 128 128 64 3 1" "8 128 256 32 32 3 1"; do
    echo "[$arm] $shape: $(UMAMD_TUNING="$arm" timeout -k 10 60 python3 tools/conv_micro.py $shape --reflect --only dgrad 2>&1 | grep -i dgrad | tail -1)"
  done
done
