#!/bin/bash
# data-gradient micro timings: reflect (fold) vs zero padding, stride 2
mkdir -p gpurun_out
O=gpurun_out/dgrad_micro.txt
rm -f $O
for shape in "8 256 512 48 32 3 1" "8 32 64 320 256 3 1" "8 128 256 88 64 3 1" "8 256 512 32 8 3 1" "8 64 128 64 128 3 2" "8 128 256 32 64 5 2"; do
  for refl in "" "--reflect"; do
    echo "== $shape $refl" >> $O
    timeout -k 10 60 python -u tools/conv_micro.py $shape $refl --only dgrad >> $O 2>&1 || exit 1
  done
done
