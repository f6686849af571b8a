#!/bin/bash
# ablation arms of the captured bench step: tools/gpu_ablate.sh TAG GROUP...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
FAST="--no-cpu-baseline --no-loss-delta --loader-steps 0 --fp32-steps 0 --eager-steps 0 --no-roofline --steps 30"
for rep in 1 2; do
  for G in "$@"; do
    timeout -k 10 300 python -u tools/ablate.py $G $FAST > $OUT/$G.$rep.json 2> $OUT/$G.$rep.err || { echo "ARM [$G] FAILED"; tail -20 $OUT/$G.$rep.err; exit 1; }
    echo "arm [$G].$rep $(python3 -c "import json;d=json.load(open('$OUT/$G.$rep.json'));print(d['value'],d['ms_per_step'])")"
  done
done
