#!/bin/bash
# run one test under several knob settings: tools/gpu_bisect.sh TAG TESTID "ENV1" "ENV2" ...
set -o pipefail
TAG=$1; TID=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u -m pytest "$TID" -x -q --timeout 240 --timeout-method thread > $OUT/b$i.log 2>&1
  rc=$?
  echo "[$E] rc=$rc $(tail -1 $OUT/b$i.log)"
  if [ $rc -ge 124 ]; then echo "stopping (rc $rc)"; exit 1; fi
done
