#!/bin/bash
# stride-2 data-gradient micro-benchmark (per shape, UMAMD_TUNING arms) + kernel names
# usage: tools/gpu_s2_micro.sh TAG "ARM1" "ARM2" ...
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for arm in "$@"; do
  for shape in "8 128 256 32 64 5 2" "8 64 128 64 128 3 2" "8 32 64 128 256 3 2" "8 16 32 256 512 3 2"; do
    echo "[$arm] $shape: $(UMAMD_TUNING="$arm" timeout -k 10 60 python3 $GRAFT_REPO_ROOT/tools/conv_micro.py $shape --only dgrad 2>&1 | grep -i dgrad | tail -1)"
  done
done
cd /tmp
UMAMD_TUNING="$1" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py 8 64 128 64 128 3 2 --only dgrad > $OUT/kt.log 2>&1 || exit 1
python3 - <<PY
import csv, glob
for f in glob.glob('$OUT/kt/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print(r['Name'][:90], r['Calls'], '%.1f us' % (float(r['AverageNs']) / 1e3))
PY
