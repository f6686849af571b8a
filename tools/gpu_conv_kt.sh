#!/bin/bash
# kernels of one conv entry on one shape (kernel trace): tools/gpu_conv_kt.sh TAG ENTRY "N H W C K R s" ...
set -o pipefail
TAG=$1; ENTRY=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for shape in "$@"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/k$i -o kt -- python3 $GRAFT_REPO_ROOT/tools/conv_micro.py $shape --only $ENTRY --iters 10 > $OUT/k$i.log 2>&1 || { tail $OUT/k$i.log; exit 1; }
  echo "== $shape: $(grep -i $ENTRY $OUT/k$i.log | tail -1)"
  python3 - <<PY
import csv, glob
for f in glob.glob('$OUT/k$i/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        n = r['Name'].replace('(anonymous namespace)::', '')
        if 'at::native' in n: continue
        print('   ', n[:100], r['Calls'], '%.1f us' % (float(r['AverageNs']) / 1e3))
PY
done
