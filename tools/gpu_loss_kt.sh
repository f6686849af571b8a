#!/bin/bash
# loss micro-benchmark + its per-kernel averages (kernel trace): tools/gpu_loss_kt.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-lkt}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/loss_micro.py > $OUT/micro.txt 2>&1 || { cat $OUT/micro.txt; exit 1; }
cat $OUT/micro.txt
R=$GRAFT_REPO_ROOT/$OUT
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt -o kt -- python3 $GRAFT_REPO_ROOT/tools/loss_micro.py --reps 5 > $R/kt.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python3 - <<PY
import csv, glob
for f in glob.glob('$R/kt/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'loss' in r['Name'] or 'recon' in r['Name'] or 'pyramid' in r['Name']:
            print(r['Name'].replace('(anonymous namespace)::', '')[:60], r['Calls'], '%.1f us' % (float(r['AverageNs']) / 1e3))
PY
