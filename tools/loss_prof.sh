#!/bin/bash
# per-kernel times of the loss stack for each scatter form, smooth and
# per-pixel-noise disparities: tools/loss_prof.sh TAG
set -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for c in smooth noise; do
  LOSS_MICRO_CASE=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$c -o run -- python3 -u tools/loss_scatter_micro.py ${KNOB:-loss_scatter} ${VALS:-0 2} > $OUT/$c.txt 2>&1 || { tail -20 $OUT/$c.txt; exit 1; }
  grep "scatter=" $OUT/$c.txt
  f=$(find $OUT/$c -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if 'loss' in n: print('$c', n.split('(')[0][-60:], r['Calls'], '%.1f us' % (float(r['AverageNs'])/1e3))
"
done
