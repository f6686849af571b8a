#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter CSVs (one dispatch row per
counter): python tools/pmc_summary.py gpurun_out/lm/pmc1 [gpurun_out/lm/pmc2 ...]"""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    for f in glob.glob(f'{d}/**/*counter_collection.csv', recursive=True):
        tot = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0][-40:]
            tot[k][r['Counter_Name']] += float(r['Counter_Value'])
            disp[k].add(r['Dispatch_Id'])
        for k, v in tot.items():
            n = len(disp[k])
            print(f'{k:42s} n={n:3d} ' + ' '.join(f'{c}={x / n:.4g}' for c, x in sorted(v.items())))
