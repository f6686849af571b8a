#!/usr/bin/env python3
"""Every launch of ONE replayed step (as tools/step_stats.py picks it) in
dispatch order: start offset, duration, grid / workgroup size, queue, name.
usage: tools/step_launches.py TRACE.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Dispatch_Id']))
name = [r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
        for r in rows]
idx = [i for i, n in enumerate(name) if 'adam_kernel' in n]
pairs = [(idx[j] + 1, idx[j + 1] + 1) for j in range(len(idx) - 1)]
bf = [(x, y) for x, y in pairs if any('bfloat16' in name[i] for i in range(x, y))]
a, b = (bf or pairs)[-1]
t0 = int(rows[a]['Start_Timestamp'])


def g(r, k):
    return r.get(k) or r.get(k.replace('_Size', '_Size_X')) or '?'


for i in range(a, b):
    r = rows[i]
    s = (int(r['Start_Timestamp']) - t0) / 1e3
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    print(f'{s:9.1f} {d:7.1f}  grid {g(r, "Grid_Size"):>9} wg {g(r, "Workgroup_Size"):>4} '
          f'q {r.get("Queue_Id", "?"):>3}  {name[i][:110]}')
