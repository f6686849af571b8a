#!/usr/bin/env python3
"""Per-kernel totals of ONE replayed step from a rocprofv3 kernel trace (the
dispatches between the last two adam_kernel launches), so eager warm-up steps
do not skew per-step counts.  usage: tools/step_stats.py TRACE.csv [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Dispatch_Id']))
name = [r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
        for r in rows]
idx = [i for i, n in enumerate(name) if 'adam_kernel' in n]
# the last replayed bf16 step (the bench also runs an fp32 line after it)
pairs = [(idx[j] + 1, idx[j + 1] + 1) for j in range(len(idx) - 1)]
bf = [(x, y) for x, y in pairs if any('bfloat16' in name[i] for i in range(x, y))]
a, b = (bf or pairs)[-1]
tot = collections.defaultdict(lambda: [0, 0.0])
t0, t1 = int(rows[a]['Start_Timestamp']), int(rows[b - 1]['End_Timestamp'])
for i in range(a, b):
    d = (int(rows[i]['End_Timestamp']) - int(rows[i]['Start_Timestamp'])) / 1e3
    tot[name[i]][0] += 1
    tot[name[i]][1] += d
busy = sum(v[1] for v in tot.values())
print(f'kernels {b - a}, span {(t1 - t0) / 1e3:.1f} us, summed kernel time {busy:.1f} us')
for k, (n, us) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f'{us:8.1f} us {n:4d}x {us / n:7.1f}  {k[:100]}')
