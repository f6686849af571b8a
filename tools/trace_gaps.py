#!/usr/bin/env python3
"""Idle time inside ONE step of a rocprofv3 kernel trace: the span between the
last two adam_kernel launches, the union of all kernel intervals in it (any
stream) and the idle gaps (no kernel running), with the largest gaps and the
kernels on either side.  usage: tools/trace_gaps.py TRACE.csv [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
name = [r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
        for r in rows]
idx = [i for i, n in enumerate(name) if 'adam_kernel' in n]
a, b = idx[-2] + 1, idx[-1] + 1
iv = sorted((int(rows[i]['Start_Timestamp']), int(rows[i]['End_Timestamp']), name[i])
            for i in range(a, b))
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
busy, cur_s, cur_e, gaps, last = 0, iv[0][0], iv[0][1], [], iv[0][2]
for s, e, n in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, last, n))
        cur_s, cur_e = s, e
    elif e > cur_e:
        cur_e = e
    if e >= cur_e:
        last = n
busy += cur_e - cur_s
span = t1 - t0
print(f'kernels {len(iv)}, span {span / 1e3:.1f} us, busy (union) {busy / 1e3:.1f} us, '
      f'idle {(span - busy) / 1e3:.1f} us ({100 * (span - busy) / span:.1f} %), gaps {len(gaps)}')
for g, p, n in sorted(gaps, reverse=True)[:int(sys.argv[2]) if len(sys.argv) > 2 else 15]:
    print(f'{g / 1e3:8.2f} us  {p[:50]} -> {n[:50]}')
