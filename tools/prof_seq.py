#!/usr/bin/env python3
"""Per-dispatch timeline of ONE graph-replayed train step from a rocprofv3
--kernel-trace sqlite db (the dispatches between the last two Adam launches),
plus a per-kernel-family summary.  usage: prof_seq.py DB [out.txt]"""
import re
import sqlite3
import sys


def short(n):
    n = n.replace('(anonymous namespace)::', '')
    if n.startswith('void '):
        n = n[5:]
    return n.split('(')[0]


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute('select name,start,end,grid_x,grid_y,grid_z,workgroup_x,vgpr_count,'
                     'accum_vgpr_count,lds_size from kernels order by start').fetchall()
    idx = [i for i, r in enumerate(rows) if 'adam_kernel' in r[0]]
    a, b = idx[-2], idx[-1]
    seq = rows[a + 1:b + 1]
    busy = sum(r[2] - r[1] for r in seq)
    span = seq[-1][2] - seq[0][1]
    out = open(sys.argv[2], 'w') if len(sys.argv) > 2 else sys.stdout
    print(f'# step: {len(seq)} dispatches, busy {busy / 1e6:.3f} ms, span {span / 1e6:.3f} ms', file=out)
    prev = None
    fam = {}
    for r in seq:
        n = short(r[0])
        gap = (r[1] - prev) / 1e3 if prev else 0.0
        prev = r[2]
        d = (r[2] - r[1]) / 1e3
        print(f'{d:8.1f} gap{gap:6.1f} grid=({r[3]},{r[4]},{r[5]})x{r[6]} v{r[7]}+{r[8]} lds{r[9]} {n[:120]}', file=out)
        k = re.split(r'<', n)[0]
        f = fam.setdefault(k, [0, 0.0])
        f[0] += 1
        f[1] += d
    print('# family: calls, us', file=out)
    for k, (cnt, us) in sorted(fam.items(), key=lambda x: -x[1][1]):
        print(f'# {k:40s} {cnt:5d} {us:9.1f}', file=out)


if __name__ == '__main__':
    main()
