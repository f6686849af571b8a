#!/usr/bin/env python3
"""Per-dispatch timeline of ONE graph-replayed step from rocprofv3
--kernel-trace csv output (dispatches between the last two Adam launches)
and a per-kernel-family summary.  usage: prof_csv.py kernel_trace.csv [out]"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    ad = [i for i, r in enumerate(rows) if 'adam_kernel' in r['Kernel_Name']]
    seq = rows[ad[-2] + 1:ad[-1] + 1]
    out = open(sys.argv[2], 'w') if len(sys.argv) > 2 else sys.stdout
    busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in seq)
    span = int(seq[-1]['End_Timestamp']) - int(seq[0]['Start_Timestamp'])
    print(f'# step: {len(seq)} dispatches, busy {busy / 1e6:.3f} ms, span {span / 1e6:.3f} ms',
          file=out)
    fam = {}
    for r in seq:
        n = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('__hip_bfloat16', 'bf')
        n = re.sub(r'^void ', '', n).split('(')[0]
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        wg = int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X']))
        print(f'{d:8.1f} wg={wg:6d}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]} {n[:90]}', file=out)
        k = n.split('<')[0]
        f = fam.setdefault(k, [0, 0.0])
        f[0] += 1
        f[1] += d
    for k, (c, us) in sorted(fam.items(), key=lambda x: -x[1][1]):
        print(f'# {k:40s} {c:5d} {us:9.1f}', file=out)


if __name__ == '__main__':
    main()
