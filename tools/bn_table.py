#!/usr/bin/env python3
"""Per-launch bandwidth table of the BN passes of one eager bench step.

tools/bn_table.py TRACE_DIR LABELS: joins the kernel trace of a
``tools/pmc_counters.py run --entries <BN entries> --labels LABELS`` pass
(marker-bracketed launches) with the launch arguments it recorded and prints,
per launch, the entry, dtype, M x C, duration and the compulsory bytes over
that duration (read da / y, write dy / a; y f32 unless the dtype carries
UM_Y_ACT).
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_counters import MARK  # noqa: E402


def main(d, labels):
    args = json.load(open(labels + '.args.json'))
    rows = []
    for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
        rows += [(int(r['Dispatch_Id']), r['Kernel_Name'],
                  float(r['End_Timestamp']) - float(r['Start_Timestamp'])) for r in csv.DictReader(open(f))]
    rows.sort()
    groups, cur = [], None
    for _, name, ns in rows:
        if MARK in name:
            if cur is None:
                cur = []
            else:
                groups.append(cur)
                cur = None
        elif cur is not None:
            cur.append((name, ns))
    assert len(groups) == len(args), (len(groups), len(args))
    tot = {}
    for (entry, a, _), g in zip(args, groups):
        dt, M, C = int(a[0]), int(a[1]), int(a[2])
        act = 2 if dt & 0xff else 4
        ybytes = act if dt & 0x100 else 4
        if 'fwd' in entry:
            b = M * C * (ybytes + act)
        elif 'reduce' in entry:
            b = M * C * (act + ybytes)
        else:
            b = M * C * (2 * act + ybytes)
        us = sum(ns for _, ns in g) / 1e3
        t = tot.setdefault(entry, [0, 0.0, 0.0])
        t[0] += 1
        t[1] += us
        t[2] += b
        print(f'{entry:28s} dt {dt:#5x} M {M:8d} C {C:4d} {us:7.1f} us {b / 1e6:7.1f} MB '
              f'{b / us / 1e3:6.0f} GB/s  {len(g)}k')
    for e, (n, us, b) in tot.items():
        print(f'TOTAL {e:28s} {n:3d} launches {us:8.1f} us {b / 1e6:8.1f} MB {b / us / 1e3:6.0f} GB/s')


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
