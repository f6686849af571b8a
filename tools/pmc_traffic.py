#!/usr/bin/env python3
"""HBM traffic per launch of one C-ABI entry, from rocprofv3 PMC counters.

Two modes:

``run`` (executed under rocprofv3, one counter set per pass):
    builds the bench model (B=8, 256x512, bf16, bayesian), runs W eager
    warm-up steps, then ONE eager step in which every launch of ``--entry``
    is bracketed by a one-cycle ``spin_kernel`` marker
    (``umamd._lib.Recorder(marker=True)``).  The dispatches between a marker
    pair are that entry's kernels (igemm / halo / split-K epilogue ...).

``parse``:
    reads the ``*_counter_collection.csv`` of the FETCH_SIZE pass and of the
    WRITE_SIZE pass, sums each counter over the bracketed dispatches and
    writes ``profiles/pmc_traffic.json`` with bytes per entry launch:

        traffic = 2 * FETCH_SIZE + WRITE_SIZE     (both KiB -> bytes)

    FETCH_SIZE is doubled per MI355X_MICROARCH.md ("On gfx950 FETCH_SIZE
    reports exactly 1/2 of the bytes of a wide coalesced streaming read");
    WRITE_SIZE is exact for 16-B-per-lane stores.

Recipe (separate passes; never combine --pmc with trace domains):
    cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace \
        --output-format csv -d OUT/fetch -o run -- python3 REPO/tools/pmc_traffic.py run
    ... same with --pmc WRITE_SIZE -d OUT/write ...
    python3 tools/pmc_traffic.py parse OUT/fetch OUT/write
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MARK = 'spin_kernel'


def run(a):
    sys.path.insert(0, REPO)
    import torch
    import bench
    from umamd import _lib
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    cfg = bench.load_cfg('config.yml', 'bayesian')
    m, lf, opt = bench.build(cfg, 'bf16', dev, 1)
    g = torch.Generator(device='cpu').manual_seed(1234)
    left = torch.rand(8, 3, 256, 512, generator=g).to(dev)
    right = torch.rand(8, 3, 256, 512, generator=g).to(dev)
    for _ in range(a.warmup):
        bench.step(m, lf, opt, left, right, 0.3)
    torch.cuda.synchronize()
    rec = _lib.Recorder({a.entry}, marker=True)
    with rec:
        bench.step(m, lf, opt, left, right, 0.3)
    torch.cuda.synchronize()
    print(json.dumps({'entry': a.entry, 'launches': len(rec.items)}))


def _dispatches(d):
    """{dispatch_id: (kernel_name, {counter: value})} of one pass."""
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    if not files:
        raise SystemExit(f'no counter_collection.csv under {d}')
    out = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            did = int(r['Dispatch_Id'])
            name, ctrs = out.setdefault(did, (r['Kernel_Name'], {}))
            ctrs[r['Counter_Name']] = ctrs.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    return out


def _bracketed(disp, counter):
    """Sum ``counter`` over the dispatches between marker pairs; returns
    (per-launch totals, kernel names seen)."""
    ids = sorted(disp)
    per, names, cur = [], set(), None
    for i in ids:
        name, ctrs = disp[i]
        if MARK in name:
            if cur is None:
                cur = 0.0
            else:
                per.append(cur)
                cur = None
            continue
        if cur is not None:
            cur += ctrs.get(counter, 0.0)
            names.add(name.replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0])
    return per, names


def _lib_digest():
    path = os.path.join(REPO, 'uncertainty-model_amd', 'umamd', 'libumamd.so.stamp')
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def parse(a):
    f_per, names = _bracketed(_dispatches(a.fetch_dir), 'FETCH_SIZE')
    w_per, _ = _bracketed(_dispatches(a.write_dir), 'WRITE_SIZE')
    if not f_per or len(f_per) != len(w_per):
        raise SystemExit(f'marker pairs disagree: fetch {len(f_per)} write {len(w_per)}')
    kib = 1024.0
    fetch = [2.0 * v * kib for v in f_per]
    write = [v * kib for v in w_per]
    n = len(fetch)
    res = {
        'entry': a.entry,
        'launches': n,
        'fetch_bytes_per_launch': sum(fetch) / n,
        'write_bytes_per_launch': sum(write) / n,
        'traffic_bytes_per_launch': (sum(fetch) + sum(write)) / n,
        'formula': '2*FETCH_SIZE(KiB) + WRITE_SIZE(KiB), x1024; gfx950 FETCH_SIZE halving '
                   'corrected per MI355X_MICROARCH.md; separate --pmc passes',
        'workload': 'one eager bench step (B=8, 256x512, bf16, bayesian) after warm-up',
        'kernels': sorted(names),
        'source': a.tag,
        # the library these counters were taken on (bench.py reports the
        # traffic only while the library it loads has the same digest)
        'lib_digest': _lib_digest(),
    }
    out = a.out or os.path.join(REPO, 'profiles', 'pmc_traffic.json')
    with open(out, 'w') as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != 'kernels'}))


def parse1(a):
    """one counter of one pass, per launch of the entry, merged into the
    JSON ``a.out`` under the entry's name (e.g. SQ_INSTS_VALU of the loss
    launches: VALU wave-instructions per launch, bench.py's loss_stack)"""
    per, names = _bracketed(_dispatches(a.dir), a.counter)
    if not per:
        raise SystemExit('no marker pairs')
    out = a.out
    res = {}
    if os.path.exists(out):
        with open(out) as f:
            res = json.load(f)
    res[a.entry] = {'counter': a.counter, 'launches': len(per),
                    'per_launch': sum(per) / len(per), 'kernels': sorted(names),
                    'source': a.tag, 'lib_digest': _lib_digest()}
    with open(out, 'w') as f:
        json.dump(res, f, indent=1)
    print(json.dumps({a.entry: {k: v for k, v in res[a.entry].items() if k != 'kernels'}}))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest='mode', required=True)
    q = sub.add_parser('parse1')
    q.add_argument('dir')
    q.add_argument('--counter', default='SQ_INSTS_VALU')
    q.add_argument('--entry', default='um_loss_fwd')
    q.add_argument('--tag', default='')
    q.add_argument('--out', required=True)
    r = sub.add_parser('run')
    r.add_argument('--entry', default='um_conv2d_dgrad')
    r.add_argument('--warmup', type=int, default=3)
    p = sub.add_parser('parse')
    p.add_argument('fetch_dir')
    p.add_argument('write_dir')
    p.add_argument('--entry', default='um_conv2d_dgrad')
    p.add_argument('--tag', default='')
    p.add_argument('--out', default='')
    a = ap.parse_args()
    {'run': run, 'parse': parse, 'parse1': parse1}[a.mode](a)


if __name__ == '__main__':
    main()
