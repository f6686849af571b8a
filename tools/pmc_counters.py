#!/usr/bin/env python3
"""Per-kernel rocprofv3 counters of one bench step, attributed to C-ABI entries.

``run`` (under rocprofv3, one counter set per pass -- or --kernel-trace only):
    the bench model (B=8, 256x512, bf16, bayesian), W eager warm-up steps,
    then ONE eager step in which every launch of the selected entries is
    bracketed by a one-cycle ``spin_kernel`` marker; the entry names in launch
    order are written to --labels.

``parse PASS_DIR... --labels L --out O``:
    joins every pass's ``*_counter_collection.csv`` (and the
    ``*_kernel_trace.csv`` durations when a pass has one) by dispatch id and
    writes per entry and per kernel name: launches, summed counters, mean
    duration, and the derived ratios

      mfma_busy      = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * GRBM_GUI_ACTIVE/8)
                       (GRBM_GUI_ACTIVE is summed over the 8 XCDs; checked on
                       MI355X: equals 512 * MOPS_BF16 / duration / 2.5 PF within
                       ~10 %, so it is the fraction of the dense bf16 peak)
      mfma_tflops    = 512 * SQ_INSTS_VALU_MFMA_MOPS_BF16 / duration
      valu_issue     = 2 * SQ_INSTS_VALU / (1024 * GRBM_GUI_ACTIVE/8)
                       (2 cycles per wave64 VALU op on a SIMD32 pair; a lower
                       bound of the issue time's share of the kernel)
      lds_conflict   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
      occupancy      = 4 * SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE/8) / 256
                       (mean resident waves per CU; SQ_WAVE_CYCLES counts
                       quad-cycles; SQ_ACCUM_PREV_HIRES read 0 on gfx950)
      wait_any       = SQ_WAIT_ANY / SQ_WAVE_CYCLES (share of wave time stalled)
      wait_lds       = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
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
ENTRIES = ['um_conv2d_fwd', 'um_conv2d_dgrad', 'um_conv2d_wgrad', 'um_loss_fwd', 'um_loss_bwd',
           'um_bn_elu_fwd_slots', 'um_bn_elu_bwd_reduce_slots', 'um_bn_elu_bwd_apply_slots']


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
    rec = _lib.Recorder(set(a.entries.split(',')), marker=True)
    with rec:
        bench.step(m, lf, opt, left, right, 0.3)
    torch.cuda.synchronize()
    with open(a.labels, 'w') as f:
        json.dump([name for name, *_ in rec.items], f)
    with open(a.labels + '.args.json', 'w') as f:  # per launch: entry, scalar args, FLOPs
        json.dump([[name, [v for v in args if isinstance(v, (int, float))], work]
                   for name, args, _, _, work in rec.items], f)
    print(json.dumps({'launches': len(rec.items)}))


def _short(name):
    return name.replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]


def _load(d):
    """-> ({dispatch_id: (kernel, {counter: value})}, {dispatch_id: ns})"""
    ctr = {}
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            did = int(r['Dispatch_Id'])
            name, c = ctr.setdefault(did, (r['Kernel_Name'], {}))
            c[r['Counter_Name']] = c.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    dur = {}
    for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            did = int(r['Dispatch_Id'])
            dur[did] = (r['Kernel_Name'], float(r['End_Timestamp']) - float(r['Start_Timestamp']))
    return ctr, dur


def _brackets(items):
    """[(kernel, data)] in dispatch order -> [[(kernel, data)] per marker pair]"""
    out, cur = [], None
    for name, data in items:
        if MARK in name:
            if cur is None:
                cur = []
            else:
                out.append(cur)
                cur = None
            continue
        if cur is not None:
            cur.append((name, data))
    return out


def parse(a):
    labels = json.load(open(a.labels))
    per_entry, per_kernel = {}, {}
    npass = {}  # counter -> number of passes that collected it (GRBM_GUI_ACTIVE is in each)
    for d in a.dirs:
        ctr, dur = _load(d)
        for cn in {cn for _, c in ctr.values() for cn in c}:
            npass[cn] = npass.get(cn, 0) + 1
        # durations only from the trace-only pass (counter passes serialise
        # and slow the kernels down)
        src = ctr if ctr else {k: (v[0], {}) for k, v in dur.items()}
        items = [(src[i][0], (src[i][1], None if ctr else dur[i][1])) for i in sorted(src)]
        br = _brackets(items)
        if len(br) != len(labels):
            raise SystemExit(f'{d}: {len(br)} marker pairs vs {len(labels)} labels')
        for lab, group in zip(labels, br):
            e = per_entry.setdefault(lab, {'launches': 0, 'dispatches': 0, 'ns': 0.0,
                                           'counters': {}})
            for name, (c, ns) in group:
                k = per_kernel.setdefault(_short(name), {'entry': lab, 'dispatches': 0,
                                                         'ns': 0.0, 'counters': {}})
                for cn, v in c.items():
                    e['counters'][cn] = e['counters'].get(cn, 0.0) + v
                    k['counters'][cn] = k['counters'].get(cn, 0.0) + v
                if ns is not None:
                    e['ns'] += ns
                    k['ns'] += ns
                    k['dispatches'] += 1
                    e['dispatches'] += 1
            if any(ns is not None for _, (_, ns) in group):
                e['launches'] += 1
    for t in list(per_entry.values()) + list(per_kernel.values()):
        # counters collected in several passes: the per-pass mean
        t['counters'] = {cn: v / npass.get(cn, 1) for cn, v in t['counters'].items()}
        c = t['counters']
        cyc = c.get('GRBM_GUI_ACTIVE', 0.0) / 8.0
        der = {}
        if cyc and 'SQ_VALU_MFMA_BUSY_CYCLES' in c:
            der['mfma_busy'] = c['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024.0 * cyc)
        if t['ns'] and 'SQ_INSTS_VALU_MFMA_MOPS_BF16' in c:
            der['mfma_tflops'] = 512.0 * c['SQ_INSTS_VALU_MFMA_MOPS_BF16'] / (t['ns'] * 1e-9) / 1e12
        if cyc and 'SQ_INSTS_VALU' in c:
            der['valu_issue'] = 2.0 * c['SQ_INSTS_VALU'] / (1024.0 * cyc)
        if c.get('SQ_LDS_IDX_ACTIVE'):
            der['lds_conflict'] = c.get('SQ_LDS_BANK_CONFLICT', 0.0) / c['SQ_LDS_IDX_ACTIVE']
        if cyc and 'SQ_WAVE_CYCLES' in c:  # quad-cycles (MI355X_MICROARCH.md)
            der['occupancy_waves_per_cu'] = 4.0 * c['SQ_WAVE_CYCLES'] / cyc / 256.0
        if c.get('SQ_WAVE_CYCLES'):
            if 'SQ_WAIT_ANY' in c:
                der['wait_any'] = c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']
            if 'SQ_WAIT_INST_LDS' in c:
                der['wait_lds'] = c['SQ_WAIT_INST_LDS'] / c['SQ_WAVE_CYCLES']
        t['derived'] = {k: round(v, 4) for k, v in der.items()}
        n = t.get('launches') or t.get('dispatches') or 1
        t['mean_us'] = round(t['ns'] / max(n, 1) / 1e3, 2)
    # per-launch table from the trace-only pass: entry, shape args, kernels, us
    launches = []
    args_path = a.labels + '.args.json'
    if os.path.exists(args_path):
        largs = json.load(open(args_path))
        for d in a.dirs:
            ctr, dur = _load(d)
            if ctr:
                continue
            items = [(dur[i][0], dur[i][1]) for i in sorted(dur)]
            for (lab, args, work), group in zip(largs, _brackets(items)):
                ns = sum(v for _, v in group)
                launches.append({'entry': lab, 'args': args, 'us': round(ns / 1e3, 2),
                                 'tflops': round(work / ns / 1e3, 1) if work and ns else None,
                                 'kernels': [_short(n) for n, _ in group]})
            break
    res = {'launch_table': sorted(launches, key=lambda r: -r['us']),
           'workload': 'one eager bench step (B=8, 256x512, bf16, bayesian) after warm-up; '
                       'entries bracketed by spin_kernel markers',
           'passes': a.dirs, 'entries': per_entry,
           'kernels': dict(sorted(per_kernel.items(), key=lambda kv: -kv[1]['ns']))}
    with open(a.out, 'w') as f:
        json.dump(res, f, indent=1)
    for lab, e in per_entry.items():
        print(lab, e['launches'], e['mean_us'], e['derived'])


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest='mode', required=True)
    r = sub.add_parser('run')
    r.add_argument('--entries', default=','.join(ENTRIES))
    r.add_argument('--warmup', type=int, default=3)
    r.add_argument('--labels', required=True)
    p = sub.add_parser('parse')
    p.add_argument('dirs', nargs='+')
    p.add_argument('--labels', required=True)
    p.add_argument('--out', required=True)
    a = ap.parse_args()
    run(a) if a.mode == 'run' else parse(a)


if __name__ == '__main__':
    main()
