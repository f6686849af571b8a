#!/usr/bin/env python3
"""Per-call table of the conv entries of one eager train step (bench shape):
shape, HIP-event time and TFLOP/s, sorted by time.  Each launch is bracketed
by a device synchronize so the events time the kernel alone.
usage: python tools/conv_table.py [--dtype bf16] [--top 60]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, 'uncertainty-model_amd'), REPO):
    sys.path.insert(0, p)

import torch  # noqa: E402

import bench  # noqa: E402
from umamd import _lib as L  # noqa: E402

NAMES = ('um_conv2d_fwd', 'um_conv2d_dgrad', 'um_conv2d_wgrad', 'um_conv_wgrad_reduce_seg')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--dtype', default='bf16')
    ap.add_argument('--top', type=int, default=70)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    cfg = bench.load_cfg('config.yml', 'bayesian')
    m, lf, opt = bench.build(cfg, a.dtype, dev, 1)
    g = torch.Generator().manual_seed(1234)
    left = torch.rand(8, 3, 256, 512, generator=g).to(dev)
    right = torch.rand(8, 3, 256, 512, generator=g).to(dev)
    for _ in range(2):
        bench.step(m, lf, opt, left, right, 0.3)
    torch.cuda.synchronize()
    orig = L.call
    rows = []

    def timed(name, *args, work=None):
        if name not in NAMES:
            return orig(name, *args, work=work)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(name, *args, work=work)
        e1.record()
        e1.synchronize()
        rows.append((name, args, e0.elapsed_time(e1), work))

    L.call = timed
    import umamd.functional as F
    F.call = timed
    bench.step(m, lf, opt, left, right, 0.3)
    torch.cuda.synchronize()
    L.call = F.call = orig
    tot = {}
    for name, args, ms, work in rows:
        tot[name] = tot.get(name, 0.0) + ms
    print('totals (ms):', {k: round(v, 3) for k, v in tot.items()})
    rows.sort(key=lambda r: -r[2])
    for name, args, ms, work in rows[:a.top]:
        if name == 'um_conv2d_fwd':
            N, H, W, C, K, R, s = args[1], args[2], args[3], args[4], args[9], args[10], args[11]
        elif name == 'um_conv2d_dgrad':
            N, H, W, C, K, R, s = args[1], args[2], args[3], args[4], args[9], args[10], args[11]
        elif name == 'um_conv2d_wgrad':
            N, H, W, C, K, R, s = args[1], args[2], args[3], args[4], args[7], args[8], args[9]
        else:
            print(f'{ms * 1e3:8.1f} us  {name} splits={args[1]} K={args[2]} R={args[4]} C={args[5]}')
            continue
        tf = (work / (ms * 1e-3) / 1e12) if work else 0.0
        pm = ' refl' if name != 'um_conv2d_wgrad' and args[13] == 1 else ''
        print(f'{ms * 1e3:8.1f} us  {name[10:]:6s} N{N} {H}x{W} C{C} K{K} R{R} s{s}{pm}  '
              f'{tf:7.1f} TFLOP/s')


if __name__ == '__main__':
    main()
