#!/usr/bin/env python3
"""Micro-benchmark of the fused loss launches at the bench shape (B=8,
256x512, 4 scales): pyramid, recon, loss forward, loss backward, each timed
with HIP events over R repetitions on random predictions.  Used under
rocprofv3 (--kernel-trace / --pmc) to look at one kernel at a time.

    python tools/loss_micro.py [--reps 20] [--only fwd|bwd|all]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'uncertainty-model_amd'), REPO]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--height', type=int, default=256)
    ap.add_argument('--width', type=int, default=512)
    ap.add_argument('--only', default='all')
    a = ap.parse_args()
    from umamd import lossfn as LF
    dev = torch.device('cuda', 0)
    g = torch.Generator(device='cpu').manual_seed(0)
    N, H, W = a.batch, a.height, a.width
    imgs = torch.rand(N, 6, H, W, generator=g).to(dev)
    preds = [(0.05 + 0.25 * torch.rand(N, H >> i, W >> i, 4, generator=g)).to(dev)
             .permute(0, 3, 1, 2).requires_grad_(True) for i in range(4)]
    cfg = {'alpha': 0.85, 'loss_type': 1, 'esw': 0.0, 'ecw': 0.5, 'w_wssim': 1.0,
           'w_cons': 1.0, 'w_smooth': 1.0, 'w_err': 1.0}
    pyr = LF.scale_pyramid(imgs, 4)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / a.reps * 1e3

    px = sum(N * (H >> i) * (W >> i) for i in range(4))
    res = {}
    if a.only in ('all', 'pyr'):
        res['pyramid'] = timed(lambda: LF.scale_pyramid(imgs, 4))
    if a.only in ('all', 'recon'):
        res['recon'] = timed(lambda: LF.reconstruct_pyramid(preds, pyr))
    if a.only in ('all', 'fwd'):
        def fwd_plain():
            with torch.no_grad():
                LF.tukra_loss(cfg, preds, pyr)
        res['loss_fwd'] = timed(fwd_plain)
        res['loss_fwd_fused'] = timed(lambda: LF.tukra_loss(cfg, preds, pyr))
    if a.only in ('all', 'bwd'):
        def fb():
            dl, el, _, _ = LF.tukra_loss(cfg, preds, pyr)
            torch.autograd.grad(dl + el, preds)
        res['loss_fwd_bwd'] = timed(fb)
    for k, us in res.items():
        print(f'{k:14s} {us:9.1f} us')
    if 'loss_fwd' in res:
        print(f'loss fwd: {40 * px / (res["loss_fwd"] * 1e-6) / 1e9:.0f} GB/s (40 B/px)')
    if 'loss_fwd_bwd' in res:
        print(f'loss fwd+bwd: {56 * px / (res["loss_fwd_bwd"] * 1e-6) / 1e9:.0f} GB/s (SURVEY 56 B/px)')


if __name__ == '__main__':
    main()
