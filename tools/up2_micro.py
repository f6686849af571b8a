#!/usr/bin/env python3
"""Micro-benchmark of the decoder skip conv pieces at the full-resolution
stage (B=8, 256x512, fm 3->8 channels, skip 64 ch at 128x256, K=32): the
feature-map 1x1 conv with and without the up2 epilogue (um_conv2d_fwd_up2 vs
um_conv2d_fwd), f32 or bf16 output, with and without the BN statistics
slots, HIP events."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'uncertainty-model_amd'))

import torch  # noqa: E402

from umamd import functional as U  # noqa: E402
from umamd import _lib as L  # noqa: E402
from umamd._lib import call, ptr  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    dev = torch.device('cuda')
    for (N, H, W, Cf, K) in ((8, 256, 512, 8, 32), (8, 128, 256, 32, 64), (8, 64, 128, 64, 128)):
        h, w = H // 2, W // 2
        fm = torch.rand(N, H, W, Cf, device=dev).to(torch.bfloat16)
        z = torch.randn(N, h, w, K, device=dev)
        wt = torch.randn(K, Cf, 1, 1, device=dev)
        wf, _ = U._pack(wt, Cf, torch.bfloat16)
        bias = torch.zeros(K, device=dev)
        y = torch.empty(N, H, W, K, device=dev)
        yb = torch.empty(N, H, W, K, device=dev, dtype=torch.bfloat16)
        zb = z.to(torch.bfloat16)
        slots = torch.zeros(L.STAT_SLOTS * K * 2 + 1, dtype=torch.float64, device=dev)

        def up2():
            call('um_conv2d_fwd_up2', L.UM_BF16, N, H, W, Cf, Cf, ptr(fm), ptr(wf), ptr(bias), K,
                 H, W, ptr(y), K, L.EPI_STAT_SLOTS, ptr(slots), ptr(z), h, w, K)

        def up2b():
            call('um_conv2d_fwd_up2', L.UM_BF16 | L.Y_ACT, N, H, W, Cf, Cf, ptr(fm), ptr(wf),
                 ptr(bias), K, H, W, ptr(yb), K, L.EPI_STAT_SLOTS, ptr(slots), ptr(zb), h, w, K)

        def conv(out, epi):
            return lambda: U._conv_fwd(fm, wf, bias, K, 1, 1, 0, L.PAD_ZERO, out_dtype=out.dtype,
                                       epi=epi, stats=slots if epi else None, out=out)
        print(f'N{N} {H}x{W} C{Cf} K{K}: f32 none {timeit(conv(y, L.EPI_NONE)):6.1f}  '
              f'f32 slots {timeit(conv(y, L.EPI_STAT_SLOTS)):6.1f}  '
              f'bf16 none {timeit(conv(yb, L.EPI_NONE)):6.1f}  '
              f'bf16 slots {timeit(conv(yb, L.EPI_STAT_SLOTS)):6.1f}  '
              f'up2 f32 {timeit(up2):6.1f}  up2 bf16 {timeit(up2b):6.1f} us', flush=True)

if __name__ == '__main__':
    main()
