#!/usr/bin/env python3
"""Micro-benchmark of the conv entry points on one shape (bf16, NHWC):
times um_conv2d_fwd / um_conv2d_dgrad / um_conv2d_wgrad (+ slab reduce)
with HIP events and prints TFLOP/s.  For kernel tuning and rocprofv3 PMC
passes:  python tools/conv_micro.py N H W C K R stride [reflect] [--only wgrad]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'uncertainty-model_amd'))

import torch  # noqa: E402

from umamd import functional as U  # noqa: E402
from umamd import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    for k in ('N', 'H', 'W', 'C', 'K', 'R', 'stride'):
        ap.add_argument(k, type=int)
    ap.add_argument('--reflect', action='store_true')
    ap.add_argument('--only', default='all')
    ap.add_argument('--iters', type=int, default=20)
    a = ap.parse_args()
    dev = torch.device('cuda')
    pad = (a.R - 1) // 2
    pm = L.PAD_REFLECT if a.reflect else L.PAD_ZERO
    P = (a.H + 2 * pad - a.R) // a.stride + 1
    Q = (a.W + 2 * pad - a.R) // a.stride + 1
    x = torch.randn(a.N, a.H, a.W, a.C, device=dev).to(torch.bfloat16)
    dy = torch.randn(a.N, P, Q, a.K, device=dev).to(torch.bfloat16)
    w = torch.randn(a.K, a.C, a.R, a.R, device=dev)
    wf, wT = U._pack(w, a.C, torch.bfloat16)
    flops = 2.0 * a.N * P * Q * a.K * a.R * a.R * a.C
    ops = {
        'fwd': lambda: U._conv_fwd(x, wf, None, a.K, a.R, a.stride, pad, pm),
        'dgrad': lambda: U._conv_dgrad(dy, wT, x.shape, a.K, a.R, a.stride, pad, pm),
        'wgrad': lambda: U._conv_wgrad(x, dy, a.K, a.K, a.C, a.R, a.stride, pad, pm),
    }
    for name, fn in ops.items():
        if a.only not in ('all', name):
            continue
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        print(f'{name:6s} {ms * 1e3:9.1f} us  {flops / ms / 1e9:8.1f} TFLOP/s')


if __name__ == '__main__':
    main()
