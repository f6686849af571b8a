#!/usr/bin/env python3
"""What a library GEMM (hipBLASLt via torch.matmul) does on the deep layers'
implicit-GEMM shapes, beside the umamd conv entries on the same conv:
M = N*P*Q pixels, N = K output channels, K = R*R*C.  The library number is
the plain GEMM on an explicit (pre-built) im2col operand -- a ceiling for the
contraction alone, not a drop-in (it skips the gather and the epilogue).
usage: tools/gemm_ceiling.py [--iters 50]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'uncertainty-model_amd'))

import torch  # noqa: E402

from umamd import functional as U  # noqa: E402
from umamd import _lib as L  # noqa: E402

SHAPES = [  # N H W C K R
    (8, 32, 64, 128, 128, 3),
    (8, 16, 32, 256, 256, 3),
    (8, 8, 16, 512, 512, 3),
    (8, 64, 128, 64, 64, 3),
    (8, 16, 32, 512, 256, 3),
    (8, 32, 64, 256, 128, 3),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=50)
    a = ap.parse_args()
    dev = torch.device('cuda')
    torch.manual_seed(0)
    print(f'{"shape":28s} {"GFLOP":>6s} {"mm us":>7s} {"mm TF":>6s} {"fwd us":>7s} {"fwd TF":>6s} '
          f'{"dgrad us":>8s} {"dg TF":>6s}')
    for (N, H, W, C, K, R) in SHAPES:
        pad = (R - 1) // 2
        M, KK = N * H * W, R * R * C
        flops = 2.0 * M * K * KK
        A = (torch.rand(M, KK, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(KK, K, device=dev) * 2 - 1).to(torch.bfloat16)
        mm = timeit(lambda: torch.matmul(A, B), a.iters)
        x = (torch.rand(N, H, W, C, device=dev) * 2 - 1).to(torch.bfloat16)
        dy = (torch.rand(N, H, W, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = torch.randn(K, C, R, R, device=dev)
        wf, wT = U._pack(w, C, torch.bfloat16)
        fwd = timeit(lambda: U._conv_fwd(x, wf, None, K, R, 1, pad, L.PAD_ZERO), a.iters)
        dg = timeit(lambda: U._conv_dgrad(dy, wT, x.shape, K, R, 1, pad, L.PAD_ZERO), a.iters)
        tf = lambda us: flops / us / 1e6  # noqa: E731
        print(f'{str((N, H, W, C, K, R)):28s} {flops / 1e9:6.2f} {mm:7.1f} {tf(mm):6.0f} {fwd:7.1f} '
              f'{tf(fwd):6.0f} {dg:8.1f} {tf(dg):6.0f}', flush=True)


if __name__ == '__main__':
    main()
