"""Micro-benchmark of the one-pass disparity-head kernels (csrc/disphead.hip)
at the four C2 head shapes (B=8): mean kernel time over repeated launches
(HIP events on the launch stream) against the compulsory HBM bytes.
usage: python tools/head_micro.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'uncertainty-model_amd'))
from umamd._lib import call, ptr  # noqa: E402
from umamd import functional as U  # noqa: E402

SHAPES = [(32, 64, 256), (64, 128, 128), (128, 256, 64), (256, 512, 32)]  # (H, W, C) at B=8


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps  # us


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    N = 8
    torch.manual_seed(0)
    for H, W, C in SHAPES:
        conv = torch.nn.Conv2d(C, 4, 3).cuda()
        wf, wT = U._pack(conv.weight, C, torch.bfloat16, ldT=8, split=True)
        b = conv.bias.detach().float().contiguous()
        x = torch.randn(N, H, W, C, device='cuda').to(torch.bfloat16)
        d = torch.empty(N, H, W, 4, device='cuda')
        dl = torch.randn(N, H, W, 8, device='cuda').to(torch.bfloat16)
        dx = torch.empty_like(x)
        M = N * H * W
        tf = timed(lambda: call('um_disp_head_fwd', N, H, W, C, ptr(x), C, ptr(wf), ptr(b), 0.3,
                                ptr(d), 4), reps)
        tg = timed(lambda: call('um_disp_head_dgrad', N, H, W, C, ptr(dl), 8, ptr(wT), ptr(dx),
                                C, 0), reps)
        bf = M * (C * 2 + 16)
        bg = M * (16 + C * 2)
        print(f'N{N} {H}x{W} C{C}: fwd {tf:7.1f} us ({bf / tf / 1e3:6.0f} GB/s)  '
              f'dgrad {tg:7.1f} us ({bg / tg / 1e3:6.0f} GB/s)', flush=True)


if __name__ == '__main__':
    main()
