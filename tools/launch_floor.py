#!/usr/bin/env python3
"""Calibrate the per-kernel floor on this box: N dependent tiny kernels
(torch add_ on a 1-element tensor) eager vs captured in one HIP graph."""
import time

import torch

x = torch.zeros(1, device='cuda')
N = 500
for _ in range(3):
    for _ in range(N):
        x.add_(1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    x.add_(1)
torch.cuda.synchronize()
eager = (time.perf_counter() - t0) / N * 1e6
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    with torch.cuda.graph(g):
        for _ in range(N):
            x.add_(1)
torch.cuda.current_stream().wait_stream(s)
g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
graph = (time.perf_counter() - t0) / (5 * N) * 1e6
big = torch.zeros(64 * 1024 * 1024 // 4, device='cuda')
for _ in range(3):
    big.add_(1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    big.add_(1)
torch.cuda.synchronize()
bw = 2 * big.numel() * 4 * 20 / (time.perf_counter() - t0) / 1e9
print(f'per-kernel: eager {eager:.2f} us, graph replay {graph:.2f} us; 64MB add_ {bw:.0f} GB/s')

# the same with a umamd kernel (um_axpy over 1 element) to compare the floor
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'uncertainty-model_amd'))
from umamd._lib import call, ptr  # noqa: E402

y = torch.zeros(1, device='cuda')
for _ in range(3):
    call('um_axpy', 0, 1, 1.0, ptr(x), ptr(y))
g2 = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    with torch.cuda.graph(g2):
        for _ in range(N):
            call('um_axpy', 0, 1, 1.0, ptr(x), ptr(y))
torch.cuda.current_stream().wait_stream(s)
g2.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    g2.replay()
torch.cuda.synchronize()
print(f'umamd um_axpy(n=1) graph replay {(time.perf_counter() - t0) / (5 * N) * 1e6:.2f} us')
