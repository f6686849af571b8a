"""Evaluation metrics over the umamd C ABI (reference train/evaluate.py:66-196,
train/sparsification.py:8-61).  No CPU path: every op calls the HIP library.

  * ``ssim``            torchmetrics.functional.structural_similarity_index_measure
                        as the reference calls it (gaussian window sigma 1.5
                        -> 11 taps, data_range, k1 0.01, k2 0.03); reductions
                        'sum' / 'elementwise_mean' / 'none' over the batch
  * ``avg_pool_valid``  nn.AvgPool2d(k, stride=1)
  * ``sparsification_curve``  argsort(pred, descending) + gather(oracle) per
                        (image, view), then the 100-step curve
"""
from __future__ import annotations

import torch

from . import _lib as L
from ._lib import call, ptr, query


def _f32c(t):
    t = t.detach()
    if t.dtype != torch.float32 or not t.is_contiguous():
        t = t.float().contiguous()
    return t


def ssim(preds, target, kernel_size: int = 11, sigma: float = 1.5, reduction='elementwise_mean',
         data_range: float = 1.0):
    L.require_device(preds)
    x, y = _f32c(preds), _f32c(target)
    if x.shape != y.shape or x.dim() != 4:
        raise L.UmamdError(f'ssim: preds {tuple(x.shape)} / target {tuple(y.shape)}')
    N, C, H, W = x.shape
    ws = torch.empty((max(query('um_ssim_ws', N, H, W), 8) // 8,), dtype=torch.float64,
                     device=x.device)
    per = torch.empty((N,), dtype=torch.float32, device=x.device)
    call('um_ssim_gauss', ptr(x), ptr(y), N, C, H, W, float(data_range), float(sigma), ptr(ws),
         ptr(per))
    if reduction == 'sum':
        return per.sum()
    if reduction in ('elementwise_mean', 'mean'):
        return per.mean()
    return per


def avg_pool_valid(x, k: int):
    L.require_device(x)
    xc = _f32c(x)
    N, C, H, W = xc.shape
    out = torch.empty((N, C, H - k + 1, W - k + 1), dtype=torch.float32, device=x.device)
    call('um_avgpool_valid', ptr(xc), N * C, H, W, k, ptr(out))
    return out


def sparsification_curve(oracle_error, predicted_error, kernel_size: int = 11, steps: int = 100):
    """Reference sparsification.curve (:8-36): [B,2,H,W] maps -> curve[steps]."""
    L.require_device(oracle_error)
    b = predicted_error.shape[0]
    o = avg_pool_valid(oracle_error, kernel_size).reshape(b * 2, -1)
    p = avg_pool_valid(predicted_error, kernel_size).reshape(b * 2, -1)
    nseg, n = o.shape
    keys_out = torch.empty_like(p)
    vals_out = torch.empty_like(o)
    wsb = query('um_spars_sort_ws', nseg, n)
    ws = torch.empty((wsb,), dtype=torch.uint8, device=o.device)
    call('um_spars_sort', ptr(p), ptr(o), nseg, n, ptr(keys_out), ptr(vals_out), ptr(ws), wsb)
    norm = torch.empty((nseg, steps), dtype=torch.float64, device=o.device)
    curve = torch.empty((steps,), dtype=torch.float32, device=o.device)
    call('um_spars_curve', ptr(vals_out), nseg, n, steps, ptr(norm), ptr(curve))
    return curve
