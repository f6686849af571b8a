"""Autograd functions of the adversarial path over the umamd C ABI
(reference model/discriminator.py:53-86, train/loss.py:267-337).

  * ``image_to_nhwc``  NCHW f32 -> NHWC compute dtype WITH a gradient (the
                       discriminator sees the recon pyramid, whose gradient
                       flows back to the disparities through the warp)
  * ``disc_head``      sigmoid(Linear(flatten(x))) on the last NHWC feature map
  * ``l1_mean``        mean |a - b| of two NHWC feature maps (PerceptualLoss)
"""
from __future__ import annotations

import torch

from . import _lib as L
from . import functional as U
from ._lib import call, ptr, query


class ImageToNHWCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, dtype):
        out = U.image_to_nhwc(img, dtype)
        ctx.shape = img.shape
        ctx.in_dtype = img.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        N, C, H, W = ctx.shape
        gc = g.contiguous()
        out = torch.empty((N, C, H, W), dtype=torch.float32, device=g.device)
        call('um_nhwc_to_image', L.dtype_code(gc.dtype), ptr(gc), N, C, H, W, gc.shape[-1],
             ptr(out))
        return out.to(ctx.in_dtype), None


def image_to_nhwc(img: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    if not img.requires_grad:
        return U.image_to_nhwc(img, dtype)
    return ImageToNHWCFn.apply(img, dtype)


class DiscHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        L.require_device(x)
        N, H, W, C = x.shape
        if weight.numel() != H * W * C:
            raise L.UmamdError(f'disc_head: Linear in_features {weight.numel()} != flattened '
                               f'feature {C}x{H}x{W}')
        xc = x.contiguous()
        w = weight.detach().float().contiguous()
        b = bias.detach().float().contiguous()
        prob = torch.empty((N, 1), dtype=torch.float32, device=x.device)
        call('um_disc_head_fwd', L.dtype_code(xc.dtype), ptr(xc), N, H * W, C, ptr(w), ptr(b),
             ptr(prob))
        ctx.save_for_backward(xc, w, prob)
        return prob

    @staticmethod
    def backward(ctx, dprob):
        xc, w, prob = ctx.saved_tensors
        N, H, W, C = xc.shape
        dp = dprob.float().contiguous()
        dx = torch.empty_like(xc) if ctx.needs_input_grad[0] else None
        dw = torch.empty((1, H * W * C), dtype=torch.float32, device=xc.device)
        db = torch.empty((1,), dtype=torch.float32, device=xc.device)
        call('um_disc_head_bwd', L.dtype_code(xc.dtype), ptr(xc), N, H * W, C, ptr(w), ptr(prob),
             ptr(dp), ptr(dx), ptr(dw), ptr(db))
        return dx, dw, db


def disc_head(x: torch.Tensor, linear: torch.nn.Linear) -> torch.Tensor:
    return DiscHeadFn.apply(x, linear.weight, linear.bias)


class L1MeanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        L.require_device(a)
        if a.shape != b.shape or a.dtype != b.dtype:
            raise L.UmamdError(f'l1_mean: {tuple(a.shape)}/{a.dtype} vs {tuple(b.shape)}/{b.dtype}')
        ac, bc = a.contiguous(), b.contiguous()
        ws = torch.empty((query('um_l1_mean_ws') // 8,), dtype=torch.float64, device=a.device)
        out = torch.empty((), dtype=torch.float32, device=a.device)
        call('um_l1_mean', L.dtype_code(ac.dtype), ptr(ac), ptr(bc), ac.numel(), ptr(ws), ptr(out))
        ctx.save_for_backward(ac, bc)
        return out

    @staticmethod
    def backward(ctx, g):
        ac, bc = ctx.saved_tensors
        gc = g.float().reshape(1).contiguous()
        da = torch.empty_like(ac) if ctx.needs_input_grad[0] else None
        db = torch.empty_like(bc) if ctx.needs_input_grad[1] else None
        call('um_l1_mean_bwd', L.dtype_code(ac.dtype), ptr(ac), ptr(bc), ac.numel(), ptr(gc),
             ptr(da), ptr(db))
        return da, db


def l1_mean(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return L1MeanFn.apply(a, b)
