"""Loss-stack autograd functions over the umamd C ABI.

  * ``scale_pyramid``       reference train/utils.py:27-50
  * ``reconstruct``         reference train/utils.py:65-97 (+ _left/_right 100-109)
  * ``reconstruct_pyramid`` reference train/utils.py:112-135
  * ``tukra_loss``          reference train/loss.py:512-568 with the sub-losses
                            of loss.py:15-264,340-434, fused per scale into a
                            forward kernel pair (DSSIM map + per-pixel terms)
                            and one backward kernel that produces the gradient
                            w.r.t. all four prediction channels, including the
                            WSSIM term's path through the bilinear warp.

Images are NCHW f32; predictions are the model's disparity tensors (logical
[N,4,h,w], stored channels-last).  Recon tensors are produced by
``reconstruct_pyramid`` and tagged; the fused loss needs them to be exactly
warp(pred, pyramid) -- which is what train/train.py passes (train.py:122-124).
"""
from __future__ import annotations

from typing import List, Sequence

import torch

from . import _lib as L
from ._lib import call, ptr, query

LOSS_TYPES = {'l1': 0, 'bayesian': 1, 'log_bayesian': 2}


def _f32c(t: torch.Tensor) -> torch.Tensor:
    t = t.detach()
    if t.dtype != torch.float32 or not t.is_contiguous():
        t = t.float().contiguous()
    return t


def scale_pyramid(x: torch.Tensor, scales: int) -> List[torch.Tensor]:
    L.require_device(x)
    xc = _f32c(x)
    N, C, H, W = xc.shape
    out = []
    for i in range(scales):
        h, w = H // 2 ** i, W // 2 ** i
        o = torch.empty((N, C, h, w), dtype=torch.float32, device=x.device)
        call('um_pyramid_level', ptr(xc), N * C, H, W, ptr(o), h, w)
        out.append(o)
    return out


def _pred_nhwc(p: torch.Tensor) -> torch.Tensor:
    """Logical [N,C,h,w] -> NHWC memory view [N,h,w,C] (copy if needed)."""
    v = p.permute(0, 2, 3, 1)
    if v.dtype != torch.float32 or not v.is_contiguous():
        v = v.float().contiguous()
    return v


class _WarpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, disp, img, sign: float):
        L.require_device(img)
        ctx.set_materialize_grads(False)
        imgc = _f32c(img)
        N, C, H, W = imgc.shape
        d = disp.detach()
        if d.dtype != torch.float32:
            d = d.float()
        # element (n, 0, y, x) at d.data_ptr + n*sn + (y*W + x)*sp requires
        # uniform pixel stride: true for NCHW planes and NHWC channel slices
        sn, sc, sy, sx = d.stride()
        if sy != W * sx:
            d = d.contiguous()
            sn, sc, sy, sx = d.stride()
        out = torch.empty((N, C, H, W), dtype=torch.float32, device=img.device)
        call('um_warp', ptr(imgc), N, C, H, W, d.data_ptr(), sn, sx, float(sign), ptr(out))
        return out

    @staticmethod
    def backward(ctx, g):
        if g is None:
            return None, None, None
        raise NotImplementedError(
            'gradient through reconstruct() is provided by TukraUncertaintyLoss directly '
            '(fused); a standalone warp backward (adversarial path) is not implemented yet')


def reconstruct(disparity: torch.Tensor, opposite_image: torch.Tensor, sign: float = 1.0):
    return _WarpFn.apply(disparity, opposite_image, sign)


def reconstruct_pyramid(disparities: Sequence[torch.Tensor],
                        pyramid: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    out = []
    for d, im in zip(disparities, pyramid):
        # left recon = warp(right image, -d_L); right recon = warp(left image, d_R)
        lr = reconstruct(d[:, 0:1], im[:, 3:6], -1.0)
        rr = reconstruct(d[:, 1:2], im[:, 0:3], 1.0)
        r = torch.cat([lr, rr], 1)
        r._umamd_recon = (id(d), id(im))
        out.append(r)
    return out


class TukraLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, n, *tensors):
        preds = [_pred_nhwc(t) for t in tensors[:n]]
        pyr = [_f32c(t) for t in tensors[n:2 * n]]
        rec = [_f32c(t) for t in tensors[2 * n:3 * n]]
        dev = preds[0].device
        parts, nparts, npix, emaps = [], [], [], []
        for i in range(n):
            N, H, W, pld = preds[i].shape
            D = torch.empty((N, 2, H - 2, W - 2), dtype=torch.float32, device=dev)
            e = torch.empty((N, 2, H, W), dtype=torch.float32, device=dev)
            np_ = query('um_loss_parts', N, H, W)
            pt = torch.empty((np_, 8), dtype=torch.float32, device=dev)
            call('um_loss_fwd_scale', ptr(pyr[i]), ptr(rec[i]), ptr(preds[i]), pld, N, H, W,
                 cfg['alpha'], cfg['loss_type'], cfg['esw'], cfg['ecw'], ptr(D), ptr(e), ptr(pt))
            parts.append(pt)
            nparts.append(np_)
            npix.append(float(N * H * W))
            emaps.append(e)
        out = torch.empty(6, dtype=torch.float32, device=dev)
        import ctypes
        parr = (ctypes.c_void_p * n)(*[p.data_ptr() for p in parts])
        narr = (ctypes.c_int * n)(*nparts)
        darr = (ctypes.c_double * n)(*npix)
        call('um_loss_finalize', n, parr, narr, darr, cfg['w_wssim'], cfg['w_cons'],
             cfg['w_smooth'], cfg['w_err'], cfg['esw'], cfg['ecw'], cfg['loss_type'], ptr(out))
        ctx.cfg = cfg
        ctx.n = n
        ctx.save_for_backward(*preds, *pyr, *rec, *emaps)
        ctx.shapes = [t.shape for t in tensors[:n]]
        dl = out[0].clone()
        el = out[1].clone()
        ctx.mark_non_differentiable(out)
        for e in emaps:
            ctx.mark_non_differentiable(e)
        return (dl, el, out, *emaps)

    @staticmethod
    def backward(ctx, gd, ge, *unused):
        cfg, n = ctx.cfg, ctx.n
        sv = ctx.saved_tensors
        preds, pyr, rec, emaps = sv[:n], sv[n:2 * n], sv[2 * n:3 * n], sv[3 * n:]
        dev = preds[0].device
        gout = torch.stack([gd.reshape(()).float(), ge.reshape(()).float()]).contiguous()
        grads = []
        for i in range(n):
            N, H, W, pld = preds[i].shape
            # the kernel stores channels 0-3 of every pixel; only padding needs zeros
            dp = (torch.empty if pld == 4 else torch.zeros)((N, H, W, pld), dtype=torch.float32,
                                                             device=dev)
            call('um_loss_bwd_scale', ptr(pyr[i]), ptr(rec[i]), ptr(preds[i]), pld, N, H, W,
                 cfg['alpha'], cfg['loss_type'], cfg['esw'], cfg['ecw'], ptr(emaps[i]),
                 ptr(gout), cfg['w_wssim'], cfg['w_cons'], cfg['w_smooth'], cfg['w_err'],
                 float(2 ** i), ptr(dp))
            grads.append(dp.permute(0, 3, 1, 2))  # logical NCHW, NHWC memory
        return (None, None, *grads, *([None] * (2 * n)))


def tukra_loss(cfg: dict, preds, pyramid, recon):
    """The fused backward differentiates through the warp itself, so the
    recon tensors enter as plain (detached) data."""
    n = len(preds)
    return TukraLossFn.apply(cfg, n, *preds, *[p.detach() for p in pyramid],
                             *[r.detach() for r in recon])
