"""Loss-stack autograd functions over the umamd C ABI.

  * ``scale_pyramid``       reference train/utils.py:27-50, every level in one launch
  * ``reconstruct``         reference train/utils.py:65-97 (+ _left/_right 100-109)
  * ``reconstruct_pyramid`` reference train/utils.py:112-135, one launch
  * ``tukra_loss``          reference train/loss.py:512-568 with the sub-losses
                            of loss.py:15-264,340-434: ONE forward launch over
                            every scale (the six terms, finished on the device)
                            and ONE backward launch producing the gradient
                            w.r.t. all four prediction channels of every scale,
                            including the WSSIM term's path through the warp.
  * ``image_error``         WeightedSSIMLoss.image_error (loss.py:96-131) of an
                            explicit recon (evaluation)

Images are NCHW f32; predictions are the model's disparity tensors (logical
[N,4,h,w], stored channels-last).  The fused loss re-derives the recon from
the pyramid and the predictions inside its kernels, so the recon tensors it is
given must be exactly ``reconstruct_pyramid(predictions, pyramid)`` -- which
is what train/train.py passes (reference train.py:122-124); they are tagged
and checked.  The recon tensors are still real (``reconstruct_pyramid`` runs
its own launch, or -- under ``deferred_recon`` -- the loss forward writes them)
and differentiable w.r.t. the disparities (adversarial terms).
"""
from __future__ import annotations

import contextlib
import ctypes
from typing import List, Sequence

import torch

from . import _lib as L
from ._lib import call, ptr, query

LOSS_TYPES = {'l1': 0, 'bayesian': 1, 'log_bayesian': 2}
MAX_LEVELS = 6

_defer = [False]
@contextlib.contextmanager
def deferred_recon():
    """Inside this context ``reconstruct_pyramid`` only allocates its outputs
    and marks them pending; the fused loss forward that follows fills them
    as a side output of the kernel that derives the reconstruction anyway
    (saving the separate recon launch).  Only for step bodies where the loss
    directly consumes the recon (train.train.train_step, the captured step):
    a pending recon holds no values until that loss forward has run."""
    old = _defer[0]
    _defer[0] = True
    try:
        yield
    finally:
        _defer[0] = old


def _f32c(t: torch.Tensor) -> torch.Tensor:
    t = t.detach()
    if t.dtype != torch.float32 or not t.is_contiguous():
        t = t.float().contiguous()
    return t


def _parr(ts) -> ctypes.Array:
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


def scale_pyramid(x: torch.Tensor, scales: int) -> List[torch.Tensor]:
    L.require_device(x)
    if not 1 <= scales <= MAX_LEVELS:
        raise L.UmamdError(f'scale_pyramid: {scales} scales (1..{MAX_LEVELS})')
    xc = _f32c(x)
    N, C, H, W = xc.shape
    out = [torch.empty((N, C, H >> i, W >> i), dtype=torch.float32, device=x.device)
           for i in range(scales)]
    call('um_pyramid', ptr(xc), N * C, H, W, scales, _parr(out))
    return out


def _pred_nhwc(p: torch.Tensor) -> torch.Tensor:
    """Logical [N,C,h,w] -> NHWC memory view [N,h,w,C] (copy if needed)."""
    v = p.permute(0, 2, 3, 1)
    if v.dtype != torch.float32 or not v.is_contiguous():
        v = v.float().contiguous()
    return v


def _disp_strides(d: torch.Tensor):
    """(tensor, image stride, pixel stride) such that element (n, 0, y, x) of
    the [N,1,H,W] view is at data_ptr + n*sn + (y*W + x)*sp (NCHW planes and
    NHWC channel slices both qualify)."""
    W = d.shape[-1]
    sn, _, sy, sx = d.stride()
    if sy != W * sx:
        d = d.contiguous()
        sn, _, sy, sx = d.stride()
    return d, sn, sx


class _WarpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, disp, img, sign: float):
        L.require_device(img)
        imgc = _f32c(img)
        N, C, H, W = imgc.shape
        d = disp.detach()
        if d.dtype != torch.float32:
            d = d.float()
        d, sn, sp = _disp_strides(d)
        out = torch.empty((N, C, H, W), dtype=torch.float32, device=img.device)
        call('um_warp', ptr(imgc), N, C, H, W, d.data_ptr(), sn, sp, float(sign), ptr(out))
        ctx.sign = float(sign)
        ctx.save_for_backward(d, imgc)
        ctx.dshape = disp.shape
        ctx.ddtype = disp.dtype
        return out

    @staticmethod
    def backward(ctx, g):
        if ctx.needs_input_grad[1]:
            raise NotImplementedError('umamd reconstruct(): gradient w.r.t. the image (a data '
                                      'tensor in every reference call site) is not implemented')
        d, imgc = ctx.saved_tensors
        N, C, H, W = imgc.shape
        gd = torch.empty((N, 1, H, W), dtype=torch.float32, device=g.device)
        _, sn, sp = _disp_strides(d)
        gc = _f32c(g)  # keep alive until the launch is queued (no temporaries by pointer)
        call('um_warp_bwd', ptr(imgc), N, C, H, W, d.data_ptr(), sn, sp, ctx.sign,
             ptr(gc), ptr(gd), H * W, 1)
        return gd.to(ctx.ddtype).reshape(ctx.dshape), None, None


def reconstruct(disparity: torch.Tensor, opposite_image: torch.Tensor, sign: float = 1.0):
    return _WarpFn.apply(disparity, opposite_image, sign)


class _ReconPyramidFn(torch.autograd.Function):
    """Every level of reconstruct_pyramid in one launch; backward = the warp
    adjoint w.r.t. d_L (channel 0) and d_R (channel 1)."""

    @staticmethod
    def forward(ctx, n, defer, *tensors):
        disps, pyr = tensors[:n], [_f32c(t) for t in tensors[n:]]
        N, _, H, W = pyr[0].shape
        dev = pyr[0].device
        ds, strides = [], []
        for i, d in enumerate(disps):
            if d.shape[0] != N or d.shape[2:] != (H >> i, W >> i) or d.shape[1] < 2:
                raise L.UmamdError(f'reconstruct_pyramid: level {i} disparity {tuple(d.shape)} '
                                   f'vs pyramid {tuple(pyr[i].shape)}')
            dd = d.detach()
            if dd.dtype != torch.float32:
                dd = dd.float()
            dd, sn, sp = _disp_strides(dd)
            ds.append(dd)
            strides += [sn, dd.stride(1), sp]
        out = [torch.empty((N, 6, H >> i, W >> i), dtype=torch.float32, device=dev)
               for i in range(n)]
        if not defer:
            sarr = (ctypes.c_long * len(strides))(*strides)
            call('um_recon_pyramid', n, N, H, W, _parr(pyr), _parr(ds), sarr, _parr(out))
        ctx.n = n
        ctx.meta = [(d.shape, d.dtype) for d in disps]
        ctx.save_for_backward(*ds, *pyr)
        return tuple(out)

    @staticmethod
    def backward(ctx, *gouts):
        n = ctx.n
        sv = ctx.saved_tensors
        ds, pyr = sv[:n], sv[n:]
        grads = []
        for i in range(n):
            g = gouts[i]
            shape, dtype = ctx.meta[i]
            if g is None or not ctx.needs_input_grad[2 + i]:
                grads.append(None)
                continue
            g = _f32c(g)
            N, _, h, w = pyr[i].shape
            gd = torch.zeros((N, h, w, shape[1]), dtype=torch.float32, device=g.device)
            _, sn, sp = _disp_strides(ds[i])
            cs = ds[i].stride(1)
            # left recon = warp(right image, -d_L); right recon = warp(left image, +d_R)
            for v, (img, gsl, sign) in enumerate(((pyr[i][:, 3:6], g[:, 0:3], -1.0),
                                                  (pyr[i][:, 0:3], g[:, 3:6], 1.0))):
                # bind the contiguous copies: a temporary passed only by pointer
                # could be freed (and its memory reused) before the launch runs
                imgc, gc = img.contiguous(), gsl.contiguous()
                call('um_warp_bwd', ptr(imgc), N, 3, h, w,
                     ds[i].data_ptr() + v * cs * 4, sn, sp, sign, ptr(gc),
                     gd.data_ptr() + v * 4, h * w * shape[1], shape[1])
            grads.append(gd.permute(0, 3, 1, 2).to(dtype))
        return (None, None, *grads, *([None] * n))


def reconstruct_pyramid(disparities: Sequence[torch.Tensor],
                        pyramid: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    n = min(len(disparities), len(pyramid))
    if not 1 <= n <= MAX_LEVELS:
        raise L.UmamdError(f'reconstruct_pyramid: {n} levels (1..{MAX_LEVELS})')
    L.require_device(pyramid[0])
    defer = _defer[0]
    out = list(_ReconPyramidFn.apply(n, defer, *disparities[:n],
                                     *[p.detach() for p in pyramid[:n]]))
    for d, im, r in zip(disparities, pyramid, out):
        r._umamd_recon = (id(d), id(im))
        r._umamd_pending = defer
    return out


def _check_levels(preds, pyr):
    N, _, H, W = pyr[0].shape
    for i, (p, im) in enumerate(zip(preds, pyr)):
        want = (N, H >> i, W >> i)
        if tuple(im.shape) != (N, 6, H >> i, W >> i) or \
                (p.shape[0], p.shape[1], p.shape[2]) != want or p.shape[3] != 4:
            raise L.UmamdError(f'tukra_loss: level {i}: pyramid {tuple(im.shape)}, prediction '
                               f'(NHWC) {tuple(p.shape)}; expected [N,6,H>>i,W>>i] / [N,4,...]')
    return N, H, W


class TukraLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, n, recon_out, grad, *tensors):
        preds = [_pred_nhwc(t) for t in tensors[:n]]
        pyr = [_f32c(t) for t in tensors[n:2 * n]]
        N, H, W = _check_levels(preds, pyr)
        rarr = None
        if recon_out is not None:
            for i, r in enumerate(recon_out):
                if r.shape != pyr[i].shape or r.dtype != torch.float32 or not r.is_contiguous():
                    raise L.UmamdError('tukra_loss: recon_out must be the [N,6,h,w] f32 '
                                       'contiguous reconstruct_pyramid outputs')
            rarr = _parr(recon_out)
        dev = preds[0].device
        ws = torch.empty((max(query('um_loss_ws', n, N, H, W), 8) // 8,), dtype=torch.float64,
                         device=dev)
        emap = torch.empty((N, 2, H >> (n - 1), W >> (n - 1)), dtype=torch.float32, device=dev)
        out = torch.empty(6, dtype=torch.float32, device=dev)
        dl = torch.empty((), dtype=torch.float32, device=dev)
        el = torch.empty_like(dl)

        # a step that will differentiate the loss gets the gradient partials
        # from the same tile pass (um_loss_fwd gpart); backward = the scatter
        gpart = None
        if grad:
            gpart = [torch.empty((N, H >> i, W >> i, 4), dtype=torch.float32, device=dev)
                     for i in range(n)]
        call('um_loss_fwd', n, N, H, W, _parr(pyr), _parr(preds), cfg['alpha'],
             cfg['loss_type'], cfg['esw'], cfg['ecw'], cfg['w_wssim'], cfg['w_cons'],
             cfg['w_smooth'], cfg['w_err'], ptr(ws), ptr(emap), rarr, ptr(out), ptr(dl),
             ptr(el), _parr(gpart) if gpart is not None else None)
        ctx.cfg = cfg
        ctx.n = n
        ctx.geom = (N, H, W)
        ctx.gpart = gpart
        ctx.save_for_backward(*preds, *pyr)
        ctx.mark_non_differentiable(out, emap)
        return dl, el, out, emap

    @staticmethod
    def backward(ctx, gd, ge, *unused):
        cfg, n = ctx.cfg, ctx.n
        N, H, W = ctx.geom
        sv = ctx.saved_tensors
        preds, pyr = sv[:n], sv[n:2 * n]
        dev = preds[0].device
        # the two upstream gradients stay device scalars (None = 0): no stack
        gd = gd.float().contiguous() if gd is not None else None
        ge = ge.float().contiguous() if ge is not None else None
        grads = [torch.empty((N, H >> i, W >> i, 4), dtype=torch.float32, device=dev)
                 for i in range(n)]
        gpart, ctx.gpart = ctx.gpart, None
        call('um_loss_bwd', n, N, H, W, _parr(pyr), _parr(preds), cfg['alpha'],
             cfg['loss_type'], cfg['esw'], cfg['ecw'], cfg['w_wssim'], cfg['w_cons'],
             cfg['w_smooth'], cfg['w_err'], ptr(gd) if gd is not None else None,
             ptr(ge) if ge is not None else None,
             _parr(gpart) if gpart is not None else None, _parr(grads))
        return (None, None, None, None, *[g.permute(0, 3, 1, 2) for g in grads],
                *([None] * n))


def tukra_loss(cfg: dict, preds, pyramid, recon_out=None):
    """Returns (disp_loss, error_loss, terms[6], last-scale error map).  The
    backward differentiates through the warp itself (the recon is re-derived).
    ``recon_out``: pending reconstruct_pyramid outputs to fill (deferred_recon)."""
    n = len(preds)
    if not 1 <= n <= MAX_LEVELS:
        raise L.UmamdError(f'tukra_loss: {n} scales (1..{MAX_LEVELS})')
    # the gradient partials are computed with the forward when it will be differentiated
    grad = torch.is_grad_enabled() and any(p.requires_grad for p in preds)
    out = TukraLossFn.apply(cfg, n, recon_out, grad, *preds, *[p.detach() for p in pyramid])
    if recon_out is not None:
        for r in recon_out:
            r._umamd_pending = False
    return out


def image_error(images: torch.Tensor, recon: torch.Tensor, alpha: float) -> torch.Tensor:
    L.require_device(images)
    img, rec = _f32c(images), _f32c(recon)
    N, C, H, W = img.shape
    if C != 6 or rec.shape != img.shape:
        raise L.UmamdError(f'image_error: images {tuple(img.shape)} / recon {tuple(rec.shape)}')
    out = torch.empty((N, 2, H, W), dtype=torch.float32, device=img.device)
    call('um_image_error', ptr(img), ptr(rec), N, H, W, float(alpha), ptr(out))
    return out
