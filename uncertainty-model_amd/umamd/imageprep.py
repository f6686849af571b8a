"""The reference's training transforms on the device (C ABI um_stereo_prep).

Reference pipeline (main.py:78-89, parallel_main.py:111-124):

    Compose([ResizeImage((256, 512)), RandomFlip(0.5), ToTensor(),
             RandomAugment(0.5, gamma=(0.8, 1.2), brightness=(0.5, 2.0),
                           colour=(0.8, 1.2))])

applied per sample in DataLoader workers (PIL resize, numpy draws, torch CPU
arithmetic).  Here the workers only decode to uint8 and take the random
draws -- with ``numpy.random`` in the reference's order, so a seeded worker
makes the reference's decisions -- and one batched HIP pass does resize,
ToTensor, flip and augment for both views (csrc/imageprep.hip):

  * ``resize_coeffs``: Pillow's bilinear resampling coefficients
    (libImaging/Resample.c precompute_coeffs + normalize_coeffs_8bpc,
    Pillow 12.2 as installed: triangle filter of support 1 scaled by the
    downscale factor, per-pixel normalisation, 22-bit fixed point), cached
    per (source, target) size and uploaded once;
  * ``StereoDraws``: the worker-side transform, returning
    ``{'left': uint8 HWC, 'right': uint8 HWC, 'prep': float32[8]}``
    (flip, augment, gamma, brightness, colour[3], 0);
  * ``stereo_prep``: the device pass, a batch of those -> {'left', 'right'}
    f32 [N, 3, H, W] on the device, what the reference's loader yields.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import numpy as np
import torch
from numpy import random

from . import _lib as L

PRECISION_BITS = 22  # Pillow: 32 - 8 - 2


def _bilinear(x: float) -> float:
    x = abs(x)
    return 1.0 - x if x < 1.0 else 0.0


def resize_coeffs(in_size: int, out_size: int) -> Tuple[np.ndarray, np.ndarray, int]:
    """Pillow's precompute_coeffs (box = the whole axis) for the bilinear
    filter and normalize_coeffs_8bpc -> (bounds int32 [out, 2] = (first
    source index, tap count), kk int32 [out, ksize], ksize)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.int32)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)  # C (int) truncates toward 0, as int()
        xmax = min(int(center + support + 0.5), in_size) - xmin
        k = [_bilinear((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = sum(k)
        if ww != 0.0:
            k = [w / ww for w in k]
        for x, w in enumerate(k):
            kk[xx, x] = int(-0.5 + w * (1 << PRECISION_BITS)) if w < 0 else \
                int(0.5 + w * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, kk, ksize


_COEFFS: Dict[tuple, tuple] = {}


def _device_coeffs(hs, ws, hd, wd, device):
    key = (hs, ws, hd, wd, str(device))
    c = _COEFFS.get(key)
    if c is None:
        bh, kh, ksh = resize_coeffs(ws, wd)
        bv, kv, ksv = resize_coeffs(hs, hd)
        c = tuple(torch.from_numpy(a).to(device) for a in (bh, kh, bv, kv)) + (ksh, ksv)
        _COEFFS[key] = c
    return c


class StereoDraws:
    """Worker-side half of the reference's augmenting pipeline: takes the
    decoded PIL / uint8 pair and the numpy draws of RandomFlip (:56) and
    RandomAugment (:120-124) in the reference's order; the arithmetic is
    deferred to ``stereo_prep``.  ``augment=False`` is the no-augment
    pipeline (ResizeImage + ToTensor only, main.py:91-93): no draws."""

    def __init__(self, flip_p: float = 0.5, augment_p: float = 0.5,
                 gamma=(0.8, 1.2), brightness=(0.5, 2.0), colour=(0.8, 1.2),
                 augment: bool = True, size=(256, 512)) -> None:
        self.size = (int(size[0]), int(size[1]))
        self.flip_p, self.augment_p = flip_p, augment_p
        self.gamma, self.brightness, self.colour = gamma, brightness, colour
        self.augment = augment

    @staticmethod
    def _u8(x) -> torch.Tensor:
        a = np.asarray(x)
        if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 3:
            raise TypeError(f'StereoDraws: RGB uint8 HWC image expected, got {a.dtype} '
                            f'{a.shape}')
        if not a.flags.writeable or not a.flags.c_contiguous:
            a = np.array(a, copy=True, order='C')  # np.asarray(PIL image) is read-only
        return torch.from_numpy(a)

    def __call__(self, image_pair):
        prep = np.zeros(8, np.float32)
        prep[2:7] = 1.0
        if self.augment:
            if random.random() < self.flip_p:            # RandomFlip.__call__
                prep[0] = 1.0
            if random.random() < self.augment_p:         # RandomAugment.__call__
                prep[1] = 1.0
                prep[2] = random.uniform(*self.gamma)
                prep[3] = random.uniform(*self.brightness)
                prep[4:7] = random.uniform(*self.colour, 3)
        return {'left': self._u8(image_pair['left']), 'right': self._u8(image_pair['right']),
                'prep': torch.from_numpy(prep), 'size': torch.tensor(self.size)}


def stereo_prep(batch, size=(256, 512), device=None) -> Dict[str, torch.Tensor]:
    """{'left', 'right': uint8 [N, Hs, Ws, 3], 'prep': f32 [N, 8]} (host or
    device) -> {'left', 'right': f32 [N, 3, H, W] on ``device``}: resize
    (Pillow bilinear, bit-exact), flip, ToTensor and augment in two launches."""
    left, right, prep = batch['left'], batch['right'], batch['prep']
    if device is None:
        device = torch.device('cuda', torch.cuda.current_device())
    if left.shape != right.shape or left.dim() != 4 or left.shape[-1] != 3:
        raise L.UmamdError(f'stereo_prep: left {tuple(left.shape)} / right '
                           f'{tuple(right.shape)}; expected equal [N, H, W, 3] uint8')
    if left.dtype != torch.uint8 or right.dtype != torch.uint8:
        raise L.UmamdError('stereo_prep: uint8 images expected')
    N, Hs, Ws, _ = left.shape
    Hd, Wd = int(size[0]), int(size[1])
    lg = left.to(device, non_blocking=True).contiguous()
    rg = right.to(device, non_blocking=True).contiguous()
    pg = prep.to(device, torch.float32, non_blocking=True).contiguous()
    if pg.shape != (N, 8):
        raise L.UmamdError(f'stereo_prep: prep {tuple(pg.shape)}, expected [{N}, 8]')
    L.require_device(lg)
    bh, kh, bv, kv, ksh, ksv = _device_coeffs(Hs, Ws, Hd, Wd, lg.device)
    tmp = torch.empty((L.query('um_stereo_prep_ws', N, Hs, Wd),), dtype=torch.uint8,
                      device=lg.device)
    out_l = torch.empty((N, 3, Hd, Wd), dtype=torch.float32, device=lg.device)
    out_r = torch.empty_like(out_l)
    L.call('um_stereo_prep', N, Hs, Ws, L.ptr(lg), L.ptr(rg), Hd, Wd, L.ptr(bh), L.ptr(kh), ksh,
           L.ptr(bv), L.ptr(kv), ksv, L.ptr(pg), L.ptr(tmp), L.ptr(out_l), L.ptr(out_r))
    return {'left': out_l, 'right': out_r}


def is_prep_batch(batch) -> bool:
    return isinstance(batch, dict) and 'prep' in batch


def to_device(batch, device, size: Optional[Tuple[int, int]] = None):
    """A loader batch -> (left, right) on ``device``: StereoDraws batches go
    through ``stereo_prep``; anything else is the reference's f32 batch."""
    if is_prep_batch(batch):
        if size is None:
            sz = batch.get('size')
            size = (256, 512) if sz is None else tuple(int(v) for v in sz.reshape(-1, 2)[0])
        out = stereo_prep(batch, size, device)
        return out['left'], out['right']
    return batch['left'].to(device), batch['right'].to(device)
