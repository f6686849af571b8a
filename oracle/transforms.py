"""CPU restatement of the input pipeline's arithmetic -- TEST ORACLE.

Follows the reference's transforms (train/transforms.py:15-129): torchvision
Resize on PIL images is Pillow's ``Image.resize((w, h), BILINEAR)``, a
third-party dependency absent from /root/reference (Pillow 12.2.0 is
installed here and is itself the pin: tests/test_imageprep_cpu.py checks this
restatement against PIL bit for bit).  Pillow's published algorithm
(libImaging/Resample.c): per axis, a triangle filter of support
max(in/out, 1), taps [xmin, xmin + n) around center = (x + 0.5) * in/out,
weights normalised to sum 1 and rounded to 22-bit fixed point; the
horizontal pass first into an 8-bit image (sum + 2^21, >> 22, clip), then the
vertical pass.  Then ToTensor (/255), flip, gamma/brightness/colour, clamp.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def pil_coeffs(n_in: int, n_out: int):
    scale = n_in / n_out
    fs = max(scale, 1.0)
    support = fs
    out = []
    for x in range(n_out):
        c = (x + 0.5) * scale
        lo = max(int(c - support + 0.5), 0)
        hi = min(int(c + support + 0.5), n_in)
        w = [max(0.0, 1.0 - abs((i - c + 0.5) / fs)) for i in range(lo, hi)]
        s = sum(w)
        w = [v / s for v in w] if s else w
        q = [int(math.floor(v * (1 << 22) + 0.5)) if v >= 0 else
             -int(math.floor(-v * (1 << 22) + 0.5)) for v in w]
        out.append((lo, q))
    return out


def _pass(a: np.ndarray, coeffs, axis: int) -> np.ndarray:
    a = np.moveaxis(a.astype(np.int64), axis, 0)
    res = np.empty((len(coeffs),) + a.shape[1:], np.int64)
    for i, (lo, q) in enumerate(coeffs):
        acc = np.full(a.shape[1:], 1 << 21, np.int64)
        for j, w in enumerate(q):
            acc += a[lo + j] * w
        res[i] = np.clip(acc >> 22, 0, 255)
    return np.moveaxis(res, 0, axis).astype(np.uint8)


def pil_resize(img: np.ndarray, h: int, w: int) -> np.ndarray:
    """uint8 HWC -> uint8 [h, w, C] (PIL Image.resize((w, h), BILINEAR))"""
    if img.shape[:2] == (h, w):
        return img.copy()
    a = img
    if a.shape[1] != w:
        a = _pass(a, pil_coeffs(a.shape[1], w), 1)
    if a.shape[0] != h:
        a = _pass(a, pil_coeffs(a.shape[0], h), 0)
    return a


def prep_pair(left: np.ndarray, right: np.ndarray, prep, h: int, w: int):
    """one sample: the reference's ResizeImage -> RandomFlip -> ToTensor ->
    RandomAugment with the decisions/values in ``prep`` (flip, augment,
    gamma, brightness, colour[3]) -> (left, right) f32 [3, h, w]"""
    out = []
    for img in (left, right):
        r = pil_resize(img, h, w)
        if prep[0]:
            r = r[:, ::-1]
        t = torch.from_numpy(np.ascontiguousarray(r)).permute(2, 0, 1).float().div(255)
        if prep[1]:
            t = t ** float(prep[2])
            t = t * float(prep[3])
            t = t * torch.tensor(np.asarray(prep[4:7], np.float32)).view(3, 1, 1)
            t = torch.clamp(t, 0, 1)
        out.append(t)
    return out
