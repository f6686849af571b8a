"""Per-model cache of the packed conv weights, refreshed in ONE launch.

Every conv kernel reads its weight in a packed layout ([K][R][R][Cp] for the
forward / weight-gradient pass, [Cp][R][R][K] for the data gradient) in the
compute dtype, while the parameters stay NCHW f32 (the reference layout, so
state_dict, DDP and Adam are unchanged).  Instead of one repack launch per
conv per step (64 launches of 5-20 us at B=8 256x512), the model keeps the
packed buffers and refreshes all of them with a single ``um_pack_batch``
launch at the start of each forward.

The first forward records the pack sites (each one packed by its own
launch); later forwards launch the batch and the sites reuse the refreshed
buffers.  A site seen for the first time after that is packed individually
and marks the table for a rebuild at the next forward.  While a HIP graph is
being captured the table is never (re)built (that needs a host->device copy),
so a capture that starts before any eager forward simply packs per site.
"""
from __future__ import annotations

import ctypes
from contextlib import contextmanager
from typing import Optional

import torch

from . import _lib as L
from ._lib import call, ptr

MAXSEG = 4


class PackDesc(ctypes.Structure):
    """mirror of um_pack_desc (include/umamd.h)"""
    _fields_ = [('w', ctypes.c_void_p), ('wf', ctypes.c_void_p), ('wT', ctypes.c_void_p),
                ('K', ctypes.c_int), ('Creal', ctypes.c_int), ('R', ctypes.c_int),
                ('C', ctypes.c_int), ('ldT', ctypes.c_int), ('block0', ctypes.c_int),
                ('nseg', ctypes.c_int), ('src0', ctypes.c_int * MAXSEG),
                ('dst0', ctypes.c_int * MAXSEG), ('len', ctypes.c_int * MAXSEG),
                ('split', ctypes.c_int)]


def _tiles(K, C, R):
    return L.query('um_pack_tiles', K, C, R)


class WeightPacker:
    def __init__(self):
        self.entries = {}
        self.registered = set()
        self.descs = []       # (weight, wf_ptr, wT_ptr, K, Creal, R, C, ldT, segs, w_ptr, dtype)
        self.tables = {}      # dtype -> (table tensor, blk2desc tensor, ndesc, nblocks)
        self.dirty = True
        self.batched = False

    def __deepcopy__(self, memo):  # a copied model records its own sites
        return WeightPacker()

    def __getstate__(self):
        return {}

    def __setstate__(self, state):
        self.__init__()

    def reset(self):
        self.__init__()

    # -------------------------------------------------------------- refresh --
    def begin(self):
        """Called at the start of a forward: refresh every recorded site."""
        self.batched = False
        if not self.descs:
            return
        if any(d[0].data_ptr() != d[-2] for d in self.descs):
            # a parameter's storage moved (.to(), .data = ...): record again
            self.reset()
            return
        if self.dirty:
            if torch.cuda.is_current_stream_capturing():
                return
            self._build()
        for dt, (table, b2d, nd, nb) in self.tables.items():
            call('um_pack_batch', dt, ptr(table), nd, ptr(b2d), nb)
        self.batched = True

    def _build(self):
        by_dt = {}
        for d in self.descs:
            by_dt.setdefault(d[-1], []).append(d[:-2] + (d[-1],))
        self.tables = {}
        for dt, ds in by_dt.items():
            arr = (PackDesc * len(ds))()
            blk = []
            for i, (w, wf, wT, K, Creal, R, C, ldT, segs, split, _) in enumerate(ds):
                e = arr[i]
                e.w, e.wf, e.wT = w.data_ptr(), wf, wT
                e.K, e.Creal, e.R, e.C, e.ldT = K, Creal, R, C, ldT
                e.block0 = len(blk)
                e.nseg = len(segs) if segs else 0
                for j, (a, b, n) in enumerate(segs or []):
                    e.src0[j], e.dst0[j], e.len[j] = a, b, n
                e.split = int(split)
                blk += [i] * _tiles(2 * K if split else K, C, R)
            dev = ds[0][0].device
            raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
            table = raw.to(dev)
            b2d = torch.tensor(blk, dtype=torch.int32).to(dev)
            self.tables[dt] = (table, b2d, len(ds), len(blk))
        self.dirty = False

    # ---------------------------------------------------------------- sites --
    def pack(self, weight: torch.Tensor, Cp: int, dtype: torch.dtype, wf=True, wT=True,
             ldT: Optional[int] = None, segs=None, split: bool = False):
        """``split`` (bf16): 2K packed rows, the weight and its bf16 rounding
        residual (um_pack_weight_split)"""
        K, Creal, R, _ = weight.shape
        K2 = 2 * K if split else K
        ldT = ldT or K2
        if split and (dtype != torch.bfloat16 or segs):
            raise ValueError('split packing: bf16 without segments only')
        key = ('w', weight.data_ptr(), tuple(weight.shape), Cp, dtype, ldT,
               tuple(segs) if segs else None, bool(wf), bool(wT), bool(split))
        e = self.entries.get(key)
        if e is not None and self.batched and key in self.registered:
            return e
        w = _f32(weight)
        if e is None:
            f = torch.empty((K2, R, R, Cp), dtype=dtype, device=w.device) if wf else None
            t = None
            if wT:
                t = (torch.zeros if ldT != K2 else torch.empty)((Cp, R, R, ldT), dtype=dtype,
                                                                 device=w.device)
            e = (f, t)
            if self._register(weight, w, ptr(f), ptr(t), K, Creal, R, Cp, ldT, segs, dtype,
                              split):
                self.registered.add(key)
            self.entries[key] = e
        _pack_one(w, e[0], e[1], Cp, ldT, segs, dtype, split)
        return e

    def pack_rows(self, weights, C: int, dtype: torch.dtype):
        """The attention's fused K/Q/V 1x1 weights: wf [nC][1][1][C] (rows
        i*C...) and wT [C][1][1][nC] (columns i*C...)."""
        n = len(weights)
        key = ('rows', tuple(w.data_ptr() for w in weights), C, dtype)
        e = self.entries.get(key)
        if e is not None and self.batched and key in self.registered:
            return e
        dev = weights[0].device
        if e is None:
            f = torch.empty((n * C, 1, 1, C), dtype=dtype, device=dev)
            t = torch.empty((C, 1, 1, n * C), dtype=dtype, device=dev)
            e = (f, t)
            es = t.element_size()
            if all(_f32(wg).data_ptr() == wg.data_ptr() for wg in weights):
                for i, wg in enumerate(weights):
                    self._register(wg, wg, f[i * C].data_ptr(), t.data_ptr() + i * C * es,
                                   C, C, 1, C, n * C, None, dtype)
                self.registered.add(key)
            self.entries[key] = e
        f, t = e
        es = t.element_size()
        for i, wg in enumerate(weights):
            call('um_pack_weight', L.dtype_code(dtype), ptr(_f32(wg)), C, C, 1, C,
                 f[i * C].data_ptr(), t.data_ptr() + i * C * es, n * C)
        return e

    def pack_bias(self, biases, C: int):
        """The attention's fused K/Q/V bias: one f32 [nC] vector of the n
        biases (each [C], f32 parameters), refreshed by the f32 batch launch
        (a bias is packed as a [C][1][1][1] weight into the data-gradient
        layout [1][1][1][nC] at column i*C) instead of a torch.cat per
        attention block and step."""
        n = len(biases)
        key = ('bias', tuple(b.data_ptr() for b in biases), C)
        e = self.entries.get(key)
        if e is not None and self.batched and key in self.registered:
            return e
        dev = biases[0].device
        if e is None:
            e = torch.empty((n * C,), dtype=torch.float32, device=dev)
            if all(_f32(b).data_ptr() == b.data_ptr() for b in biases):
                for i, b in enumerate(biases):
                    self._register(b, b, None, e.data_ptr() + i * C * 4, C, 1, 1, 1, n * C,
                                   None, torch.float32)
                self.registered.add(key)
            self.entries[key] = e
        torch.cat([_f32(b) for b in biases], out=e)
        return e

    def _register(self, weight, w32, wf, wT, K, Creal, R, C, ldT, segs, dtype, split=False):
        if w32.data_ptr() != weight.data_ptr():
            # the batch reads the parameter memory directly: only f32 contiguous params
            return False
        if R not in (1, 3, 5, 7):  # pack_batch_kernel's compile-time filter sizes
            return False
        self.descs.append((weight, wf, wT, K, Creal, R, C, ldT, list(segs) if segs else None,
                           bool(split), weight.data_ptr(), L.dtype_code(dtype)))
        self.dirty = True
        return True


def _f32(weight):
    w = weight.detach()
    if w.dtype != torch.float32 or not w.is_contiguous():
        w = w.float().contiguous()
    return w


def _pack_one(w, f, t, Cp, ldT, segs, dtype, split=False):
    K, Creal, R, _ = w.shape
    if split:
        call('um_pack_weight_split', ptr(w), K, Creal, R, Cp, ptr(f), ptr(t), ldT)
        return
    if segs:
        n = len(segs)
        a0 = (ctypes.c_int * n)(*[a for a, _, _ in segs])
        b0 = (ctypes.c_int * n)(*[b for _, b, _ in segs])
        l0 = (ctypes.c_int * n)(*[c for _, _, c in segs])
    else:
        n, a0, b0, l0 = 0, None, None, None
    call('um_pack_weight_seg', L.dtype_code(dtype), ptr(w), K, Creal, R, Cp, ptr(f), ptr(t), ldT,
         n, a0, b0, l0)


_ACTIVE: Optional[WeightPacker] = None


def active() -> Optional[WeightPacker]:
    return _ACTIVE


@contextmanager
def scope(packer: Optional[WeightPacker]):
    """Make ``packer`` the pack cache of the convs called inside (one forward)."""
    global _ACTIVE
    prev = _ACTIVE
    _ACTIVE = packer
    try:
        if packer is not None:
            packer.begin()
        yield packer
    finally:
        _ACTIVE = prev
