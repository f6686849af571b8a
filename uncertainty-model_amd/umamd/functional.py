"""Autograd functions over the umamd C ABI (HIP kernels on gfx950).

Activations inside the model are NHWC tensors ``[N, H, W, C]`` (C a multiple
of 8), element type float32 or bfloat16; parameters stay in the reference's
NCHW float32 layout and are repacked per call by ``um_pack_weight``.  No
function here has a CPU path: every op calls the HIP library.

Granularity (one autograd node each):
  * ``conv_bn_elu``     Conv2d (+zero/reflect pad) -> BatchNorm2d(train) -> ELU,
                        optionally followed by the SE squeeze/excite gate
                        (reference model/layers/encoder.py:21-52,
                        model/layers/decoder.py:55-87,90-136)
  * ``merge``           NodeBlock weighted predecessor sum (encoder.py:115-124)
  * ``attention_block`` EfficientAttention incl. 1x1 convs and residual
                        (model/layers/attention.py:42-76)
  * ``concat``          decoder concat of copy / x2-bilinear / pixel-shuffle
                        sources with optional per-(n,c) gates
                        (model/layers/decoder.py:228-242)
  * ``disp_head``       ConvLayer(sigmoid) * scale (decoder.py:244-247)
  * ``tukra_loss``      the 4-scale loss stack (train/loss.py:512-568)
"""
from __future__ import annotations

import os
from contextlib import contextmanager
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from . import _lib as L
from . import overlap as _overlap
from . import packer as _packer
from . import bnx as _bnx
from . import rccl as _rccl
from ._lib import call, ptr, query


def ceil8(c: int) -> int:
    return (c + 7) // 8 * 8


def _dt(t: torch.Tensor) -> int:
    return L.dtype_code(t.dtype)


# --------------------------------------------------------------- helpers ----
def _seg_arrays(segs):
    if not segs:
        return 0, None, None, None
    n = len(segs)
    return (n, (ctypes_i * n)(*[a for a, _, _ in segs]), (ctypes_i * n)(*[b for _, b, _ in segs]),
            (ctypes_i * n)(*[c for _, _, c in segs]))


def _pack(weight: torch.Tensor, Cp: int, dtype: torch.dtype, wf=True, wT=True, ldT=None,
          segs=None, split=False):
    """Repack an NCHW f32 conv weight to [K][R][R][Cp] and [Cp][R][R][ldT];
    ``segs`` = [(ref_c0, packed_c0, len)] places input-channel ranges.
    ``split`` (bf16): 2K rows, the weight then its bf16 rounding residual
    (um_pack_weight_split)."""
    pk = _packer.active()
    if pk is not None:
        return pk.pack(weight, Cp, dtype, wf=wf, wT=wT, ldT=ldT, segs=segs, split=split)
    if split:
        K, Creal, R, _ = weight.shape
        ldT = ldT or 2 * K
        w = weight.detach().float().contiguous()
        f = torch.empty((2 * K, R, R, Cp), dtype=dtype, device=w.device) if wf else None
        t = (torch.zeros if ldT != 2 * K else torch.empty)((Cp, R, R, ldT), dtype=dtype,
                                                            device=w.device) if wT else None
        call('um_pack_weight_split', ptr(w), K, Creal, R, Cp, ptr(f), ptr(t), ldT)
        return f, t
    K, Creal, R, _ = weight.shape
    ldT = ldT or K
    w = weight.detach()
    if w.dtype != torch.float32 or not w.is_contiguous():
        w = w.float().contiguous()
    f = torch.empty((K, R, R, Cp), dtype=dtype, device=w.device) if wf else None
    t = None
    if wT:
        t = (torch.zeros if ldT != K else torch.empty)((Cp, R, R, ldT), dtype=dtype,
                                                        device=w.device)
    n, a0, b0, l0 = _seg_arrays(segs)
    call('um_pack_weight_seg', L.dtype_code(dtype), ptr(w), K, Creal, R, Cp, ptr(f), ptr(t), ldT,
         n, a0, b0, l0)
    return f, t


def _conv_flops(N, P, Q, K, R, C):
    """algorithmic FLOPs of a conv pass with the REAL (unpadded) channel counts"""
    return 2.0 * N * P * Q * K * R * R * C


def _conv_fwd(x, wf, bias, K, R, stride, pad, pad_mode, out_dtype=None, epi=L.EPI_NONE,
              epi_scale=1.0, residual=None, stats=None, out=None, ldo=None, creal=None):
    N, H, W, C = x.shape
    P = (H + 2 * pad - R) // stride + 1
    Q = (W + 2 * pad - R) // stride + 1
    od = out_dtype or x.dtype
    if out is None:
        ldo = ldo or K
        out = torch.empty((N, P, Q, ldo), dtype=od, device=x.device)
    wsb = query('um_conv_fwd_ws', _dt(x), N, P, Q, K, R, C)
    ws = torch.empty((wsb // 4,), dtype=torch.float32, device=x.device) if wsb else None
    call('um_conv2d_fwd', _dt(x), N, H, W, C, C, ptr(x), ptr(wf), ptr(bias), K, R, stride, pad,
         pad_mode, P, Q, L.dtype_code(od), ptr(out), out.shape[-1], epi, float(epi_scale),
         ptr(residual), residual.shape[-1] if residual is not None else 0, ptr(stats),
         ptr(ws), wsb, work=_conv_flops(N, P, Q, K, R, creal or C))
    return out


def _conv_dgrad(dy, wT, x_shape, K, R, stride, pad, pad_mode, dx=None, accumulate=False,
                creal=None, kreal=None):
    N, H, W, C = x_shape
    _, P, Q, ldy = dy.shape
    if dx is None:
        dx = torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
    wsb = query('um_conv_dgrad_ws_pad', _dt(dy), N, H, W, C, R, K, stride, pad, pad_mode)
    ws = torch.empty((wsb // 4,), dtype=torch.float32, device=dy.device) if wsb else None
    call('um_conv2d_dgrad', _dt(dy), N, H, W, C, C, ptr(dx), int(accumulate), ptr(wT), K, R,
         stride, pad, pad_mode, P, Q, ptr(dy), ldy, ptr(ws), wsb,
         work=_conv_flops(N, P, Q, kreal or K, R, creal or C))
    return dx


def _conv_wgrad(x, dy, K, Kreal, Creal, R, stride, pad, pad_mode, dw=None, segs=None):
    """dW in the reference NCHW layout [Kreal][Creal][R][R] (f32).  Under
    ``overlap.WgradStream`` it is issued on the side stream (see there)."""
    ov = _overlap.active()
    if dw is None:
        dw = torch.empty((Kreal, Creal, R, R), dtype=torch.float32, device=x.device)
    if ov is None:
        _conv_wgrad_on(x, dy, K, Kreal, Creal, R, stride, pad, pad_mode, ptr(dw), segs)
        return dw
    # the queued launch holds dw's address, not the tensor: an extra reference
    # would make AccumulateGrad copy the (not yet written) gradient on the
    # launch stream instead of taking it over.  dw stays alive as param.grad.
    dw.record_stream(ov.stream)
    dw_ptr = ptr(dw)
    N, _, _, _ = x.shape
    _, P, Q, _ = dy.shape
    launch = lambda: _conv_wgrad_on(x, dy, K, Kreal, Creal, R, stride, pad,  # noqa: E731
                                    pad_mode, dw_ptr, segs)
    ov.defer((x, dy), launch, out_ptr=dw_ptr, flop=_conv_flops(N, P, Q, Kreal, R, Creal),
             out_bytes=dw.numel() * 4)
    return dw


# the merge-weight gradients of a side-stream flush as one um_merge_wgrad_batch
# launch (15 single-workgroup launches -> 1 per flush)
_MWG_BATCH = os.environ.get('UMAMD_MWG_BATCH', '1') == '1'


def batched_launch(descs):
    """The batched launches of a side-stream flush: every um_mwg_desc in
    um_merge_wgrad_batch calls, every um_csum_desc in um_colsum_batch calls
    (in chunks of the entries' maxima)."""
    ds = [d for d in descs if isinstance(d, L.MwgDesc)]
    for i in range(0, len(ds), L.MWG_MAX):
        chunk = ds[i:i + L.MWG_MAX]
        arr = (L.MwgDesc * len(chunk))(*chunk)
        call('um_merge_wgrad_batch', _ct.cast(arr, ctypes_p), len(chunk))
    cs = [d for d in descs if isinstance(d, _Csum)]
    for dt in sorted({d.dtype for d in cs}):
        ds = [d.desc for d in cs if d.dtype == dt]
        for i in range(0, len(ds), L.CSUM_MAX):
            chunk = ds[i:i + L.CSUM_MAX]
            arr = (L.CsumDesc * len(chunk))(*chunk)
            call('um_colsum_batch', dt, _ct.cast(arr, ctypes_p), len(chunk))


def _conv_wgrad_on(x, dy, K, Kreal, Creal, R, stride, pad, pad_mode, dw_ptr, segs):
    N, H, W, C = x.shape
    _, P, Q, ldy = dy.shape
    M = N * P * Q
    RRC = R * R * C
    splits = query('um_conv_wgrad_splits', _dt(x), N, H, W, C, C, K, R, stride, pad, pad_mode,
                   P, Q, ldy)
    slabs = torch.empty((splits, K, RRC), dtype=torch.float32, device=x.device)
    call('um_conv2d_wgrad', _dt(x), N, H, W, C, C, ptr(x), K, R, stride, pad, pad_mode, P, Q,
         ptr(dy), ldy, ptr(slabs), splits, work=_conv_flops(N, P, Q, Kreal, R, Creal))
    n, a0, b0, l0 = _seg_arrays(segs)
    call('um_conv_wgrad_reduce_seg', ptr(slabs), splits, K, Kreal, R, C, Creal, dw_ptr, 0,
         n, a0, b0, l0)


def _colred_ws(nparts, C, nv, device):
    """f64 slab rows of the one-launch column reductions (um_colred_ws)"""
    n = query('um_colred_ws', nparts, C, nv)
    return torch.empty((max(n, 8) // 8,), dtype=torch.float64, device=device)


def _reduce_rows(parts, nparts, C, out, accumulate=False, out_ptr=None):
    call('um_reduce_rows', ptr(parts), nparts, C, C, out_ptr or ptr(out), int(accumulate),
         ptr(_colred_ws(nparts, C, 1, parts.device)))
    return out


def _colsum(y, C):
    """sum over pixels of y[..., :C] -> f32 [C]"""
    out = torch.empty((C,), dtype=torch.float32, device=y.device)
    _colsum_into(y, C, ptr(out))
    return out


def _colsum_into(y, C, out_ptr):
    M = y.numel() // y.shape[-1]
    parts_n = query('um_colsum_parts', M)
    parts = torch.empty((parts_n, C), dtype=torch.float32, device=y.device)
    call('um_colsum', _dt(y), M, C, y.shape[-1], ptr(y), ptr(parts))
    _reduce_rows(parts, parts_n, C, None, out_ptr=out_ptr)


def _param_grad(tensors, out, launch):
    """Launches whose only product is a parameter gradient ``out`` (read
    by the optimiser after the whole backward): under overlap.WgradStream
    they are queued onto the weight-gradient side stream like the conv
    weight gradients (off the data-gradient chain), else run now.
    ``tensors``: what ``launch`` reads; ``launch`` must reach ``out`` by
    address only (as _conv_wgrad: a second reference would make autograd's
    AccumulateGrad copy the not yet written gradient instead of taking it)."""
    ov = _overlap.active()
    if ov is None:
        launch()
        return out
    out.record_stream(ov.stream)
    ov.defer(tensors, launch, out_ptr=out.data_ptr(), out_bytes=out.numel() * out.element_size())
    return out


class _Csum:
    """a queued bias gradient for um_colsum_batch (descriptor + dtype)"""
    __slots__ = ('desc', 'dtype')

    def __init__(self, desc, dtype):
        self.desc, self.dtype = desc, dtype


# the side stream's bias gradients as one um_colsum_batch (two launches) per
# flush instead of um_colsum + um_reduce_rows per bias
_CSUM_BATCH = os.environ.get('UMAMD_CSUM_BATCH', '1') == '1'


def _colsum_grad(y, C):
    """a bias gradient (sum over pixels of y[..., :C]) as _param_grad"""
    out = torch.empty((C,), dtype=torch.float32, device=y.device)
    optr = ptr(out)
    if _CSUM_BATCH and _overlap.active() is not None and C % 8 == 0 and y.shape[-1] % 8 == 0:
        M = y.numel() // y.shape[-1]
        nparts = query('um_colsum_parts', M)
        parts = torch.empty((nparts, C), dtype=torch.float32, device=y.device)
        d = L.CsumDesc()
        d.y, d.parts, d.out = y.data_ptr(), parts.data_ptr(), optr
        d.M, d.C, d.ld, d.nparts, d.creal = M, C, y.shape[-1], nparts, C
        # parts is allocated on the launch stream: listed with y so the flush
        # marks it used by the side stream (record_stream) before it is freed
        return _param_grad((y, parts), out, lambda d=_Csum(d, _dt(y)), keep=parts: (keep, d))
    return _param_grad((y,), out, lambda: _colsum_into(y, C, optr))


_CONSTS = {}
# A/B switches for two fused paths (bench step, tools/sweep.sh):
#  - the SE squeeze summed inside the BN forward (per-block channel sums,
#    finished by the SE MLP kernel): on, 676 -> 678 pairs/s (-10 launches)
#  - (removed round 5) the BN backward coefficients finished inside the
#    reduce kernel by a two-level last-arriver tree: 676 -> 652 -- every
#    block's agent-scope release + ticket cost more than the separate
#    reduction launch it replaced
_FUSED_SE = os.environ.get('UMAMD_FUSED_SE', '1') == '1'
#  - single-process BN statistics as f64 atomics into zeroed slots, finished
#    by the consumer kernels (no reduction launch per BN layer and direction)
_BN_SLOTS = os.environ.get('UMAMD_BN_SLOTS', '1') == '1'
#  - the pre-BN conv output y stored in the activation dtype (bf16) instead of
#    f32, as a bf16 autocast conv feeding BatchNorm2d: the conv epilogue still
#    takes the statistics from its f32 accumulators; the three BN passes and
#    the conv's store move 2 bytes per element less.  OFF by default since
#    round 4: +2.3 % throughput (790 -> 808 pairs/s, round 3), but the
#    step-0 error loss at BASELINE config 2 moves 4.7e-3 from the reference
#    with bf16 y against 1.9e-3 with f32 y (tools/bf16_arms.py,
#    profiles/r04/bf16_arms.txt): in the smooth layers the batch std is ~1/17
#    of the mean, so the rounding of y is ~17x larger relative to the
#    normalised x-hat than the rounding of the activations.  (Round 5 removed
#    the f16 y and the centred bf16 y: both measured, neither reached the
#    f32 y's error.)
_Y_ACT = os.environ.get('UMAMD_Y_ACT', '0') == '1'


def _ydtype(dt):
    """storage dtype of the pre-BN conv output for activations of ``dt``"""
    return dt if (_Y_ACT and dt == torch.bfloat16) else torch.float32


def _ydt(a, y):
    """dtype code of a BN entry: activations ``a`` (a / da), plus UM_Y_ACT
    when the pre-BN ``y`` is stored in their dtype"""
    return _dt(a) | (L.Y_ACT if y.dtype != torch.float32 else 0)


class StatArena:
    """Zeroed f64 scratch for the BN statistics slots of one model forward
    and its backward (``um_bn_elu_fwd_slots`` / ``*_bwd_*_slots``).

    ``begin`` allocates ONE zeroed buffer (one fill launch per forward, sized
    by the previous forward's use) and ``take`` hands out views of it; the
    autograd graph keeps the buffer alive until its backward has run, so two
    forwards in flight never share slots.  A forward that needs more than the
    hint grows by further zeroed chunks (the first forward of a model)."""

    CHUNK = 1 << 16

    def __init__(self):
        self.hint = 0
        self.buf = None
        self.off = 0
        self.used = 0

    def begin(self, device):
        self.buf = torch.zeros((max(self.hint, self.CHUNK),), dtype=torch.float64, device=device)
        self.off = 0
        self.used = 0

    def take(self, n: int) -> torch.Tensor:
        n = (n + 31) // 32 * 32  # 256-byte aligned views
        if self.off + n > self.buf.numel():
            self.buf = torch.zeros((max(n, self.CHUNK),), dtype=torch.float64,
                                   device=self.buf.device)
            self.off = 0
        v = self.buf[self.off:self.off + n]
        self.off += n
        self.used += n
        return v

    def end(self):
        self.hint = max(self.hint, self.used)
        self.buf = None

    def __deepcopy__(self, memo):
        return StatArena()


_ARENA: Optional[StatArena] = None


@contextmanager
def stat_scope(arena: Optional[StatArena], device):
    """Make ``arena`` the BN statistics scratch of the convs called inside
    (one model forward); without one, BN uses the partial-row reductions."""
    global _ARENA
    prev = _ARENA
    _ARENA = arena if _BN_SLOTS else None
    try:
        if _ARENA is not None:
            _ARENA.begin(device)
            _bnx.begin_forward()  # SyncBN IPC exchange slots count from each forward
        yield
    finally:
        if _ARENA is not None:
            _ARENA.end()
        _ARENA = prev


class GradSlots:
    """Input gradients of activations that several umamd autograd functions
    consume inside one model forward: encoder stage outputs (next stage +
    decoder), decoder outputs (next stage + disparity head), SE-gated skips
    (this stage's concat + the next stage's skip conv), the decoder's input.
    The first consumer to run its backward writes the gradient into a fresh
    buffer and hands that to autograd; every later one ACCUMULATES into the
    same buffer (GEMM / concat-adjoint accumulate epilogues) and returns None,
    so autograd sums nothing -- it would launch one elementwise add per extra
    consumer (12 bf16 adds per step).
    Limitation: a tensor with two or more registered consumers must have NO
    unregistered one (the loss, user code).  Autograd would sum that
    consumer's gradient with the first registered one's into a new buffer
    (or into that buffer in place, by its own choice), so a later registered
    consumer's accumulate could land in a tensor autograd no longer passes
    on: its term would be lost.  In the model every pooled tensor is
    consumed only inside the forward (the submodules run through their
    ``_fwd`` paths, so no forward hook sees an intermediate; the
    disparities, which the loss reads, have a single registered use and are
    never pooled).
    Guard: every pooled tensor gets a gradient hook that checks that the
    gradient autograd finally hands on IS the pooled buffer; if another
    consumer made autograd sum into a new one, it raises (the step's
    gradient is incomplete) and turns pooling off for every later forward
    (``GradSlots.broken``), so the next step runs on autograd's sums.
    UMAMD_GRAD_SLOTS=0 turns it off."""

    broken = False

    def __init__(self):
        self.uses = {}
        self.bufs = {}
        self.final = {}   # key -> data_ptr of the pooled buffer (set by done)
        self.hooked = set()

    @staticmethod
    def key(t):
        return (t.data_ptr(), tuple(t.shape), t.dtype)

    def use(self, t):
        """a consumer's forward: note one more registered use of t"""
        if t is not None and t.requires_grad:
            k = self.key(t)
            self.uses[k] = self.uses.get(k, 0) + 1
            if self.uses[k] == 2 and k not in self.hooked:
                self.hooked.add(k)
                t.register_hook(lambda g, k=k: self._check(k, g))
            return k
        return None

    def _check(self, k, g):
        """gradient hook of a pooled tensor: autograd's final gradient must
        be the pooled buffer (no unregistered consumer summed into another)"""
        want = self.final.get(k)
        if want is not None and g is not None and g.data_ptr() != want:
            GradSlots.broken = True
            raise RuntimeError(
                'umamd GradSlots: an activation that umamd ops accumulate gradients into in '
                'place also has a consumer outside them, so its gradient is incomplete for this '
                'step; pooling is now off for later forwards (UMAMD_GRAD_SLOTS=0 avoids it)')
        return None

    def target(self, k):
        """a consumer's backward: (buffer to accumulate into, or None)"""
        if k is None or self.uses.get(k, 0) <= 1:
            return None
        e = self.bufs.get(k)
        return e[0] if e is not None else None

    def done(self, k, g):
        """after writing (or accumulating into) g: what to return to autograd"""
        if k is None or self.uses.get(k, 0) <= 1:
            return g
        e = self.bufs.get(k)
        if e is None:  # first consumer: keep the buffer for the others
            self.bufs[k] = [g, self.uses[k] - 1]
            self.final[k] = g.data_ptr()
            return g
        e[1] -= 1
        if e[1] <= 0:
            del self.bufs[k]
        return None


_GSLOTS: Optional[GradSlots] = None
_GRAD_SLOTS = os.environ.get('UMAMD_GRAD_SLOTS', '1') == '1'


@contextmanager
def grad_slots():
    """one GradSlots registry for the consumers called inside (a model forward)"""
    global _GSLOTS
    prev = _GSLOTS
    _GSLOTS = GradSlots() if _GRAD_SLOTS and not GradSlots.broken else None
    try:
        yield
    finally:
        _GSLOTS = prev


def _use(ctx, *ts):
    """forward: register the inputs ts; ctx.gk = their keys, ctx.gs = registry"""
    ctx.gs = _GSLOTS
    ctx.gk = [(_GSLOTS.use(t) if _GSLOTS is not None else None) for t in ts]


def _slot(ctx, i):
    """backward: (accumulate target or None) for registered input i"""
    gs = getattr(ctx, 'gs', None)
    return gs.target(ctx.gk[i]) if gs is not None else None


def _give(ctx, i, g):
    gs = getattr(ctx, 'gs', None)
    return gs.done(ctx.gk[i], g) if gs is not None and g is not None else g


def _const_vec(value: float, n: int, device) -> torch.Tensor:
    """A read-only f32 vector of ``value`` (first n entries of a cached
    buffer): identity BN coefficients without a fill launch per conv."""
    key = (str(device), float(value))
    buf = _CONSTS.get(key)
    if buf is None or buf.numel() < n:
        buf = torch.full((max(n, 512),), float(value), dtype=torch.float32, device=device)
        _CONSTS[key] = buf
    return buf[:n]


class BNSync:
    """How a BN layer exchanges statistics (SyncBatchNorm semantics).
    UMAMD_DIST=1 keeps the all-reduce with a single rank (rehearsal of the
    data-parallel path on one GPU)."""

    force = os.environ.get('UMAMD_DIST') == '1'

    def __init__(self, bn: torch.nn.Module):
        self.bn = bn
        self.group = None
        self.world = 1
        if isinstance(bn, torch.nn.SyncBatchNorm) and dist.is_available() and \
                dist.is_initialized():
            self.group = bn.process_group or dist.group.WORLD
            self.world = dist.get_world_size(self.group)

    @property
    def collective(self) -> bool:
        """statistics go through the process group (else the one-launch
        single-process kernels are used)"""
        return self.group is not None and (self.world > 1 or self.force)

    def all_reduce(self, t: torch.Tensor):
        if self.collective:
            c = _rccl.active(self.group)  # the captured step's own communicator
            if c is not None:
                c.all_reduce(t)
            else:
                dist.all_reduce(t, group=self.group)

    def all_reduce_slots(self, t: torch.Tensor, C: int):
        """in-place all-reduce of a statistics-slot tensor ([16][C][2] f64 +
        count): over the IPC exchange (umamd.bnx, UMAMD_SYNCBN_IPC=1) -- one
        kernel, no RCCL call -- else as all_reduce"""
        if not self.collective:
            return
        x = _bnx.get(self.group) if self.world > 1 else None
        if x is not None:
            x.all_reduce_slots(t, C)
        else:
            self.all_reduce(t)


def _bn_forward_coeffs(parts, nparts, K, count, bn, sync: BNSync, training: bool, device):
    mean = torch.empty(K, dtype=torch.float32, device=device)
    invstd = torch.empty_like(mean)
    scale = torch.empty_like(mean)
    shift = torch.empty_like(mean)
    gamma = bn.weight if bn.affine else None
    beta = bn.bias if bn.affine else None
    if training or not bn.track_running_stats:
        upd = training and bn.track_running_stats and bn.running_mean is not None
        if upd and bn.momentum is None:
            raise NotImplementedError('BatchNorm momentum=None (cumulative average) is not supported')
        ws = _colred_ws(nparts, K, 2, device)
        rs = (ptr(bn.running_mean) if upd else None, ptr(bn.running_var) if upd else None,
              ptr(bn.num_batches_tracked) if upd and bn.num_batches_tracked is not None else None)
        if not sync.collective:
            # one launch: reduce the conv-epilogue partials and finish the coefficients
            call('um_bn_stats_coeffs', ptr(parts), nparts, K, ptr(ws), float(count), ptr(gamma),
                 ptr(beta), float(bn.eps), float(bn.momentum or 0.0), *rs, ptr(mean),
                 ptr(invstd), ptr(scale), ptr(shift))
        else:
            # (K + 1) x 2 f64: the channel sums, then this rank's element
            # count, all-reduced together (per-rank batches may differ, as in
            # torch SyncBatchNorm's count all-gather) -- no host sync
            st = torch.empty((K + 1, 2), dtype=torch.float64, device=device)
            st[K].fill_(float(count))
            call('um_bn_stats_reduce', ptr(parts), nparts, K, ptr(st), ptr(ws))
            sync.all_reduce(st)
            call('um_bn_coeffs', ptr(st), -1.0, K, ptr(gamma), ptr(beta),
                 float(bn.eps), float(bn.momentum or 0.0), *rs,
                 ptr(mean), ptr(invstd), ptr(scale), ptr(shift))
    else:
        # eval mode: normalise with the running statistics
        st = torch.stack([bn.running_mean.double(), (bn.running_var.double() + bn.running_mean.double() ** 2)], 1).contiguous()
        call('um_bn_coeffs', ptr(st), 1.0, K, ptr(gamma), ptr(beta), float(bn.eps), 0.0, None,
             None, None, ptr(mean), ptr(invstd), ptr(scale), ptr(shift))
    return mean, invstd, scale, shift


# ---------------------------------------------------------- conv+BN+ELU ----
class ConvSpec:
    """Static description of a conv block (non-tensor autograd argument)."""

    def __init__(self, conv: torch.nn.Conv2d, bn: Optional[torch.nn.Module], pad: int,
                 pad_mode: int, elu: bool = True, segs=None):
        self.segs = segs
        self.conv = conv
        self.bn = bn
        self.stride = conv.stride[0]
        self.pad = pad
        self.pad_mode = pad_mode
        self.elu = elu


class _CBEState:
    """What a conv+BN+ELU forward keeps for its backward (the autograd ctx
    of ConvBNELUFn, or one node of a GraphBlockFn)."""
    __slots__ = ('spec', 'sync', 'slots_b', 'has_bn', 'geom', 'se', 'saved', 'merged', 'prereduced')


def _cbe_fwd(x, weight, bias, gamma, beta, w1, w2, spec: ConvSpec, merge=None, yconv=None):
    """Conv2d -> BatchNorm2d -> ELU [-> SE gate] forward without autograd:
    -> (outputs tuple, _CBEState).  ``merge`` = (srcs with None for this
    layer's output, widx, mean_weight): also compute that NodeBlock merge
    (fused into the BN apply pass where the statistics slots are used), the
    result in ``state.merged``.  ``yconv(epi, stats, bias)`` replaces the conv
    (it returns the f32 pre-BN output; the state then saves no packed
    weights: its backward brings its own conv part, see skip_conv_bn_elu)."""
    ctx = _CBEState()
    ctx.prereduced = False  # GraphBlockFn: the merge backward took the BN-backward sums
    L.require_device(x)
    N, H, W, Cp = x.shape
    K, Creal, R, _ = weight.shape
    bn = spec.bn
    dev = x.device
    wf, wT = _pack(weight, Cp, x.dtype, segs=spec.segs) if yconv is None else (None, None)
    P = (H + 2 * spec.pad - R) // spec.stride + 1
    Q = (W + 2 * spec.pad - R) // spec.stride + 1
    M = N * P * Q
    bias_f = bias.detach().float().contiguous() if bias is not None else None
    slots_f = slots_b = None
    if bn is not None:
        training = bn.training
        sync = BNSync(bn)
    count = float(M)
    if bn is not None and training and _ARENA is not None:
        # statistics in f64 slots: the conv adds them atomically, the BN
        # apply finishes them (no reduction launch).  SyncBN: the slots
        # and this rank's element count after them are all-reduced in
        # place (the count rides along: uneven per-rank batches)
        if bn.track_running_stats and bn.running_mean is not None and bn.momentum is None:
            raise NotImplementedError('BatchNorm momentum=None (cumulative average) is not supported')
        nslot = L.STAT_SLOTS * K * 2
        slots_f = _ARENA.take(nslot + 1)
        slots_b = _ARENA.take(nslot + 1)
        y = _conv_fwd(x, wf, bias_f, K, R, spec.stride, spec.pad, spec.pad_mode,
                      out_dtype=_ydtype(x.dtype), epi=L.EPI_STAT_SLOTS, stats=slots_f,
                      creal=Creal) if yconv is None else yconv(L.EPI_STAT_SLOTS, slots_f, bias_f)
        if sync.collective:  # the conv stored this rank's count after the slots
            sync.all_reduce_slots(slots_f, K)
            count = -1.0  # read the all-reduced count after the slots
        mean = torch.empty(K, dtype=torch.float32, device=dev)
        invstd = torch.empty_like(mean)
        scale = torch.empty_like(mean)
        shift = torch.empty_like(mean)
    elif bn is not None:
        nparts = query('um_conv_stats_parts', M, K)
        parts = torch.empty((nparts, K, 2), dtype=torch.float32, device=dev)
        epi = L.EPI_STATS if training else L.EPI_NONE
        y = _conv_fwd(x, wf, bias_f, K, R, spec.stride, spec.pad, spec.pad_mode,
                      out_dtype=_ydtype(x.dtype), epi=epi, stats=parts, creal=Creal) \
            if yconv is None else yconv(epi, parts, bias_f)
        mean, invstd, scale, shift = _bn_forward_coeffs(parts, nparts, K, M, bn, sync,
                                                        training, dev)
    else:  # ConvELUBlock(batch_norm=False): identity normalisation
        sync = None
        training = False
        y = _conv_fwd(x, wf, bias_f, K, R, spec.stride, spec.pad, spec.pad_mode,
                      out_dtype=_ydtype(x.dtype), creal=Creal) if yconv is None \
            else yconv(L.EPI_NONE, None, bias_f)
        mean = shift = _const_vec(0.0, K, dev)
        invstd = scale = _const_vec(1.0, K, dev)
    a = torch.empty(y.shape, dtype=x.dtype, device=dev)  # y: pre-BN, f32 or bf16 (_ydtype)
    pool = None
    if w1 is not None and _FUSED_SE:  # the SE squeeze rides in the BN-apply pass
        npool = query('um_bn_fwd_pool_parts_c', M, P * Q, K)
        pool = torch.empty((npool, K), dtype=torch.float32, device=dev)
    merged = None
    if slots_f is not None:
        upd = bn.track_running_stats and bn.running_mean is not None
        nbt = bn.num_batches_tracked if upd else None
        rs = (ptr(bn.running_mean) if upd else None, ptr(bn.running_var) if upd else None,
              ptr(nbt))
        if merge is not None and pool is None and _FUSED_MERGE:
            msrcs, mwidx, mw = merge
            n = len(msrcs)
            merged = torch.empty_like(a)
            call('um_bn_elu_fwd_slots_merge', _ydt(a, y), M, K, ptr(y), K, ptr(slots_f), count,
                 ptr(gamma), ptr(beta), float(bn.eps), float(bn.momentum or 0.0), *rs,
                 ptr(mean), ptr(invstd), ptr(scale), ptr(shift), ptr(a), K, int(spec.elu), n,
                 (ctypes_p * n)(*[t.data_ptr() if t is not None else None for t in msrcs]),
                 (ctypes_i * n)(*mwidx), ptr(mw), msrcs.index(None), ptr(merged))
        else:
            call('um_bn_elu_fwd_slots', _ydt(a, y), M, K, ptr(y), K, ptr(slots_f), count,
                 ptr(gamma), ptr(beta), float(bn.eps), float(bn.momentum or 0.0), *rs,
                 ptr(mean), ptr(invstd), ptr(scale), ptr(shift), ptr(a), K,
                 int(spec.elu), P * Q, ptr(pool))
    else:
        call('um_bn_elu_fwd', _ydt(a, y), M, K, ptr(y), K, ptr(scale), ptr(shift), ptr(a), K,
             int(spec.elu), P * Q, ptr(pool))
    inv_hw = 1.0 / (P * Q)
    if w1 is not None and not _FUSED_SE:  # separate squeeze: the means, one row per image
        npool, inv_hw = N, 1.0
        pool = torch.zeros((N, K), dtype=torch.float32, device=dev)
        call('um_channel_mean', _dt(a), N, P * Q, K, ptr(a), K, ptr(pool))
    outs = [a]
    se = None
    if w1 is not None:
        R1 = w1.shape[0]
        pooled = torch.empty((N, K), dtype=torch.float32, device=dev)
        z1 = torch.empty((N, R1), dtype=torch.float32, device=dev)
        s = torch.empty((N, K), dtype=torch.float32, device=dev)
        w1c, w2c = w1.detach().float().contiguous(), w2.detach().float().contiguous()
        call('um_se_mlp_fwd', N, K, R1, ptr(pool), npool // N, inv_hw, ptr(pooled),
             ptr(w1c), ptr(w2c), ptr(z1), ptr(s))
        se = (pooled, z1, s)
        outs.append(s)
    if merge is not None and merged is None:  # not fused: the separate merge launch
        msrcs, mwidx, mw = merge
        merged = _merge_launch([a if t is None else t for t in msrcs], mw, mwidx, None,
                               torch.empty_like(a))
    ctx.merged = merged
    ctx.spec = spec
    ctx.sync = sync
    ctx.slots_b = slots_b
    ctx.has_bn = bn is not None and training
    ctx.geom = (N, H, W, Cp, K, Creal, R, P, Q)
    ctx.se = se
    ctx.saved = (x, wT, y, mean, invstd, scale, shift, gamma, w1, w2)
    return tuple(outs), ctx


def _cbe_bwd(ctx, da, ds=None, need_x=True, need_b=True, dx=None, dx_accumulate=False,
             conv_bwd=None):
    """Backward of _cbe_fwd -> (dx, dW, dbias, dgamma, dbeta, dw1, dw2).
    ``dx``: write (or with ``dx_accumulate`` add) the input gradient into
    this tensor instead of a new one (a GraphBlockFn predecessor's gradient
    buffer)."""
    x, wT, y, mean, invstd, scale, shift, gamma, w1, w2 = ctx.saved
    N, H, W, Cp, K, Creal, R, P, Q = ctx.geom
    spec = ctx.spec
    M = N * P * Q
    dev = y.device
    adt = x.dtype
    da = da.contiguous() if da is not None else torch.zeros(y.shape, dtype=adt, device=dev)
    if da.dtype != adt:
        da = da.to(adt)
    add_nc = None
    dw1 = dw2 = None
    if ctx.se is not None and ds is not None:
        pooled, z1, s = ctx.se
        R1 = w1.shape[0]
        dw1 = torch.empty(w1.shape, dtype=torch.float32, device=dev)
        dw2 = torch.empty(w2.shape, dtype=torch.float32, device=dev)
        add_nc = torch.empty((N, K), dtype=torch.float32, device=dev)
        dz = torch.empty((N, R1), dtype=torch.float32, device=dev)
        dsc = ds.float().contiguous()
        w1c, w2c = w1.detach().float().contiguous(), w2.detach().float().contiguous()
        call('um_se_mlp_bwd', N, K, R1, ptr(dsc), ptr(s), ptr(z1), ptr(pooled), ptr(w1c),
             ptr(w2c), ptr(dw1), ptr(dw2), ptr(add_nc), ptr(dz), 1.0 / (P * Q))
    dgamma = dbeta = dbias = None
    slots_b = ctx.slots_b
    if ctx.has_bn and slots_b is not None:
        # backward sums into the slots; the apply kernel finishes them
        if need_b:
            dbias = torch.empty(K, dtype=torch.float32, device=dev)
        if gamma is not None:
            dgamma = torch.empty(K, dtype=torch.float32, device=dev)
            dbeta = torch.empty(K, dtype=torch.float32, device=dev)
        if not ctx.prereduced:  # else um_merge_bwd_bn summed them (GraphBlockFn)
            call('um_bn_elu_bwd_reduce_slots', _ydt(da, y), M, K, P * Q, ptr(da), K, ptr(y), K,
                 ptr(mean), ptr(invstd), ptr(scale), ptr(shift), ptr(add_nc), int(spec.elu),
                 ptr(slots_b))
        local, bcount, bscale = None, float(M), 1.0
        if ctx.sync is not None and ctx.sync.collective:
            # k1..k3 from the global sums.  dgamma/dbeta and the conv-bias
            # gradient: the global sums / world -- no copy of this rank's
            # slots before the in-place all-reduce (one launch per layer
            # less).  PRECONDITION: the parameter gradients are AVERAGED over
            # the ranks afterwards (DDP, train.parallel.data_parallel; the
            # captured step's GradBuckets, RCCL AVG).  Then every rank ends
            # with mean_r(G / world) = G / world = mean_r(local_r), exactly
            # torch SyncBatchNorm's per-rank sums averaged by DDP (the
            # reference, parallel_main.py:156-158).  A caller that SUMS the
            # ranks' gradients gets G from both forms: also equal; one that
            # keeps per-rank gradients without any reduction is not supported
            ctx.sync.all_reduce_slots(slots_b, K)
            bcount, bscale = -1.0, 1.0 / ctx.sync.world
    elif ctx.has_bn:
        k1 = torch.empty(K, dtype=torch.float32, device=dev)
        k2 = torch.empty_like(k1)
        k3 = torch.empty_like(k1)
        # the conv bias feeds a training-mode BN: its gradient comes out of
        # the coefficient kernel in closed form (no reduction of dy)
        if need_b:
            dbias = torch.empty(K, dtype=torch.float32, device=dev)
        nb = query('um_bn_bwd_parts', M)
        parts = torch.empty((nb, K, 2), dtype=torch.float32, device=dev)
        world = ctx.sync.world if ctx.sync is not None else 1
        if gamma is not None:
            dgamma = torch.empty(K, dtype=torch.float32, device=dev)
            dbeta = torch.empty(K, dtype=torch.float32, device=dev)
        single = ctx.sync is None or not ctx.sync.collective
        if single:
            call('um_bn_elu_bwd_reduce', _ydt(da, y), M, K, P * Q, ptr(da), K, ptr(y), K,
                 ptr(mean), ptr(invstd), ptr(scale), ptr(shift), ptr(add_nc), int(spec.elu),
                 ptr(parts))
            call('um_bn_bwd_stats_coeffs', ptr(parts), nb, K, ptr(_colred_ws(nb, K, 2, dev)),
                 float(M), ptr(gamma), ptr(invstd), ptr(dgamma), ptr(dbeta), ptr(dbias),
                 ptr(k1), ptr(k2), ptr(k3))
        else:
            call('um_bn_elu_bwd_reduce', _ydt(da, y), M, K, P * Q, ptr(da), K, ptr(y), K,
                 ptr(mean), ptr(invstd), ptr(scale), ptr(shift), ptr(add_nc), int(spec.elu),
                 ptr(parts))
            ws = _colred_ws(nb, K, 2, dev)
            st = torch.empty((K + 1, 2), dtype=torch.float64, device=dev)
            st[K].fill_(float(M))  # this rank's count, summed by the all-reduce
            call('um_bn_stats_reduce', ptr(parts), nb, K, ptr(st), ptr(ws))
            st_local = st.clone()
            ctx.sync.all_reduce(st)
            call('um_bn_bwd_coeffs', ptr(st), -1.0, K, ptr(gamma), ptr(invstd),
                 ptr(st_local), ptr(dgamma), ptr(dbeta), ptr(dbias), 1.0 / world, 0,
                 ptr(k1), ptr(k2), ptr(k3))
    else:
        # no batch statistics (no BN, or BN in eval mode): dy = dz * scale
        k1 = scale
        k2 = k3 = _const_vec(0.0, K, dev)
        if gamma is not None and spec.bn is not None:
            raise NotImplementedError('backward through an eval-mode BatchNorm')
    dy = torch.empty(y.shape, dtype=adt, device=dev)
    nbp = query('um_bn_bwd_parts', M)
    reduce_b = need_b and dbias is None
    bparts = torch.empty((nbp, K), dtype=torch.float32, device=dev) if reduce_b else None
    if ctx.has_bn and slots_b is not None:
        call('um_bn_elu_bwd_apply_slots', _ydt(da, y), M, K, P * Q, ptr(da), K, ptr(y), K,
             ptr(mean), ptr(invstd), ptr(scale), ptr(shift), ptr(add_nc), int(spec.elu),
             ptr(slots_b), bcount, ptr(local), ptr(gamma), ptr(dgamma), ptr(dbeta),
             ptr(dbias), bscale, ptr(dy), K)
    else:
        call('um_bn_elu_bwd_apply', _ydt(da, y), M, K, P * Q, ptr(da), K, ptr(y), K, ptr(mean),
             ptr(invstd), ptr(scale), ptr(shift), ptr(add_nc), int(spec.elu), ptr(k1),
             ptr(k2), ptr(k3), ptr(dy), K, ptr(bparts))
    if conv_bwd is not None:  # the caller's conv part (skip_conv_bn_elu): dy -> (dx, dW)
        dx, dW = conv_bwd(dy)
        need_x = False
    else:
        dW = _conv_wgrad(x, dy, K, K, Creal, R, spec.stride, spec.pad, spec.pad_mode,
                         segs=spec.segs)
    if reduce_b:
        dbias = torch.empty(K, dtype=torch.float32, device=dev)
        _reduce_rows(bparts, nbp, K, dbias)
    if need_x:
        dx = _conv_dgrad(dy, wT, (N, H, W, Cp), K, R, spec.stride, spec.pad, spec.pad_mode,
                         dx=dx, accumulate=dx_accumulate, creal=Creal)
    elif conv_bwd is None:
        dx = None
    return dx, dW, dbias, dgamma, dbeta, dw1, dw2


class ConvBNELUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, gamma, beta, w1, w2, spec: ConvSpec):
        outs, st = _cbe_fwd(x, weight, bias, gamma, beta, w1, w2, spec)
        x_, wT, y, mean, invstd, scale, shift, gamma_, w1_, w2_ = st.saved
        st.saved = None
        ctx.st = st
        _use(ctx, x)
        ctx.save_for_backward(x_, wT, y, mean, invstd, scale, shift, gamma_, w1_, w2_)
        return outs if len(outs) > 1 else outs[0]

    @staticmethod
    def backward(ctx, da, ds=None):
        st = ctx.st
        st.saved = ctx.saved_tensors
        tgt = _slot(ctx, 0) if ctx.needs_input_grad[0] else None
        dx, *rest = _cbe_bwd(st, da, ds, need_x=ctx.needs_input_grad[0],
                             need_b=ctx.needs_input_grad[2], dx=tgt,
                             dx_accumulate=tgt is not None)
        st.saved = None
        return (_give(ctx, 0, dx), *rest, None)


def conv_bn_elu(x, conv, bn, pad, pad_mode, se=None, elu=True, segs=None):
    """Conv2d -> BatchNorm2d (train: batch stats; eval: running stats; None:
    identity) -> ELU [-> SE gate].  Returns a, or (a, gate) with ``se``.
    ``segs``: input-channel placement of a concat input (see ``concat``)."""
    spec = ConvSpec(conv, bn, pad, pad_mode, elu, segs)
    w1 = se.excite[0].weight if se is not None else None
    w2 = se.excite[2].weight if se is not None else None
    affine = bn is not None and bn.affine
    return ConvBNELUFn.apply(x, conv.weight, conv.bias,
                             bn.weight if affine else None, bn.bias if affine else None,
                             w1, w2, spec)


# ------------------------------------------------ decoder skip 1x1 conv --
class SkipConvFn(torch.autograd.Function):
    """DecoderStage's squeeze-excite ConvELUBlock on cat(feature_map,
    interpolate(skip, x2) * gate) (reference model/layers/decoder.py:228-238,
    :55-87, :90-136) without the full-resolution concat: a 1x1 conv and the
    bilinear x2 upsample are both linear and act on different axes, so

        W [fm | up2(g*skip)] = W_f fm + up2(W_s (g*skip))

    The skip half is convolved at the skip's (quarter) pixel count into a
    map z (stored like the pre-BN y), and um_conv2d_fwd_up2 writes up2(z)
    into y and accumulates the feature-map half onto it (the BN statistics
    are taken on the sum).  Backward: t = up2^T(dy) at
    the low resolution, dW_s = t (x) (g*skip), d(g*skip) = W_s^T t, the gate
    adjoint as the concat's; dW_f and d fm at full resolution."""

    @staticmethod
    def forward(ctx, fm, skip, gate, weight, bias, gamma, beta, w1, w2, spec: ConvSpec,
                fin: int, skin: int):
        L.require_device(fm)
        N, H, W, Cf = fm.shape
        _, h, w, Cs = skip.shape
        K = weight.shape[0]
        dt = fm.dtype
        # g * skip at the low resolution (one gated copy)
        gs = _gated_copy(skip, gate, skin) if gate is not None else skip
        Cg = gs.shape[-1]
        wf_s, wT_s = _pack(weight, Cg, dt, segs=[(fin, 0, skin)])
        wf_f, wT_f = _pack(weight, Cf, dt, segs=[(0, 0, fin)])
        ydt = _ydtype(dt)
        z = _conv_fwd(gs, wf_s, None, K, 1, 1, 0, L.PAD_ZERO, out_dtype=ydt, creal=skin)

        def yconv(epi, stats, cbias):
            y = torch.empty((N, H, W, K), dtype=ydt, device=fm.device)
            call('um_conv2d_fwd_up2', _dt(fm) | (L.Y_ACT if ydt != torch.float32 else 0), N, H, W, Cf, Cf, ptr(fm), ptr(wf_f), ptr(cbias),
                 K, H, W, ptr(y), K, epi, ptr(stats), ptr(z), h, w, K,
                 work=_conv_flops(N, H, W, K, 1, fin))  # the z conv is its own launch
            return y

        outs, st = _cbe_fwd(fm, weight, bias, gamma, beta, w1, w2, spec, yconv=yconv)
        x_, _, y, mean, invstd, scale, shift, gamma_, w1_, w2_ = st.saved
        st.saved = None
        ctx.st = st
        ctx.geo = (N, H, W, Cf, h, w, Cg, K, fin, skin)
        _use(ctx, fm, skip, gate)
        ctx.save_for_backward(fm, skip, gate, gs, wT_s, wT_f, y, mean, invstd, scale, shift,
                              gamma_, w1_, w2_)
        return outs if len(outs) > 1 else outs[0]

    @staticmethod
    def backward(ctx, da, ds=None):
        (fm, skip, gate, gs, wT_s, wT_f, y, mean, invstd, scale, shift, gamma, w1,
         w2) = ctx.saved_tensors
        N, H, W, Cf, h, w, Cg, K, fin, skin = ctx.geo
        st = ctx.st
        st.saved = (fm, None, y, mean, invstd, scale, shift, gamma, w1, w2)
        need_fm, need_skip = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        need_gate = gate is not None and ctx.needs_input_grad[2]
        res = {}

        def conv_bwd(dy):
            dW = torch.empty((K, fin + skin, 1, 1), dtype=torch.float32, device=dy.device)
            _conv_wgrad(fm, dy, K, K, fin + skin, 1, 1, 0, L.PAD_ZERO, dw=dW,
                        segs=[(0, 0, fin)])
            # t = up2^T(dy): the concat adjoint of an UP2 source with K channels
            t = torch.empty((N, h, w, K), dtype=dy.dtype, device=dy.device)
            src = L.CatSrc(t.data_ptr(), None, K, K, L.CAT_UP2, 0, _dt(t), h, w)
            call('um_concat_bwd_src', _dt(dy), N, H, W, ptr(dy), K, _ct.byref(src), ptr(t), K,
                 _dt(t), 0, None, None)
            _conv_wgrad(gs, t, K, K, fin + skin, 1, 1, 0, L.PAD_ZERO, dw=dW,
                        segs=[(fin, 0, skin)])
            if need_skip or need_gate:
                tgt = _slot(ctx, 1) if need_skip else None
                if gate is None:
                    res['skip'] = _conv_dgrad(t, wT_s, (N, h, w, Cg), K, 1, 1, 0, L.PAD_ZERO,
                                              dx=tgt, accumulate=tgt is not None, creal=skin)
                else:
                    dgs = _conv_dgrad(t, wT_s, (N, h, w, Cg), K, 1, 1, 0, L.PAD_ZERO,
                                      creal=skin)
                    res['skip'], res['gate'] = _gated_copy_bwd(
                        dgs, skip, gate, skin, need_skip, need_gate, dsk=tgt,
                        dg=_slot(ctx, 2) if need_gate else None)
                    res['gate'] = _give(ctx, 2, res['gate'])
                res['skip'] = _give(ctx, 1, res['skip'])
            dfm = None
            if need_fm:
                tgt = _slot(ctx, 0)
                dfm = _give(ctx, 0, _conv_dgrad(dy, wT_f, (N, H, W, Cf), K, 1, 1, 0, L.PAD_ZERO,
                                                dx=tgt, accumulate=tgt is not None, creal=fin))
            return dfm, dW

        dfm, dW, dbias, dgamma, dbeta, dw1, dw2 = _cbe_bwd(
            st, da, ds, need_x=need_fm, need_b=ctx.needs_input_grad[4], conv_bwd=conv_bwd)
        st.saved = None
        return (dfm, res.get('skip'), res.get('gate'), dW, dbias, dgamma, dbeta, dw1, dw2,
                None, None, None)


def _gated_copy(skip, gate, C):
    """g * skip (per (n, c) gate) as one concat-build launch"""
    N, h, w, _ = skip.shape
    src = (L.CatSrc * 1)(L.CatSrc(skip.data_ptr(), gate.data_ptr(), C, skip.shape[-1],
                                  L.CAT_COPY, 0, _dt(skip), h, w))
    Ct = ceil8(C)
    out = torch.empty((N, h, w, Ct), dtype=skip.dtype, device=skip.device)
    call('um_concat_build', _dt(out), N, h, w, ptr(out), Ct, Ct, 1, src)
    return out


def _gated_copy_bwd(dgs, skip, gate, C, need_skip, need_gate, dsk=None, dg=None):
    """adjoint of _gated_copy: (d skip, d gate); ``dsk`` / ``dg``: accumulate
    into these tensors (else fresh ones are written)"""
    N, h, w, Ct = dgs.shape
    s = L.CatSrc(skip.data_ptr(), gate.data_ptr(), C, skip.shape[-1], L.CAT_COPY, 0, _dt(skip),
                 h, w)
    acc = int(dsk is not None) | (2 if need_gate and dg is None else 0)
    if need_skip and dsk is None:
        dsk = torch.empty_like(skip)
    if need_gate and dg is None:
        dg = torch.empty_like(gate)
    ws = None
    if need_gate:
        ws = torch.empty((query('um_concat_bwd_ws', N, h, w, C),), dtype=torch.float32,
                         device=dgs.device)
    call('um_concat_bwd_src', _dt(dgs), N, h, w, ptr(dgs), Ct, _ct.byref(s),
         ptr(dsk) if need_skip else None, skip.shape[-1], _dt(skip), acc, ptr(dg), ptr(ws))
    return (dsk if need_skip else None), dg


_SKIP_CONV = os.environ.get('UMAMD_SKIP_CONV', '1') == '1'


def skip_conv_bn_elu(feature_map, skip, gate, conv, bn, se, fin: int, skin: int):
    """ConvELUBlock(1x1, BN) [+ SE] on cat(feature_map, up2(skip) * gate)
    (see SkipConvFn); returns (a, s) with ``se`` like conv_bn_elu."""
    spec = ConvSpec(conv, bn, 0, L.PAD_ZERO, True, None)
    w1 = se.excite[0].weight if se is not None else None
    w2 = se.excite[2].weight if se is not None else None
    affine = bn is not None and bn.affine
    return SkipConvFn.apply(feature_map, skip, gate, conv.weight, conv.bias,
                            bn.weight if affine else None, bn.bias if affine else None, w1, w2,
                            spec, int(fin), int(skin))


# -------------------------------------------------------------------- merge --
class MergeFn(torch.autograd.Function):
    """out = sum_i c_i * src_i with c_i = sigmoid(w[widx[i]]) (w given) or the
    constant coefs[i] (w None: GraphBlock output-node average)."""

    @staticmethod
    def forward(ctx, w, widx: List[int], coefs, *srcs):
        out = torch.empty_like(srcs[0])
        n = len(srcs)
        arr = (ctypes_p * n)(*[s.data_ptr() for s in srcs])
        idx = (ctypes_i * n)(*widx)
        cf = (ctypes_f * n)(*coefs) if coefs is not None else None
        call('um_merge_fwd', _dt(out), n, arr, idx, ptr(w), cf, out.numel(), ptr(out))
        ctx.widx = list(widx)
        ctx.coefs = coefs
        ctx.has_w = w is not None
        ctx.save_for_backward(w, *srcs)
        return out

    @staticmethod
    def backward(ctx, dm):
        w, *srcs = ctx.saved_tensors
        n = len(srcs)
        dm = dm.contiguous()
        dsrcs = [torch.empty_like(s) if ctx.needs_input_grad[3 + i] else None
                 for i, s in enumerate(srcs)]
        need_w = ctx.has_w and ctx.needs_input_grad[0]
        nparts = query('um_merge_parts', dm.numel())
        parts = torch.empty((nparts, n), dtype=torch.float32, device=dm.device) if need_w else None
        arr = (ctypes_p * n)(*[s.data_ptr() for s in srcs])
        darr = (ctypes_p * n)(*[d.data_ptr() if d is not None else None for d in dsrcs])
        acc = (ctypes_i * n)(*([0] * n))
        idx = (ctypes_i * n)(*ctx.widx)
        cf = (ctypes_f * n)(*ctx.coefs) if ctx.coefs is not None else None
        call('um_merge_bwd', _dt(dm), n, arr, darr, acc, idx, ptr(w), cf, dm.numel(), ptr(dm),
             ptr(parts))
        dw = None
        if need_w:
            dw = torch.empty_like(w, dtype=torch.float32)
            args = (ptr(parts), nparts, n, idx, ptr(w), ptr(dw), w.numel(), 0)
            _param_grad((parts, w), dw, lambda: call('um_merge_wgrad', *args))
        return (dw, None, None, *dsrcs)


import ctypes as _ct  # noqa: E402

ctypes_p = _ct.c_void_p
ctypes_i = _ct.c_int
ctypes_f = _ct.c_float


def merge(inputs: Sequence[torch.Tensor], w: Optional[torch.Tensor], widx: Sequence[int],
          coefs: Optional[Sequence[float]] = None):
    if len(inputs) == 1 and w is None and coefs is None:
        return inputs[0]
    return MergeFn.apply(w, list(widx), list(coefs) if coefs is not None else None, *inputs)


# -------------------------------------------------------------- graph block --
_STAGE_FN = os.environ.get('UMAMD_STAGE_FN', '1') == '1'
# a GraphBlock node's merge computed by the BN pass of its last predecessor
_FUSED_MERGE = os.environ.get('UMAMD_FUSED_MERGE', '1') == '1'


class GraphSpec:
    """Static description of a GraphBlock (reference model/layers/encoder.py
    :130-198) for GraphBlockFn: node order, predecessors (adjacency order,
    F3 weight map), output nodes, one ConvSpec per node and the flat
    parameter layout [conv.weight, conv.bias, bn.weight, bn.bias,
    (mean_weight)] per node."""

    def __init__(self, block):
        self.nodes = [list(node.inputs) for node in block.nodes]
        self.out_nodes = list(block.out_nodes)
        self.specs, self.params, self.slices, self.widx = [], [], [], []
        for nb, preds in zip(block.node_blocks, self.nodes):
            conv, bn = nb.convolution.layers[0], nb.convolution.layers[1]
            self.specs.append(ConvSpec(conv, bn, nb.convolution.padding[0], L.PAD_ZERO))
            ps = [conv.weight, conv.bias, bn.weight if bn.affine else None,
                  bn.bias if bn.affine else None]
            if nb.mean_weight is not None:
                ps.append(nb.mean_weight)
            self.slices.append((len(self.params), len(ps)))
            self.params += ps
            self.widx.append([0] + list(range(len(preds) - 1)))
        # node p -> the first multi-input node s whose last predecessor (in
        # id order, the evaluation order) is p: s's merge is fused into p's
        # BN apply pass (umamd.functional._cbe_fwd, um_bn_elu_fwd_slots_merge)
        self.merge_after = {}
        for s, preds in enumerate(self.nodes):
            if len(preds) > 1 and len(preds) <= 8 and max(preds) < s:
                self.merge_after.setdefault(max(preds), s)
        # node p -> its lowest-id successor: in the reverse-id backward that
        # successor's input gradient is the last one added to p's, so a merge
        # backward there completes p's gradient (um_merge_bwd_bn)
        self.last_consumer = {}
        for s, preds in enumerate(self.nodes):
            for p in preds:
                if p not in self.last_consumer or s < self.last_consumer[p]:
                    self.last_consumer[p] = s


def _merge_launch(srcs, w, widx, coefs, out):
    n = len(srcs)
    arr = (ctypes_p * n)(*[t.data_ptr() for t in srcs])
    idx = (ctypes_i * n)(*widx)
    cf = (ctypes_f * n)(*coefs) if coefs is not None else None
    call('um_merge_fwd', _dt(out), n, arr, idx, ptr(w), cf, out.numel(), ptr(out))
    return out


class GraphBlockFn(torch.autograd.Function):
    """A whole GraphBlock as one autograd node.  Forward: every node's
    weighted predecessor merge (F3) and conv+BN+ELU in id order, the output
    nodes averaged out of place (F4).  Backward in reverse id order, where
    every node's gradient is complete once its (higher-id) successors are
    done: each node's input gradient is written or ADDED straight into its
    predecessors' gradient buffers -- the data-gradient GEMM accumulates
    into a single predecessor, the merge backward's per-source accumulate
    flags into several -- so no autograd gradient sums (one elementwise add
    launch per extra consumer of a node output: 6 per K5 stage) are left."""

    @staticmethod
    def forward(ctx, gs: GraphSpec, x, *params):
        a, states, merged = [], [], {}
        for j, preds in enumerate(gs.nodes):
            o, n = gs.slices[j]
            w, b, g, be = params[o:o + 4]
            mw = params[o + 4] if n > 4 else None
            if not preds:
                inp = x
            elif len(preds) == 1:
                inp = a[preds[0]]
            elif j in merged:  # computed by the BN pass of its last predecessor
                inp = merged.pop(j)
            else:
                inp = _merge_launch([a[p] for p in preds], mw, gs.widx[j], None,
                                    torch.empty_like(a[preds[0]]))
            mg, s = None, gs.merge_after.get(j)
            if s is not None:  # node s's merge rides in this node's BN pass
                so = gs.slices[s][0]
                mg = ([None if p == j else a[p] for p in gs.nodes[s]], gs.widx[s], params[so + 4])
            outs, st = _cbe_fwd(inp, w, b, g, be, None, None, gs.specs[j], merge=mg)
            if s is not None:
                merged[s], st.merged = st.merged, None
            a.append(outs[0])
            states.append(st)
        if len(gs.out_nodes) == 1:
            out = a[gs.out_nodes[0]]
        else:
            k = len(gs.out_nodes)
            out = _merge_launch([a[o] for o in gs.out_nodes], None, [0] * k, [1.0 / k] * k,
                                torch.empty_like(a[gs.out_nodes[0]]))
        ctx.gspec, ctx.a, ctx.states = gs, a, states
        _use(ctx, x)
        return out

    @staticmethod
    def backward(ctx, dout):
        gs, a, states = ctx.gspec, ctx.a, ctx.states
        dout = dout.contiguous()
        if dout.dtype != a[0].dtype:
            dout = dout.to(a[0].dtype)
        da = {}
        outs = gs.out_nodes
        if len(outs) == 1:
            da[outs[0]] = dout
        else:  # out = mean of the output nodes: each gets dout / k
            k = len(outs)
            bufs = [torch.empty_like(a[o]) for o in outs]
            arr = (ctypes_p * k)(*[a[o].data_ptr() for o in outs])
            darr = (ctypes_p * k)(*[t.data_ptr() for t in bufs])
            call('um_merge_bwd', _dt(dout), k, arr, darr, (ctypes_i * k)(*([0] * k)),
                 (ctypes_i * k)(*([0] * k)), None, (ctypes_f * k)(*([1.0 / k] * k)),
                 dout.numel(), ptr(dout), None)
            for o, t in zip(outs, bufs):
                da[o] = t
        grads = [None] * len(gs.params)
        need_x = ctx.needs_input_grad[1]
        dx_stage = _slot(ctx, 0) if need_x else None  # accumulate into another consumer's
        for j in reversed(range(len(gs.nodes))):
            preds = gs.nodes[j]
            o, n = gs.slices[j]
            g = da.pop(j)
            st = states[j]
            if not preds:
                if need_x:
                    dx, *pg = _cbe_bwd(st, g, None, True, True, dx=dx_stage,
                                       dx_accumulate=dx_stage is not None)
                    dx_stage = dx
                else:
                    _, *pg = _cbe_bwd(st, g, None, False, True)
            elif len(preds) == 1:
                p = preds[0]
                acc = p in da
                dx, *pg = _cbe_bwd(st, g, None, True, True, dx=da.get(p), dx_accumulate=acc)
                da[p] = dx
            else:
                dm, *pg = _cbe_bwd(st, g, None, True, True)
                k = len(preds)
                acc = [int(p in da) for p in preds]
                for p in preds:
                    if p not in da:
                        da[p] = torch.empty_like(a[p])
                mw = gs.params[o + 4]
                need_w = ctx.needs_input_grad[2 + o + 4]
                fs = _merge_bn_target(gs, j, preds, states, a)
                nparts = query('um_merge_parts' if fs is None else 'um_merge_bn_parts', dm.numel())
                parts = torch.empty((nparts, k), dtype=torch.float32, device=dm.device) \
                    if need_w else None
                idx = (ctypes_i * k)(*gs.widx[j])
                srcs = (ctypes_p * k)(*[a[p].data_ptr() for p in preds])
                dsrcs = (ctypes_p * k)(*[da[p].data_ptr() for p in preds])
                if fs is not None:
                    # this merge completes pred fs's gradient: take its BN-backward
                    # sums here (its reduce launch and re-read of da are skipped)
                    sp = states[preds[fs]]
                    y_p, mean_p, invstd_p, scale_p, shift_p = sp.saved[2:7]
                    call('um_merge_bwd_bn', _ydt(a[preds[fs]], y_p), k, srcs, dsrcs,
                         (ctypes_i * k)(*acc), idx, ptr(mw), None, dm.numel(), ptr(dm),
                         ptr(parts), fs, ptr(y_p), y_p.shape[-1], ptr(mean_p), ptr(invstd_p),
                         ptr(scale_p), ptr(shift_p), int(sp.spec.elu), ptr(sp.slots_b))
                    sp.prereduced = True
                else:
                    call('um_merge_bwd', _dt(dm), k, srcs, dsrcs, (ctypes_i * k)(*acc), idx,
                         ptr(mw), None, dm.numel(), ptr(dm), ptr(parts))
                if need_w:
                    dmw = torch.empty(mw.shape, dtype=torch.float32, device=dm.device)
                    if _MWG_BATCH and _overlap.active() is not None and k <= L.MWG_SRC:
                        # one um_merge_wgrad_batch launch per side-stream flush
                        d = L.MwgDesc()
                        d.parts, d.w, d.dw = parts.data_ptr(), mw.data_ptr(), dmw.data_ptr()
                        d.nparts, d.nsrc, d.nw, d.accumulate = nparts, k, mw.numel(), 0
                        for q, wi in enumerate(gs.widx[j]):
                            d.widx[q] = wi
                        grads[o + 4] = _param_grad((parts, mw), dmw,
                                                   lambda d=d, keep=parts: (keep, d))
                    else:
                        grads[o + 4] = _param_grad(
                            (parts, mw), dmw,
                            lambda a=(ptr(parts), nparts, k, idx, ptr(mw), ptr(dmw), mw.numel()):
                            call('um_merge_wgrad', *a, 0))
            dW, dbias, dgamma, dbeta = pg[0], pg[1], pg[2], pg[3]
            grads[o], grads[o + 1], grads[o + 2], grads[o + 3] = dW, dbias, dgamma, dbeta
            states[j] = None  # release this node's saved tensors
        ctx.a = ctx.states = None
        grads = [gr if p is not None else None for gr, p in zip(grads, gs.params)]
        return (None, _give(ctx, 0, dx_stage), *grads)


# a GraphBlock node's BN-backward statistics taken by the merge backward that
# completes its gradient (um_merge_bwd_bn); UMAMD_MERGE_BN_REDUCE=0 keeps the
# separate reduce launch
_MERGE_BN_REDUCE = os.environ.get('UMAMD_MERGE_BN_REDUCE', '1') == '1'


def _merge_bn_target(gs, j, preds, states, a):
    """index (into preds) of the predecessor whose gradient node j's merge
    backward completes and whose BN backward can take its sums there, or None"""
    if not _MERGE_BN_REDUCE:
        return None
    for q, p in enumerate(preds):
        if gs.last_consumer.get(p) != j or p in gs.out_nodes:
            continue
        st = states[p]
        if st is None or not st.has_bn or st.slots_b is None or st.se is not None:
            continue
        if st.sync is not None and st.sync.collective:
            continue
        C = a[p].shape[-1]
        if st.saved[2].shape[-1] != C or C % 8 or C > 512 or 256 % (C // 8):
            continue
        return q
    return None


def graph_block(x, block):
    """GraphBlock forward (NHWC) as one GraphBlockFn node (UMAMD_STAGE_FN=0:
    per-node autograd functions, the round-2 path)."""
    gs = GraphSpec(block)
    return GraphBlockFn.apply(gs, x, *gs.params)


# ---------------------------------------------------------------- attention --
class AttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wk, bk, wq, bq, wv, bv, wr, br, heads: int):
        L.require_device(x)
        N, H, W, C = x.shape
        S = H * W
        dt = x.dtype
        dev = x.device
        pk = _packer.active() or _packer.WeightPacker()
        # rows [iC, (i+1)C) of wf; columns [iC, (i+1)C) of wT (row stride 3C)
        wf, wT = pk.pack_rows((wk, wq, wv), C, dt)
        bqkv = pk.pack_bias((bk, bq, bv), C)  # refreshed by the per-forward batch launch
        qkv = _conv_fwd(x, wf, bqkv, 3 * C, 1, 1, 0, L.PAD_ZERO)
        kmax = torch.empty((N, C), dtype=torch.float32, device=dev)
        ksum = torch.empty_like(kmax)
        ctxm = torch.empty((N, heads, (C // heads) ** 2), dtype=torch.float32, device=dev)
        wsn = max(query('um_attn_ws_kstats', N, S, C), query('um_attn_ws_ctx', N, S, C, heads))
        ws = torch.empty(wsn, dtype=torch.float32, device=dev)
        att = torch.empty((N, H, W, C), dtype=dt, device=dev)
        call('um_attn_fwd', L.dtype_code(dt), N, S, C, heads, ptr(qkv), 3 * C, ptr(kmax),
             ptr(ksum), ptr(ctxm), ptr(ws), ptr(att), C)
        wrf, wrT = _pack(wr, C, dt)
        out = _conv_fwd(att, wrf, br.detach().float().contiguous(), C, 1, 1, 0, L.PAD_ZERO,
                        epi=L.EPI_RESIDUAL, residual=x)
        ctx.heads = heads
        ctx.save_for_backward(x, qkv, kmax, ksum, ctxm, att, wT, wrT)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, qkv, kmax, ksum, ctxm, att, wT, wrT = ctx.saved_tensors
        heads = ctx.heads
        N, H, W, C = x.shape
        S = H * W
        dev = x.device
        dt = x.dtype
        dout = dout.contiguous()
        datt = _conv_dgrad(dout, wrT, (N, H, W, C), C, 1, 1, 0, L.PAD_ZERO)
        dwr = _conv_wgrad(att, dout, C, C, C, 1, 1, 0, L.PAD_ZERO)
        dbr = _colsum_grad(dout, C)
        dqkv = torch.empty((N, H, W, 3 * C), dtype=dt, device=dev)
        dks = torch.empty((N * S, C), dtype=torch.float32, device=dev)
        ws = torch.empty(query('um_attn_ws_tiles', N, S, C, heads), dtype=torch.float32,
                         device=dev)
        dctx = torch.empty_like(ctxm)
        r = torch.empty((N, C), dtype=torch.float32, device=dev)
        call('um_attn_bwd', L.dtype_code(dt), N, S, C, heads, ptr(qkv), 3 * C, ptr(kmax),
             ptr(ksum), ptr(ctxm), ptr(datt), C, ptr(dqkv), 3 * C, ptr(dks), ptr(ws), ptr(dctx),
             ptr(r))
        dwqkv = _conv_wgrad(x, dqkv, 3 * C, 3 * C, C, 1, 1, 0, L.PAD_ZERO)
        dbqkv = _colsum_grad(dqkv, 3 * C)
        if dout.dtype == dt:
            # dx = dout (the residual path) + the K/Q/V convs' input gradient:
            # wT [C][3C] is the weight of a 3C -> C 1x1 conv, so this is one
            # forward GEMM with the residual epilogue (no copy of dout first)
            dx = _conv_fwd(dqkv, wT, None, C, 1, 1, 0, L.PAD_ZERO, epi=L.EPI_RESIDUAL,
                           residual=dout)
        else:
            dx = dout.to(dt)
            _conv_dgrad(dqkv, wT, (N, H, W, C), 3 * C, 1, 1, 0, L.PAD_ZERO, dx=dx,
                        accumulate=True)
        return (dx, dwqkv[:C], dbqkv[:C], dwqkv[C:2 * C], dbqkv[C:2 * C], dwqkv[2 * C:],
                dbqkv[2 * C:], dwr, dbr, None)


def attention_block(x, att_module):
    m = att_module
    return AttentionFn.apply(x, m.keys.weight, m.keys.bias, m.queries.weight, m.queries.bias,
                             m.values.weight, m.values.bias, m.reprojection.weight,
                             m.reprojection.bias, m.head_size)


# ------------------------------------------------------------------- concat --
class CatSource:
    """A concat input: tensor (NHWC), op, optional gate [N][C] f32."""

    def __init__(self, t: torch.Tensor, op: int, C: int, gate: Optional[torch.Tensor] = None):
        self.t, self.op, self.C, self.gate = t, op, C, gate


class ConcatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, meta, *tensors):
        # meta: list of (op, C, has_gate); tensors: src0, [gate0], src1, ...
        N, H, W, Ctot, dtype = meta['out']
        srcs, it = [], iter(tensors)
        structs = (L.CatSrc * len(meta['srcs']))()
        saved = []
        for i, (op, C) in enumerate(meta['srcs']):
            t = next(it)
            g = next(it) if meta['gates'][i] else None
            srcs.append((t, g))
            h, w = (H, W) if op == L.CAT_COPY else (H // 2, W // 2)
            structs[i] = L.CatSrc(t.data_ptr(), g.data_ptr() if g is not None else None, C,
                                  t.shape[-1], op, meta['coffs'][i], _dt(t), h, w)
            saved += [t] + ([g] if g is not None else [])
        out = torch.empty((N, H, W, Ctot), dtype=dtype, device=tensors[0].device)
        call('um_concat_build', L.dtype_code(dtype), N, H, W, ptr(out), Ctot, Ctot,
             len(srcs), structs)
        ctx.meta = meta
        # slot-able inputs: the sources (0..n-1), then the gates in source order
        _use(ctx, *[t for t, _ in srcs], *[gt for _, gt in srcs if gt is not None])
        ctx.save_for_backward(*saved)
        return out

    @staticmethod
    def backward(ctx, g):
        meta = ctx.meta
        N, H, W, Ctot, dtype = meta['out']
        g = g.contiguous()
        saved = list(ctx.saved_tensors)
        grads = []
        k = 1  # index into needs_input_grad (0 = meta)
        gi = len(meta['srcs'])  # slot index of the next gate
        for i, (op, C) in enumerate(meta['srcs']):
            coff = meta['coffs'][i]
            t = saved.pop(0)
            gate = saved.pop(0) if meta['gates'][i] else None
            need_t = ctx.needs_input_grad[k]
            need_g = gate is not None and ctx.needs_input_grad[k + 1]
            h, w = (H, W) if op == L.CAT_COPY else (H // 2, W // 2)
            s = L.CatSrc(t.data_ptr(), gate.data_ptr() if gate is not None else None, C,
                         t.shape[-1], op, coff, _dt(t), h, w)
            tgt = _slot(ctx, i) if need_t else None
            dt_ = (tgt if tgt is not None else torch.empty_like(t)) if need_t else None
            gslot = gi
            if gate is not None:
                gi += 1
            gtgt = _slot(ctx, gslot) if need_g else None
            # the gate gradient is written (flag bit 1) unless it accumulates
            # into another consumer's (no zero fill)
            dg = (gtgt if gtgt is not None else torch.empty_like(gate)) if need_g else None
            if need_t or need_g:
                ws = None
                if need_g:
                    nws = query('um_concat_bwd_ws', N, s.h, s.w, s.C)
                    ws = torch.empty((nws,), dtype=torch.float32, device=g.device)
                flags = int(tgt is not None) | (2 if need_g and gtgt is None else 0)
                call('um_concat_bwd_src', L.dtype_code(dtype), N, H, W, ptr(g), Ctot,
                     _ct.byref(s), ptr(dt_), t.shape[-1], _dt(t), flags, ptr(dg), ptr(ws))
            grads.append(_give(ctx, i, dt_))
            if gate is not None:
                grads.append(_give(ctx, gslot, dg))
            k += 2 if gate is not None else 1
        return (None, *grads)


def concat(sources: Sequence[CatSource], N, H, W, dtype):
    """Materialise a decoder concat.  Every source starts at an 8-aligned
    channel offset (vector loads/stores); returns (tensor, segs) where segs
    maps the reference's input channels of the consuming conv to the packed
    channels ([(ref_c0, packed_c0, len)], None when identical)."""
    coffs, segs, ref, off = [], [], 0, 0
    for s in sources:
        coffs.append(off)
        segs.append((ref, off, s.C))
        ref += s.C
        off = ceil8(off + s.C)
    Ctot = ceil8(coffs[-1] + sources[-1].C)
    if all(a == b for a, b, _ in segs):
        segs = None
    meta = {'out': (N, H, W, Ctot, dtype), 'srcs': [(s.op, s.C) for s in sources],
            'gates': [s.gate is not None for s in sources], 'coffs': coffs}
    tensors = []
    for s in sources:
        tensors.append(s.t)
        if s.gate is not None:
            tensors.append(s.gate)
    return ConcatFn.apply(meta, *tensors), segs


# ---------------------------------------------------------------- disp head --
# the heads' weights in split bf16 (hi + lo rows, um_pack_weight_split): the
# bf16 rounding of these 4-output weights moves the uncertainty sigma of
# every pixel the same way (a systematic error; the activation roundings
# average out over the pixels), and the Laplacian NLL e/sigma + log sigma is
# as sensitive to it as to sigma itself.  Measured at BASELINE config 2
# (tools/bf16_arms.py, step-0 error loss vs the reference): 1.9e-3 -> 1.2e-3.
# The 4 outputs pad to 8 GEMM columns anyway, so the split rows are free.
_SPLIT_HEAD = os.environ.get('UMAMD_SPLIT_HEAD', '1') == '1'
# round 6: the split heads on the one-pass kernels of csrc/disphead.hip
# (UMAMD_ONEPASS_HEAD=0: the implicit-GEMM path of rounds 4-5)
_ONEPASS_HEAD = os.environ.get('UMAMD_ONEPASS_HEAD', '1') == '1'


class DispHeadFn(torch.autograd.Function):
    """disp = scale * sigmoid(Conv3x3reflect(x)) (reference
    model/layers/decoder.py:244-247), all 4 channels."""

    @staticmethod
    def forward(ctx, x, weight, bias, scale: float):
        N, H, W, Cp = x.shape
        K, Creal, R, _ = weight.shape
        Kp = ceil8(K)
        bias_f = bias.detach().float().contiguous()
        split = _SPLIT_HEAD and x.dtype == torch.bfloat16 and 2 * K <= Kp
        # the one-pass head kernels (csrc/disphead.hip): split weights, 4
        # outputs, 3x3 reflect, C in {32..256}
        onepass = split and _ONEPASS_HEAD and K == 4 and R == 3 and Kp == 8 and \
            query('um_disp_head_ok', N, H, W, Cp, Cp) == 1
        if split:
            wf, wT = _pack(weight, Cp, x.dtype, ldT=Kp, split=True)
            d = torch.empty((N, H, W, K), dtype=torch.float32, device=x.device)
            if onepass:
                call('um_disp_head_fwd', N, H, W, Cp, ptr(x), Cp, ptr(wf), ptr(bias_f),
                     float(scale), ptr(d), K, work=_conv_flops(N, H, W, K, R, Creal))
            else:
                z = _conv_fwd(x, wf, None, 2 * K, R, 1, 1, L.PAD_REFLECT,
                              out_dtype=torch.float32, creal=Creal)
                call('um_head_split_fin', N * H * W, K, ptr(z), 2 * K, ptr(bias_f),
                     float(scale), ptr(d), K)
            # the GEMM's algorithmic work is the 4-output conv (the split
            # rows are padding columns of the same MFMA tiles)
        else:
            wf, wT = _pack(weight, Cp, x.dtype, ldT=Kp)
            d = _conv_fwd(x, wf, bias_f, K, R, 1, 1, L.PAD_REFLECT, out_dtype=torch.float32,
                          epi=L.EPI_SIGMOID_SCALE, epi_scale=scale, creal=Creal)
        ctx.scale = float(scale)
        ctx.split = split
        ctx.onepass = onepass if split else False
        _use(ctx, x)
        ctx.save_for_backward(x, wT, d)
        ctx.geom = (K, Kp, Creal, R)
        return d

    @staticmethod
    def backward(ctx, dd):
        x, wT, d = ctx.saved_tensors
        K, Kp, Creal, R = ctx.geom
        N, H, W, Cp = x.shape
        dd = dd.contiguous().float()
        M = N * H * W
        dl = torch.empty((N, H, W, Kp), dtype=x.dtype, device=x.device)
        # split: dlogit also in channels K..2K-1, so that the data gradient
        # over the split rows of wT sums dl (w_hi + w_lo)
        call('um_sigmoid_scale_bwd_split' if ctx.split else 'um_sigmoid_scale_bwd', _dt(dl), M,
             K, ptr(d), K, ptr(dd), dd.shape[-1], ctx.scale, ptr(dl), Kp)
        dW = _conv_wgrad(x, dl, Kp, K, Creal, R, 1, 1, L.PAD_REFLECT)  # rows K.. unused
        db = _colsum_grad(dl, Kp)[:K]  # channels K..Kp of dl are zero or a copy
        dx = None
        if ctx.needs_input_grad[0]:
            tgt = _slot(ctx, 0)
            if ctx.onepass:
                dx = tgt if tgt is not None else torch.empty((N, H, W, Cp), dtype=x.dtype,
                                                             device=x.device)
                call('um_disp_head_dgrad', N, H, W, Cp, ptr(dl), Kp, ptr(wT), ptr(dx), Cp,
                     int(tgt is not None), work=_conv_flops(N, H, W, K, R, Creal))
                dx = _give(ctx, 0, dx)
            else:
                dx = _give(ctx, 0, _conv_dgrad(dl, wT, (N, H, W, Cp), Kp, R, 1, 1,
                                               L.PAD_REFLECT, dx=tgt,
                                               accumulate=tgt is not None, creal=Creal,
                                               kreal=K))
        return dx, dW, db, None


def disp_head(x, conv, scale):
    return DispHeadFn.apply(x, conv.weight, conv.bias, float(scale))


# ------------------------------------------------------------------- inputs --
def image_to_nhwc(img: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """[N,C,H,W] f32 (any strides) -> NHWC [N,H,W,ceil8(C)] in ``dtype``."""
    L.require_device(img)
    x = img.detach()
    if x.dtype != torch.float32 or not x.is_contiguous():
        x = x.float().contiguous()
    N, C, H, W = x.shape
    Cp = ceil8(C)
    out = torch.empty((N, H, W, Cp), dtype=dtype, device=x.device)
    call('um_image_to_nhwc', L.dtype_code(dtype), ptr(x), N, C, H, W, Cp, ptr(out))
    return out
