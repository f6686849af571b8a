"""Weight gradients on a side HIP stream, overlapped with the data-gradient
chain of the backward pass.

In the reference backward (autograd over nn.Conv2d, train/train.py:126) each
conv's weight gradient and data gradient run back to back.  Only the data
gradient is on the critical path: the next layer's backward needs dx, while
dW is consumed by the optimiser after the whole backward.  Inside
``WgradStream`` every ``functional._conv_wgrad`` (the weight-gradient kernel
+ its slab reduce) is issued on a side stream that first waits for the
launch stream (dy is ready there), so it runs beside the following BN/dgrad
kernels, which under-fill the chip at this model's channel counts.  Leaving
the context joins the side stream back into the launch stream, before the
optimiser reads the gradients.

Inside a HIP graph capture the fork/join becomes parallel graph branches.
Tensors the side stream reads (x, dy) are marked with ``record_stream`` so
the caching allocator does not hand their memory to the launch stream while
the side stream still reads it (during capture it defers those frees to the
end of capture).

Used by ``train.graph.CapturedTrainStep``, whose data-parallel gradient
all-reduce runs after the join (DDP's per-bucket hooks would read gradients
before the side stream wrote them, so the eager DDP step does not use it).
"""
from __future__ import annotations

import os
from typing import Optional

import torch


class WgradStream:
    _active: Optional['WgradStream'] = None

    def __init__(self, params=(), batch=None):
        """``params``: the leaves whose gradients the backward produces.
        They must have ``.grad is None`` on entry (``zero_grad(set_to_none=
        True)``): AccumulateGrad then stores the side-stream tensor without a
        launch-stream kernel reading it before the join."""
        self.stream = torch.cuda.Stream()
        self.params = list(params)
        self.batch = batch or int(os.environ.get('UMAMD_WGRAD_BATCH', '24'))
        # also flush once the queued weight gradients hold this much work
        # (GFLOP; 0 = count only): a large one then starts at once instead
        # of waiting for the batch to fill (or for the end of the backward)
        self.flush_flop = float(os.environ.get('UMAMD_WGRAD_FLUSH_GFLOP', '0')) * 1e9
        self._queued_flop = 0.0
        self._launch = None
        self._pending = []
        self._pending_out = []
        self._on_flush = []
        self._events = []  # fork/join events of the current backward (stream_wait)

    def __enter__(self):
        if WgradStream._active is not None:
            raise RuntimeError('WgradStream contexts do not nest')
        if any(p.grad is not None for p in self.params):
            raise RuntimeError('WgradStream needs gradients set to None before backward '
                               '(zero_grad(set_to_none=True))')
        self._launch = torch.cuda.current_stream()
        self._events = []
        WgradStream._active = self
        return self

    def defer(self, tensors, launch, out_ptr=None, flop=0.0, out_bytes=1):
        """Queue one weight gradient (``launch`` issues its kernels on the
        current stream; ``tensors`` are the ones it touches, ``out_ptr`` /
        ``out_bytes`` the byte range it writes, ``flop`` its work) and flush
        the queue onto the
        side stream every ``batch`` entries (or ``flush_flop`` of work): one
        fork per batch instead of one per conv."""
        self._pending.append((tensors, launch))
        self._queued_flop += flop
        if out_ptr is not None:
            self._pending_out.append((out_ptr, out_ptr + max(int(out_bytes), 1)))
        if len(self._pending) >= self.batch or \
                (self.flush_flop > 0 and self._queued_flop >= self.flush_flop):
            self._flush()

    def is_pending(self, spans) -> bool:
        """True if any of these (address, bytes) spans overlaps a range
        written by a queued launch that has not been flushed onto the side
        stream yet.  Ranges, not base addresses: a gradient may be a view into
        a larger deferred output (the attention's K/V slices of the fused QKV
        weight gradient, functional.AttentionFn.backward)."""
        for p, n in spans:
            e = p + max(int(n), 1)
            for a, b in self._pending_out:
                if p < b and a < e:
                    return True
        return False

    def on_flush(self, fn):
        """call ``fn()`` after every flush of this context (gradsync: a
        bucket whose gradients were queued becomes launchable)"""
        self._on_flush.append(fn)

    def _flush(self):
        if not self._pending:
            return
        stream_wait(self.stream, torch.cuda.current_stream(), self._events)
        from . import _lib as L
        from . import functional as F
        with torch.cuda.stream(self.stream):
            keep, descs = [], []
            for _, launch in self._pending:
                # a batched piece returns (what it must keep alive, descriptor):
                # merge weights (partial sums, um_mwg_desc), biases (partial
                # rows, um_csum_desc)
                r = launch()
                if isinstance(r, tuple) and len(r) == 2 and \
                        isinstance(r[1], (L.MwgDesc, F._Csum)):
                    keep.append(r[0])
                    descs.append(r[1])
            if descs:
                F.batched_launch(descs)
            del keep  # freed on the side stream, after the batched launches
        for tensors, _ in self._pending:
            for t in tensors:
                t.record_stream(self.stream)
        self._pending = []
        self._pending_out.clear()
        self._queued_flop = 0.0
        for fn in self._on_flush:
            fn()

    def __exit__(self, *exc):
        WgradStream._active = None
        try:
            self._flush()
        finally:
            self._on_flush = []
            stream_wait(self._launch, self.stream, self._events)


def stream_wait(dst, src, keep: list):
    """``dst`` waits for the work queued on ``src`` so far (Stream.wait_stream)
    with an event object kept alive in ``keep`` until the caller drops it:
    under HIP graph capture an event that is destroyed while the capture
    runs and re-created at the same address makes a later wait attach to the
    wrong captured record (measured on MI355X: with one-parameter gradient
    buckets, ~200 fork/join pairs in one capture, most of the packed
    gradients were read before they were written)."""
    ev = torch.cuda.Event()
    ev.record(src)
    dst.wait_event(ev)
    keep.append(ev)


def active() -> Optional[WgradStream]:
    return WgradStream._active
