"""Bucketed gradient all-reduce overlapped with the backward pass.

The data-parallel step of the reference is DDP (parallel_main.py:157-158):
its reducer all-reduces ~25 MB gradient buckets from autograd hooks while
the backward still runs.  The captured step (train.graph.CapturedTrainStep)
bypasses DDP's reducer (its hooks cannot follow gradients that the side
stream writes later, umamd.overlap), so it brings its own:

  * buckets of parameters in reverse registration order (the order the
    backward produces their gradients: decoder head first, encoder stem
    last), about ``cap_mb`` each, laid out back to back in ONE flat f32
    buffer;
  * a post-accumulate-grad hook per parameter marks it ready; a bucket whose
    members are all ready -- and none of whose gradients is still queued on
    the weight-gradient side stream (``overlap.WgradStream``; checked again
    after every flush of that queue) -- is launched at once on a
    communication stream that first waits for the launch stream and the side
    stream: pack (one ``torch.cat`` into its slice of the flat buffer), then
    one all-reduce (RCCL ``AVG``; other backends sum and scale);
  * ``finish`` launches what is left, joins the communication stream back
    into the launch stream and makes every ``.grad`` a view of the reduced
    flat buffer (the fused Adam's pointer table holds those views).

Inside a HIP graph capture the communication stream and RCCL's own stream
become parallel branches of the graph, so the all-reduce of the decoder's
buckets overlaps the encoder's backward.  On CPU tensors (gloo tests) there
are no streams and the same logic runs in order.
"""
from __future__ import annotations

from typing import List, Optional

import torch
from torch import distributed as dist

from . import overlap as _overlap
from . import rccl as _rccl


class GradBuckets:
    def __init__(self, params, group, world: int, cap_mb: float = 16.0):
        self.params = [p for p in params if p.requires_grad]
        self.group, self.world = group, world
        self.cap = int(cap_mb * 2 ** 20)
        self.layout = None          # which params receive a gradient (first step)
        self.buckets: List[list] = []
        self.slices = []
        self.of = {}                # id(param) -> bucket index
        self.flat: Optional[torch.Tensor] = None
        self.stream = None
        self.armed = False
        self.ov = None
        self.ready = set()
        self.launched = set()
        self.raw = []
        self._events = []  # fork/join events of the current backward (overlap.stream_wait)
        self._hooks = [p.register_post_accumulate_grad_hook(self._hook) for p in self.params]

    # ------------------------------------------------------------ layout --
    def _build(self, have):
        used = [p for p, h in zip(self.params, have) if h]
        total = sum(p.numel() for p in used)
        dev = used[0].device
        self.flat = torch.empty(total, dtype=torch.float32, device=dev)
        # backward order ~ reverse registration order
        cur, cur_bytes = [], 0
        for p in reversed(used):
            cur.append(p)
            cur_bytes += p.numel() * 4
            if cur_bytes >= self.cap:
                self.buckets.append(cur)
                cur, cur_bytes = [], 0
        if cur:
            self.buckets.append(cur)
        # each bucket packs into a contiguous slice: lay its members out in
        # bucket order (not registration order)
        off = 0
        self.slices = []
        self.views = {}
        for bi, b in enumerate(self.buckets):
            n0 = off
            for p in b:
                self.views[id(p)] = (off, p.numel(), p.shape)
                self.of[id(p)] = bi
                off += p.numel()
            self.slices.append((n0, off - n0))
        if dev.type == 'cuda':
            self.stream = torch.cuda.Stream(device=dev)

    # ------------------------------------------------------------- steps --
    def arm(self):
        """before a backward: hooks may launch buckets (once the layout is
        known, i.e. from the second step on; the first step reduces in
        ``finish``)"""
        self.armed = True
        self.ready.clear()
        self.launched.clear()
        self.raw = []
        self._events = []
        self.ov = _overlap.active()
        if self.ov is not None and self.layout is not None:
            self.ov.on_flush(self._poll)

    def _hook(self, p):
        if not self.armed or self.layout is None:
            return
        self.ready.add(id(p))
        bi = self.of.get(id(p))
        if bi is not None:
            self._try(bi)

    def _poll(self):
        for bi in range(len(self.buckets)):
            self._try(bi)

    def _try(self, bi):
        if bi in self.launched:
            return
        b = self.buckets[bi]
        if any(id(p) not in self.ready for p in b):
            return
        if self.ov is not None and self.ov.is_pending(
                (p.grad.data_ptr(), p.grad.numel() * p.grad.element_size()) for p in b):
            return  # written by a queued side-stream launch: wait for its flush
        self._launch(bi)

    def _launch(self, bi):
        self.launched.add(bi)
        b = self.buckets[bi]
        off, n = self.slices[bi]
        dst = self.flat[off:off + n]
        grads = [p.grad for p in b]
        for g in grads:
            if g.dtype != torch.float32:
                raise TypeError('GradBuckets: float32 gradients expected')
        self.raw += grads  # the backward's own gradient tensors stay allocated
        if self.stream is None:
            self._pack(dst, grads)
            self._reduce(dst)
            return
        # The pack runs on a stream that produced (or is ordered after) the
        # gradients -- the launch stream, or the weight-gradient stream after
        # it waited for the launch stream -- and only the all-reduce of the
        # packed slice forks onto the communication stream.  Measured on
        # MI355X: a pack on the communication stream issued during the
        # captured backward (autograd's device thread, from these hooks) read
        # gradient memory before it was written in replay, although its
        # event dependency was recorded after the producer (one-parameter
        # buckets: ~150 of 233 gradients wrong; the same wait issued after
        # the backward, or a pack on the producing stream, was exact:
        # tools/ddp_tiny_probe.py, tests/test_gpu_graph.py tiny buckets).
        cur = torch.cuda.current_stream()
        src = cur
        if self.ov is not None:  # gradients written on the weight-gradient stream
            src = self.ov.stream
            _overlap.stream_wait(src, cur, self._events)
        with torch.cuda.stream(src):
            self._pack(dst, grads)
        _overlap.stream_wait(self.stream, src, self._events)
        with torch.cuda.stream(self.stream):
            self._reduce(dst)

    @staticmethod
    def _pack(dst, grads):
        torch.cat([g.reshape(-1) for g in grads], out=dst)

    def _reduce(self, dst):
        c = _rccl.active(self.group)  # the captured step's own communicator
        if c is not None:
            c.all_reduce(dst, average=True)
        elif dist.get_backend(self.group) == 'nccl':
            dist.all_reduce(dst, op=dist.ReduceOp.AVG, group=self.group)
        else:
            dist.all_reduce(dst, group=self.group)
            dst.mul_(1.0 / self.world)

    def finish(self):
        """after the backward (and the side stream's join): reduce what is
        left, join, and point every ``.grad`` into the reduced buffer"""
        have = tuple(p.grad is not None for p in self.params)
        if self.layout is None:
            if not any(have):
                raise RuntimeError('GradBuckets: no gradients')
            self.layout = have
            self._build(have)
        elif have != self.layout:
            raise RuntimeError('CapturedTrainStep: the set of parameters with gradients changed')
        for bi in range(len(self.buckets)):
            if bi not in self.launched:
                self._launch(bi)
        if self.stream is not None:
            _overlap.stream_wait(torch.cuda.current_stream(), self.stream, self._events)
        for p, h in zip(self.params, self.layout):
            if h:
                off, n, shape = self.views[id(p)]
                p.grad = self.flat[off:off + n].view(shape)
        self.armed = False
        self.ov = None
        return self.flat

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
