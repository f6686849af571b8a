"""Whole-step HIP graph capture of the training step.

The eager step (train.train.train_step, reference train/train.py:116-129)
issues ~1,300 small launches from Python; at B=8 x 256x512 the host cannot
keep the GPU fed.  ``CapturedTrainStep`` captures the same step once and
replays it:

  graph 1: pyramid -> model forward -> reconstruct -> fused loss -> backward
           (gradients land in static graph-pool tensors)
           (weight gradients on a parallel branch, umamd.overlap)
  graph 2: fused Adam over those gradients (pointer table uploaded once,
           step counter and lr read from device memory by the kernel)

Construction runs ``warmup`` eager steps (allocator warm-up, optimiser state
creation) and then captures; by default (``restore_state=True``) the
parameters, BN buffers and Adam moments / step counters are put back to their
values from before the warm-up, so the first replay is the first update.

Inputs are copied into static device buffers before each replay.  Host-side
state that the eager loop would change between steps must not change under
a captured step: the disparity ``scale`` is fixed at capture (recapture when
``adjust_disparity`` moves it) and the learning rate goes through
``umamd.optim.Adam.set_lr``.

Data parallel (one process per GPU, model wrapped by train.parallel): the
captured forward runs the wrapped module directly, so DDP's autograd hooks
stay idle, and the gradient exchange is recorded in graph 1 itself -- the
gradients are packed into ~16 MB buckets of one flat f32 buffer, each
averaged by an RCCL all-reduce launched from the backward's hooks as soon as
its gradients exist, on a communication branch that overlaps the rest of
the backward (umamd.gradsync; SyncBN's statistic all-reduces are recorded
the same way).  ``.grad`` of each parameter is then a view of the reduced
buffer, which is what the fused Adam's pointer table holds.  DDP
construction still broadcasts rank 0's parameters, and its module keeps the
reference's ``module.`` checkpoint keys; construct it under the capture
stream (``stream=``).
"""
from __future__ import annotations

import os

import torch
from torch import distributed as dist
from torch.nn.parallel import DistributedDataParallel

from umamd import lossfn as LF
from umamd import overlap
from umamd import rccl
from umamd.gradsync import GradBuckets

from . import utils as u


class CapturedTrainStep:
    def __init__(self, model, loss_function, optimiser, left, right, scale: float,
                 scales: int = 4, warmup: int = 3, restore_state: bool = True,
                 stream=None):
        """``stream``: the stream to warm up and capture on (default: a new
        one).  A DistributedDataParallel model must have been constructed
        while that stream was current: DDP keeps the parameters'
        AccumulateGrad nodes alive, and a node created on another stream
        makes the backward synchronise with that stream, which breaks the
        capture."""
        if not hasattr(optimiser, 'prepare'):
            raise TypeError('CapturedTrainStep needs umamd.optim.Adam (graph-replayable)')
        self.group, self.world = None, 1
        if isinstance(model, DistributedDataParallel):
            self.group = model.process_group
            model = model.module  # DDP's reducer stays idle; see _reduce_grads
        elif dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            self.group = dist.group.WORLD
        if self.group is not None:
            self.world = dist.get_world_size(self.group)
        self._buckets = None
        if self.group is not None:
            # bucketed all-reduce overlapped with the backward (umamd.gradsync);
            # UMAMD_GRAD_BUCKET_MB sizes the buckets, 0 = one all-reduce at the
            # end.  A one-rank group has no peer to overlap with: there the
            # buckets' packs and per-bucket collectives only cost (one-rank
            # SyncBN step on MI355X: 750 bucketed vs 795 pairs/s with one
            # all-reduce, dp1 805), so the default is one all-reduce
            default_mb = '16' if self.world > 1 else '0'
            mb = float(os.environ.get('UMAMD_GRAD_BUCKET_MB', default_mb))
            self._buckets = GradBuckets(model.parameters(), self.group, self.world,
                                        cap_mb=mb if mb > 0 else 1e9)
        # RCCL collectives of the step (SyncBN, gradient buckets) through the
        # step's own communicator, in one total order across the issuing
        # streams (umamd.rccl: no process group watchdog polling events of a
        # capturing stream, no stream hop, no cross-communicator deadlock)
        self._comm = None
        if self.group is not None and dist.get_backend(self.group) == 'nccl':
            self._comm = rccl.acquire(self.group)
        snap = self._snapshot(model, optimiser) if restore_state else None
        self.model, self.loss_function, self.optimiser = model, loss_function, optimiser
        self.scale, self.scales = float(scale), scales
        # weight gradients on a side stream beside the dgrad chain (umamd.overlap);
        # UMAMD_WGRAD_OVERLAP=0 keeps the whole backward on one stream
        self.overlap = None
        if os.environ.get('UMAMD_WGRAD_OVERLAP', '1') != '0':
            self.overlap = overlap.WgradStream(p for p in model.parameters() if p.requires_grad)
        self.left = left.detach().clone().contiguous()
        # the backward's seed d total / d (disp_loss, error_loss) = (1, 1),
        # made once: no add and no ones-fill launch inside the step
        self._seed = torch.ones((), dtype=torch.float32, device=left.device)
        self.right = right.detach().clone().contiguous()
        cur = torch.cuda.current_stream()
        side = stream if stream is not None else torch.cuda.Stream()
        if side != cur:
            side.wait_stream(cur)
        with torch.cuda.stream(side), rccl.use(self._comm):
            for _ in range(warmup):  # eager steps: allocator warm-up, optimiser state
                optimiser.zero_grad(set_to_none=True)
                self._fwd_bwd()
                optimiser.step()
        cur.wait_stream(side)
        torch.cuda.synchronize()
        optimiser.zero_grad(set_to_none=True)
        # capture on the warm-up stream so autograd's cached AccumulateGrad
        # nodes see the stream they were created on; the backward (autograd's
        # device thread) launches into the capture too.
        # Data parallel: the step's collectives go through its own RCCL
        # communicator (umamd.rccl), so the process group's watchdog never
        # polls an event of a stream that joins the capture; the capture is
        # 'thread_local' all the same, so that its event queries (of earlier
        # eager collectives: DDP's parameter broadcast, the id exchange) are
        # never refused.  UMAMD_CAPTURE_MODE overrides.
        mode = os.environ.get('UMAMD_CAPTURE_MODE',
                              'thread_local' if self.group is not None else 'global')
        self.g_fb = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_fb, stream=side, capture_error_mode=mode), \
                rccl.use(self._comm):
            self.disp_loss, self.error_loss = self._fwd_bwd()
        # the returned losses are static graph outputs; detached, they keep no
        # autograd graph alive (its AccumulateGrad nodes remember the capture
        # stream, and an eager step on another stream would synchronise with it)
        self.disp_loss, self.error_loss = self.disp_loss.detach(), self.error_loss.detach()
        if self._comm is not None and self.world > 1:
            # the captured collective sequence must be the same on every rank
            # (one ordered communicator, umamd.rccl): checked once, eagerly
            rccl.check_order(self._comm)
        optimiser.prepare()  # tables for the graph-pool gradients, outside capture
        # the captured Adam reads these device tables by address: keep them
        # alive even if an eager step (another batch shape) replaces them
        self._opt_tables = list(getattr(optimiser, '_tables', {}).values())
        torch.cuda.synchronize()
        self.g_opt = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_opt, pool=self.g_fb.pool(), stream=side,
                              capture_error_mode=mode):
            optimiser.step()
        if snap is not None:
            self._restore(model, optimiser, snap)

    @staticmethod
    @torch.no_grad()
    def _snapshot(model, opt):
        params = [p.detach().clone() for p in model.parameters()]
        bufs = [b.detach().clone() for b in model.buffers()]
        moments = {id(p): {k: v.clone() for k, v in opt.state[p].items() if torch.is_tensor(v)}
                   for g in opt.param_groups for p in g['params'] if p in opt.state}
        dev = {gi: st['step'].clone() for gi, st in opt._dev.items()}
        return params, bufs, moments, dev

    @staticmethod
    @torch.no_grad()
    def _restore(model, opt, snap):
        """Undo the warm-up updates in place (the captured graphs keep the
        same tensors)."""
        params, bufs, moments, dev = snap
        for p, v in zip(model.parameters(), params):
            p.copy_(v)
        for b, v in zip(model.buffers(), bufs):
            b.copy_(v)
        for g in opt.param_groups:
            for p in g['params']:
                for k, v in opt.state.get(p, {}).items():
                    if torch.is_tensor(v):
                        old = moments.get(id(p), {}).get(k)
                        v.copy_(old) if old is not None else v.zero_()
        for gi, st in opt._dev.items():
            old = dev.get(gi)
            st['step'].copy_(old) if old is not None else st['step'].zero_()
        torch.cuda.synchronize()

    def _fwd_bwd(self):
        images = torch.cat([self.left, self.right], dim=1)
        pyramid = u.scale_pyramid(images, self.scales)
        disparities = self.model(self.left, self.scale)
        from .loss import TukraUncertaintyLoss
        if isinstance(self.loss_function, TukraUncertaintyLoss):
            with LF.deferred_recon():  # the fused loss forward writes the recon
                recon = u.reconstruct_pyramid(disparities, pyramid)
        else:
            recon = u.reconstruct_pyramid(disparities, pyramid)
        disp_loss, error_loss = self.loss_function(pyramid, disparities, recon, 0, None)

        def backward():
            seeds = tuple(self._seed if t.dtype == self._seed.dtype and t.dim() == 0
                          else torch.ones_like(t) for t in (disp_loss, error_loss))
            torch.autograd.backward((disp_loss, error_loss), seeds)
        if self.overlap is None:
            if self._buckets is not None:
                self._buckets.arm()
            backward()
        else:
            with self.overlap:
                if self._buckets is not None:
                    self._buckets.arm()  # buckets launch from the backward's hooks
                backward()
        if self._buckets is not None:
            self._reduce_grads()
        return disp_loss, error_loss

    @property
    def _flat(self):
        return self._buckets.flat if self._buckets is not None else None

    def _reduce_grads(self):
        """Average the gradients over the group (DDP's result): the buckets
        not yet launched from the backward's hooks are packed and
        all-reduced now, the communication stream joins the launch stream
        and ``.grad`` become views of the reduced flat buffer."""
        if self._buckets is None:
            self._buckets = GradBuckets(self.model.parameters(), self.group, self.world)
        self._buckets.finish()

    def close(self):
        """Release what ties this step to the model: the gradient buckets'
        post-accumulate-grad hooks (each would keep this step's flat buffer,
        its raw gradients and its stream alive, and run on every later
        backward) and the graphs.  train.train._GraphSteps calls it before a
        recapture."""
        if self._buckets is not None:
            self._buckets.remove()
            self._buckets = None
        self.g_fb = self.g_opt = None
        self._opt_tables = []
        if self._comm is not None:  # after the graphs that recorded its collectives
            self._comm.sync()
            rccl.release(self._comm)
            self._comm = None

    def __call__(self, left=None, right=None):
        if left is not None:
            self.left.copy_(left)
        if right is not None:
            self.right.copy_(right)
        if self._comm is not None:  # the collectives recorded in g_fb run on this stream
            self._comm.note_stream(torch.cuda.current_stream())
        self.g_fb.replay()
        self.g_opt.replay()
        return self.disp_loss, self.error_loss
