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
``umamd.optim.Adam.set_lr``.  Single-process only: the DDP gradient
all-reduce runs eagerly.
"""
from __future__ import annotations

import os

import torch

from umamd import lossfn as LF
from umamd import overlap

from . import utils as u


class CapturedTrainStep:
    def __init__(self, model, loss_function, optimiser, left, right, scale: float,
                 scales: int = 4, warmup: int = 3, restore_state: bool = True):
        if not hasattr(optimiser, 'prepare'):
            raise TypeError('CapturedTrainStep needs umamd.optim.Adam (graph-replayable)')
        snap = self._snapshot(model, optimiser) if restore_state else None
        self.model, self.loss_function, self.optimiser = model, loss_function, optimiser
        self.scale, self.scales = float(scale), scales
        # weight gradients on a side stream beside the dgrad chain (umamd.overlap);
        # UMAMD_WGRAD_OVERLAP=0 keeps the whole backward on one stream
        self.overlap = None
        if os.environ.get('UMAMD_WGRAD_OVERLAP', '1') != '0':
            self.overlap = overlap.WgradStream(p for p in model.parameters() if p.requires_grad)
        self.left = left.detach().clone().contiguous()
        self.right = right.detach().clone().contiguous()
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(warmup):  # eager steps: allocator warm-up, optimiser state
                optimiser.zero_grad(set_to_none=True)
                self._fwd_bwd()
                optimiser.step()
        cur.wait_stream(side)
        torch.cuda.synchronize()
        optimiser.zero_grad(set_to_none=True)
        # capture on the warm-up stream so autograd's cached AccumulateGrad
        # nodes see the stream they were created on
        self.g_fb = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_fb, stream=side):
            self.disp_loss, self.error_loss = self._fwd_bwd()
        optimiser.prepare()  # tables for the graph-pool gradients, outside capture
        torch.cuda.synchronize()
        self.g_opt = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_opt, pool=self.g_fb.pool(), stream=side):
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
        with LF.deferred_recon():  # the loss forward writes the recon
            recon = u.reconstruct_pyramid(disparities, pyramid)
        disp_loss, error_loss = self.loss_function(pyramid, disparities, recon, 0, None)
        if self.overlap is None:
            (disp_loss + error_loss).backward()
        else:
            with self.overlap:
                (disp_loss + error_loss).backward()
        return disp_loss, error_loss

    def __call__(self, left=None, right=None):
        if left is not None:
            self.left.copy_(left)
        if right is not None:
            self.right.copy_(right)
        self.g_fb.replay()
        self.g_opt.replay()
        return self.disp_loss, self.error_loss
