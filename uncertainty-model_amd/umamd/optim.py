"""Fused multi-tensor Adam on the umamd C ABI.

Same update as torch.optim.Adam(params, lr) with default betas/eps/no
amsgrad, which is what reference train/train.py:228-229 uses.  One kernel
launch updates every parameter.

Graph-replayable: the step counter and the learning rate live on the device
(``um_adam_step_dev`` increments the counter itself), and the
{param, grad, exp_avg, exp_avg_sq, numel} table is copied from pinned host
memory with a non-blocking copy, so the whole training step (forward,
backward, optimiser) can be captured in one HIP graph and replayed.  The
table is rebuilt only when a pointer changes.
"""
from __future__ import annotations

import torch

from . import _lib as L


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._tables = {}
        self._dev = {}

    def _table(self, gi, plist):
        key = tuple((p.data_ptr(), p.grad.data_ptr(), self.state[p]['exp_avg'].data_ptr(),
                     self.state[p]['exp_avg_sq'].data_ptr(), p.numel()) for p in plist)
        cached = self._tables.get(gi)
        if cached is not None and cached[0] == key:
            return cached[1], cached[2], cached[3]
        chunk = L.query('um_adam_chunk')
        rows, chunks = [], []
        for e, (pp, gp, mp, vp, n) in enumerate(key):
            rows.append([pp, gp, mp, vp, n])
            for c in range((n + chunk - 1) // chunk):
                chunks.append([e, c])
        dev = plist[0].device
        h_tab = torch.tensor(rows, dtype=torch.int64).pin_memory()
        h_ch = torch.tensor(chunks, dtype=torch.int32).pin_memory()
        tab = h_tab.to(dev, non_blocking=True)
        ch = h_ch.to(dev, non_blocking=True)
        # keep the pinned sources alive as long as the table (graph memcpy nodes)
        self._tables[gi] = (key, tab, ch, len(chunks), h_tab, h_ch)
        return tab, ch, len(chunks)

    def _device_state(self, gi, group, dev):
        st = self._dev.get(gi)
        if st is None:
            step = torch.zeros(1, dtype=torch.int32, device=dev)
            lr = torch.full((1,), float(group['lr']), dtype=torch.float32, device=dev)
            st = {'step': step, 'lr': lr, 'lr_host': float(group['lr'])}
            self._dev[gi] = st
        if st['lr_host'] != float(group['lr']):
            st['lr'].fill_(float(group['lr']))
            st['lr_host'] = float(group['lr'])
        return st

    def _prepare_group(self, gi, group):
        plist = [p for p in group['params'] if p.grad is not None]
        if not plist:
            return None
        for p in plist:
            if p.dtype != torch.float32 or p.grad.dtype != torch.float32:
                raise TypeError('umamd Adam: float32 params/grads only')
            if not p.is_contiguous() or not p.grad.is_contiguous():
                raise ValueError('umamd Adam: contiguous params/grads only')
            L.require_device(p)
            st = self.state[p]
            if len(st) == 0:
                st['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
        ds = self._device_state(gi, group, plist[0].device)
        tab, ch, nch = self._table(gi, plist)
        return ds, tab, ch, nch

    @torch.no_grad()
    def prepare(self):
        """Create state and upload the pointer tables for the current grads
        without updating anything (call before capturing ``step`` in a graph,
        so the capture holds no host-to-device copy)."""
        for gi, group in enumerate(self.param_groups):
            self._prepare_group(gi, group)

    def set_lr(self, lr: float):
        """Change the learning rate of every group, device copy included
        (takes effect in captured graphs too)."""
        for gi, group in enumerate(self.param_groups):
            group['lr'] = lr
            st = self._dev.get(gi)
            if st is not None:
                st['lr'].fill_(float(lr))
                st['lr_host'] = float(lr)

    def sync_lr(self):
        """Copy each group's host learning rate to its device copy if it
        changed (``adjust_learning_rate`` writes ``group['lr']``; a captured
        step only sees the device copy)."""
        for gi, group in enumerate(self.param_groups):
            st = self._dev.get(gi)
            if st is not None and st['lr_host'] != float(group['lr']):
                st['lr'].fill_(float(group['lr']))
                st['lr_host'] = float(group['lr'])

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            prep = self._prepare_group(gi, group)
            if prep is None:
                continue
            ds, tab, ch, nch = prep
            b1, b2 = group['betas']
            L.call('um_adam_step_dev', tab.data_ptr(), ch.data_ptr(), nch, float(group['lr']),
                   ds['lr'].data_ptr(), float(b1), float(b2), float(group['eps']),
                   float(group['weight_decay']), ds['step'].data_ptr())
        return loss
