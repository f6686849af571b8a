"""Fused multi-tensor Adam on the umamd C ABI (um_adam_step).

Same update as torch.optim.Adam(params, lr) with default betas/eps/no
amsgrad, which is what reference train/train.py:228-229 uses.  One kernel
launch updates every parameter; the {param, grad, m, v, numel} table lives
on the device and is rebuilt only when a pointer changes (e.g. grads set to
None by zero_grad and reallocated).  The step counter is host-side, so there
is no device->host synchronisation.
"""
from __future__ import annotations

import torch

from . import _lib as L


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._tables = {}

    def _table(self, gi, group, plist):
        key = tuple((p.data_ptr(), p.grad.data_ptr(), self.state[p]['exp_avg'].data_ptr(),
                     self.state[p]['exp_avg_sq'].data_ptr(), p.numel()) for p in plist)
        cached = self._tables.get(gi)
        if cached is not None and cached[0] == key:
            return cached[1], cached[2], cached[3]
        chunk = L.query('um_adam_chunk')
        rows = []
        chunks = []
        for e, (pp, gp, mp, vp, n) in enumerate(key):
            rows.append([pp, gp, mp, vp, n])
            for c in range((n + chunk - 1) // chunk):
                chunks.append([e, c])
        dev = plist[0].device
        tab = torch.tensor(rows, dtype=torch.int64).to(dev, non_blocking=False)
        ch = torch.tensor(chunks, dtype=torch.int32).to(dev, non_blocking=False)
        self._tables[gi] = (key, tab, ch, len(chunks))
        return tab, ch, len(chunks)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            plist = [p for p in group['params'] if p.grad is not None]
            if not plist:
                continue
            for p in plist:
                if p.dtype != torch.float32 or p.grad.dtype != torch.float32:
                    raise TypeError('umamd Adam: float32 params/grads only')
                if not p.is_contiguous() or not p.grad.is_contiguous():
                    raise ValueError('umamd Adam: contiguous params/grads only')
                L.require_device(p)
                st = self.state[p]
                if len(st) == 0:
                    st['step'] = 0
                    st['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st['step'] += 1
            steps = {self.state[p]['step'] for p in plist}
            if len(steps) != 1:
                raise RuntimeError('umamd Adam: parameters of a group at different steps')
            step = steps.pop()
            tab, ch, nch = self._table(gi, group, plist)
            b1, b2 = group['betas']
            L.call('um_adam_step', tab.data_ptr(), ch.data_ptr(), nch, float(group['lr']),
                   float(b1), float(b2), float(group['eps']), float(group['weight_decay']),
                   int(step))
        return loss
