"""SyncBN statistics exchange without RCCL (``UMAMD_SYNCBN_IPC=1``).

Reference: parallel_main.py:156-158 converts BatchNorm2d to SyncBatchNorm,
whose forward all-reduces (sum, sum of squares, count) and whose backward
all-reduces (sum dz, sum dz*xhat) of every layer: 80 small collectives per
step at this model, each a latency-bound RCCL call ordered behind the
gradient buckets on the step's one communicator (umamd.rccl).

Here every rank owns an uncached device arena that the other ranks map by
HIP IPC (hipIpcGetMemHandle / hipIpcOpenMemHandle; the handles travel once
over the process group), and each exchange is ONE single-workgroup kernel
(csrc/bnx.hip: publish this rank's sums + flag, poll the peers' flags, sum
in rank order) on the issuing stream -- capturable, no host sync, no RCCL
call, so the communicator carries only the gradient buckets.

Exchange slots are numbered in issue order from the start of each forward
(``begin_forward``, called by functional.stat_scope): every rank issues the
same BN layers in the same order, so the same slot means the same layer.
Peers on other devices are reached over xGMI by the same code (the arena is
uncached, the flags and payload are system-scope accesses); it is tested
with two processes sharing one GPU (tests/test_gpu_bnx.py).
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional

import torch
import torch.distributed as dist

from ._lib import UmamdError, call, query

ENABLED = os.environ.get('UMAMD_SYNCBN_IPC') == '1'
NSLOTS = 192     # exchanges per step (40 forward + 40 backward BN layers here)
MAX_C = 1024     # channels per exchange


class BNExchange:
    def __init__(self, group):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.slot = 0
        nbytes = query('um_bnx_bytes', NSLOTS, MAX_C)
        self.base = ctypes.c_void_p()
        handle = (ctypes.c_char * 64)()
        rc = query('um_bnx_alloc', nbytes, ctypes.addressof(self.base),
                   ctypes.addressof(handle))
        if rc != 0:
            raise UmamdError(f'um_bnx_alloc failed ({rc})')
        hs = [None] * self.world
        dist.all_gather_object(hs, bytes(handle), group=group)
        self.peers = []
        addrs = []
        for r, h in enumerate(hs):
            if r == self.rank:
                addrs.append(self.base.value)
                continue
            p = ctypes.c_void_p()
            buf = (ctypes.c_char * 64).from_buffer_copy(h)
            if query('um_bnx_open', ctypes.addressof(buf), ctypes.addressof(p)) != 0:
                raise UmamdError(f'um_bnx_open of rank {r} failed')
            self.peers.append(p)
            addrs.append(p.value)
        self.table = torch.tensor(addrs, dtype=torch.int64, device='cuda')

    def begin_forward(self):
        self.slot = 0

    def all_reduce_slots(self, t: torch.Tensor, C: int):
        """in-place all-reduce of a statistics-slot tensor [16][C][2] + count"""
        if self.slot >= NSLOTS:
            raise UmamdError(f'umamd.bnx: more than {NSLOTS} BN exchanges in one step')
        if C > MAX_C:
            raise UmamdError(f'umamd.bnx: {C} channels > {MAX_C}')
        call('um_bnx_allreduce', t.data_ptr(), C, self.table.data_ptr(), self.world, self.rank,
             self.slot, NSLOTS, MAX_C)
        self.slot += 1

    def check(self):
        """raise if any exchange gave up waiting for a peer"""
        torch.cuda.synchronize()
        if query('um_bnx_status', self.base) != 0:
            raise UmamdError('umamd.bnx: an exchange timed out waiting for a peer rank')

    def close(self):
        if self.base is None:
            return
        torch.cuda.synchronize()
        for p in self.peers:
            query('um_bnx_close', p)
        query('um_bnx_free', self.base)
        self.base = None
        self.peers = []


_exchanges: Dict[int, BNExchange] = {}


def get(group) -> Optional[BNExchange]:
    """The exchange of ``group`` when UMAMD_SYNCBN_IPC=1 (created on first use,
    at the same BN call on every rank), else None."""
    if not ENABLED or group is None:
        return None
    x = _exchanges.get(id(group))
    if x is None or x.group is not group:
        x = _exchanges[id(group)] = BNExchange(group)
    return x


def begin_forward():
    for x in _exchanges.values():
        x.begin_forward()


def close_all():
    for x in list(_exchanges.values()):
        x.close()
    _exchanges.clear()
