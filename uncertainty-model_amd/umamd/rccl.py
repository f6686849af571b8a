"""The captured step's own RCCL communicator (SyncBN statistics and the
bucketed gradient all-reduce), called on the launch stream itself.

The reference's data-parallel step goes through torch's process group
(parallel_main.py:156-158: SyncBatchNorm + DDP on 'nccl').  Inside a HIP graph
that has two costs on MI355X:

  * the process group's watchdog thread polls the end events of its eager
    collectives (the warm-up steps before a capture).  HIP refuses a query of
    an event whose stream is being captured (hipErrorCapturedEvent), and the
    process group's stream joins the capture at its first recorded
    collective: the watchdog throws and aborts the process, unless it happened
    to retire every eager collective first (measured: a recapture after a
    replay aborts; a first capture survives only with a wait of ~0.5 s);
  * every collective hops to the process group's internal stream and back
    (two event edges per collective in the graph: 80 SyncBN all-reduces and
    the gradient buckets per step).

So the captured step opens its own RCCL communicators over the process
group's ranks (one per issuing stream, see ``TAGS``; the unique ids travel
over the group once, eagerly) and calls ``ncclAllReduce``
through ctypes on the caller's current stream: no watchdog, no stream hop, and
the eager warm-up steps use the same communicator (its lazy connection setup
happens there, never inside a capture).  The library is the RCCL torch itself
loaded (torch/lib/librccl.so), so there is one RCCL in the process.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional

import torch
from torch import distributed as dist

_SUM, _AVG = 0, 4
_DTYPES = {torch.float32: 7, torch.float64: 8, torch.bfloat16: 9, torch.int32: 2,
           torch.int64: 4}


class _UniqueId(ctypes.Structure):
    _fields_ = [('internal', ctypes.c_char * 128)]


_lib: Optional[ctypes.CDLL] = None


def _rccl() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        path = os.path.join(os.path.dirname(torch.__file__), 'lib', 'librccl.so')
        if not os.path.exists(path):
            path = 'librccl.so'
        lib = ctypes.CDLL(path)
        lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                         _UniqueId, ctypes.c_int]
        lib.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_void_p]
        lib.ncclGetErrorString.restype = ctypes.c_char_p
        lib.ncclGetErrorString.argtypes = [ctypes.c_int]
        _lib = lib
    return _lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = _rccl().ncclGetErrorString(rc).decode(errors='replace')
        raise RuntimeError(f'umamd.rccl: {what} failed ({rc}): {msg}')


class Comm:
    """An RCCL communicator over the ranks of a 'nccl' process group."""

    def __init__(self, group):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.ranks = dist.get_process_group_ranks(group)
        lib = _rccl()
        uid = _UniqueId()
        if self.rank == 0:
            _check(lib.ncclGetUniqueId(ctypes.byref(uid)), 'ncclGetUniqueId')
        obj = [bytes(uid.internal) if self.rank == 0 else None]
        # the id travels over the group once, eagerly (never inside a capture)
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0), group=group)
        uid.internal = obj[0]
        self.comm = ctypes.c_void_p()
        _check(lib.ncclCommInitRank(ctypes.byref(self.comm), self.world, uid, self.rank),
               'ncclCommInitRank')

    def all_reduce(self, t: torch.Tensor, average: bool = False):
        """In-place sum (or average) of ``t`` over the ranks, on the current
        stream (recorded as a graph node when that stream is capturing)."""
        if not t.is_contiguous():
            raise ValueError('umamd.rccl.all_reduce: contiguous tensor expected')
        dt = _DTYPES.get(t.dtype)
        if dt is None:
            raise TypeError(f'umamd.rccl.all_reduce: dtype {t.dtype}')
        stream = torch.cuda.current_stream(t.device).cuda_stream
        _check(_rccl().ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), dt,
                                     _AVG if average else _SUM, self.comm, stream),
               'ncclAllReduce')


_comms: Dict[tuple, Comm] = {}

# the communicators of one captured step, one per stream that issues
# collectives: SyncBN's statistics on the launch stream, the gradient buckets
# on their communication stream.  One communicator must not be driven from
# two streams at once: its collectives then run concurrently on its one set of
# channels and corrupt each other (measured on MI355X with one communicator:
# gradients of buckets all-reduced during the backward, beside the SyncBN
# all-reduces, came out wrong)
TAGS = ('bn', 'grad')


def comm_for(group, tag: str) -> Comm:
    """The process's communicator ``tag`` for ``group`` (created on first
    use; every rank of the group must call this at the same point)."""
    key = (id(group), tag)
    c = _comms.get(key)
    if c is None or c.group is not group:
        c = _comms[key] = Comm(group)
    return c


def comms_for(group) -> Dict[str, Comm]:
    return {t: comm_for(group, t) for t in TAGS}


_active: Optional[Dict[str, Comm]] = None


class use:
    """Within this context, umamd's collectives on a 'nccl' group go through
    these communicators instead of the process group (BNSync: ``'bn'``,
    GradBuckets: ``'grad'``)."""

    def __init__(self, comms: Optional[Dict[str, Comm]]):
        self.comms = comms
        self.prev = None

    def __enter__(self):
        global _active
        self.prev, _active = _active, self.comms
        return self.comms

    def __exit__(self, *exc):
        global _active
        _active = self.prev


def active(group, tag: str) -> Optional[Comm]:
    """The communicator to use for a collective ``tag`` over ``group`` (None:
    use the process group): the active one when it spans the same ranks."""
    if _active is None or group is None:
        return None
    c = _active.get(tag)
    if c is None:
        return None
    if group is c.group or dist.get_process_group_ranks(group) == c.ranks:
        return c
    return None
