"""The captured step's own RCCL communicator (SyncBN statistics and the
bucketed gradient all-reduce), called on the issuing stream itself.

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

So the captured step opens ONE RCCL communicator over the process group's
ranks (the unique id travels over the group once, eagerly) and calls
``ncclAllReduce`` through ctypes on the caller's current stream: no watchdog,
no stream hop, and the eager warm-up steps use the same communicator (its lazy
connection setup happens there, never inside a capture).  The library is the
RCCL torch itself loaded (torch/lib/librccl.so), so there is one RCCL in the
process.

Ordering (safe by construction).  Collectives are issued from two streams:
SyncBN's on the launch stream, the gradient buckets' on their communication
stream (umamd.gradsync).  Every collective of the communicator is chained
after the previous one, whatever stream issued it: when the issuing stream
changes, the new stream first waits for an event recorded on the previous
one (``Comm._order``).  So the collectives run one at a time, in the host's
issue order, which is the same on every rank (the same program: SyncBN in
forward / autograd order, buckets from the deterministic post-accumulate-grad
hooks and side-stream flushes) -- the order torch's process group gets from
its single internal stream, without its watchdog.  Two communicators driven
concurrently from two streams (round 4) had no such order: nothing stopped
rank 0 from starting a bucket's all-reduce while rank 1 started a SyncBN one,
the classic multi-communicator deadlock.  ``tests/test_ddp_cpu.py`` checks
the chain and the identical sequence on two gloo ranks with a recording
stand-in.

Lifetime: ``acquire`` counts the captured steps that use a group's
communicator, ``release`` (CapturedTrainStep.close) destroys it
(``ncclCommDestroy``) when the last one lets go.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
from typing import Dict, List, Optional

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
        lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        lib.ncclGetErrorString.restype = ctypes.c_char_p
        lib.ncclGetErrorString.argtypes = [ctypes.c_int]
        _lib = lib
    return _lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = _rccl().ncclGetErrorString(rc).decode(errors='replace')
        raise RuntimeError(f'umamd.rccl: {what} failed ({rc}): {msg}')


class _Order:
    """The total order of one communicator's collectives across issuing
    streams (see the module docstring).  ``before(stream)`` is called before
    each collective: if the previous collective came from another stream,
    ``stream`` waits for an event recorded on that one now (which follows
    the previous collective in its stream order).  Events stay referenced
    until ``reset`` (the start of the next step): under graph capture an event
    destroyed and re-created at the same address mid-capture attaches a later
    wait to the wrong record (umamd.overlap.stream_wait)."""

    def __init__(self, record=None, wait=None):
        self.last = None          # the stream of the previous collective
        self.events: List = []
        self.log: List = []       # ('wait', dst, src) / ('coll', stream) for tests
        self.sig: List = []       # (numel, dtype) per collective: check_order
        self._record = record or _cuda_record
        self._wait = wait or _cuda_wait

    def reset(self):
        self.last = None
        self.events = []
        self.log = []
        self.sig = []

    def before(self, stream):
        if self.last is not None and self.last != stream:
            ev = self._record(self.last)
            self._wait(stream, ev)
            self.events.append(ev)
            self.log.append(('wait', stream, self.last))
        self.log.append(('coll', stream))
        self.last = stream


def _cuda_record(stream):
    ev = torch.cuda.Event()
    ev.record(stream)
    return ev


def _cuda_wait(stream, ev):
    stream.wait_event(ev)


class Comm:
    """An RCCL communicator over the ranks of a 'nccl' process group."""

    def __init__(self, group):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.ranks = dist.get_process_group_ranks(group)
        self.order = _Order()
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
        # every stream that issued (eagerly) or replayed (graphs) one of this
        # communicator's collectives: close() waits for these streams only
        self._streams: Dict[int, torch.cuda.Stream] = {}

    def note_stream(self, stream):
        """``stream`` runs (or replays) collectives of this communicator"""
        self._streams[stream.cuda_stream] = stream

    def all_reduce(self, t: torch.Tensor, average: bool = False):
        """In-place sum (or average) of ``t`` over the ranks, on the current
        stream (recorded as a graph node when that stream is capturing),
        ordered after this communicator's previous collective."""
        if self.comm is None:
            raise RuntimeError('umamd.rccl.all_reduce: communicator destroyed')
        if not t.is_contiguous():
            raise ValueError('umamd.rccl.all_reduce: contiguous tensor expected')
        dt = _DTYPES.get(t.dtype)
        if dt is None:
            raise TypeError(f'umamd.rccl.all_reduce: dtype {t.dtype}')
        cur = torch.cuda.current_stream(t.device)
        self.note_stream(cur)
        self.order.before(cur)
        self.order.sig.append((int(t.numel()), str(t.dtype)))
        _check(_rccl().ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), dt,
                                     _AVG if average else _SUM, self.comm, cur.cuda_stream),
               'ncclAllReduce')

    def sync(self):
        """wait for every collective of this communicator issued so far: the
        streams that issued or replayed them, not the whole device"""
        for st in self._streams.values():
            st.synchronize()

    def close(self):
        """ncclCommDestroy (after every collective of this communicator has
        finished; graphs that recorded them must be gone)."""
        if self.comm is not None:
            self.sync()
            _check(_rccl().ncclCommDestroy(self.comm), 'ncclCommDestroy')
            self.comm = None
        self._streams = {}
        self.order.reset()


def check_order(comm, what='captured step'):
    """Compare this communicator's collective sequence since its last
    ``use`` (sizes and dtypes, in issue order) across the ranks, eagerly over
    the process group: a rank whose host issued its collectives in another
    order (hook or flush timing) fails here with the position of the first
    difference, instead of the replayed graph hanging in RCCL."""
    sig = list(comm.order.sig)
    h = hashlib.sha256(repr(sig).encode()).hexdigest()
    allh = [None] * comm.world
    dist.all_gather_object(allh, (h, len(sig)), group=comm.group)
    if any(x != allh[0] for x in allh):
        sigs = [None] * comm.world
        dist.all_gather_object(sigs, sig, group=comm.group)
        first = next((i for i in range(max(map(len, sigs)))
                      if len({repr(q[i]) if i < len(q) else None for q in sigs}) > 1), -1)
        raise RuntimeError(f'umamd.rccl: the {what} issues its collectives in a different order '
                           f'on different ranks (lengths {[len(q) for q in sigs]}, first '
                           f'difference at collective {first}); its graph would deadlock')
    return h


# group key -> [Comm, users]
_comms: Dict[int, list] = {}


def _key(group):
    return id(group)


def acquire(group) -> Comm:
    """The process's communicator for ``group`` (created on first use; every
    rank of the group must call this at the same point), one user more."""
    e = _comms.get(_key(group))
    if e is None or e[0].group is not group or e[0].comm is None:
        e = _comms[_key(group)] = [Comm(group), 0]
    e[1] += 1
    return e[0]


def release(comm: Optional[Comm]):
    """One user less; the last one destroys the communicator (every rank
    releases at the same point, as it acquired)."""
    if comm is None:
        return
    for k, e in list(_comms.items()):
        if e[0] is comm:
            e[1] -= 1
            if e[1] <= 0:
                del _comms[k]
                comm.close()
            return
    comm.close()


_active: Optional[Comm] = None


class use:
    """Within this context, umamd's collectives on a 'nccl' group go through
    this communicator instead of the process group (BNSync, GradBuckets).
    Entering starts a new collective chain (the previous step's collectives
    were joined into the launch stream at its end)."""

    def __init__(self, comm: Optional[Comm]):
        self.comm = comm
        self.prev = None

    def __enter__(self):
        global _active
        self.prev, _active = _active, self.comm
        if self.comm is not None:
            self.comm.order.reset()
        return self.comm

    def __exit__(self, *exc):
        global _active
        _active = self.prev


def active(group) -> Optional[Comm]:
    """The communicator for a collective over ``group`` (None: no step
    communicator is active, use the process group).  Raises when one is
    active but spans other ranks: a collective of the captured step must
    not fall back to the process group inside a capture (its watchdog
    aborts the process, see the module docstring)."""
    c = _active
    if c is None or group is None:
        return None
    if group is c.group or dist.get_process_group_ranks(group) == c.ranks:
        return c
    raise RuntimeError('umamd.rccl: a collective over a group other than the captured '
                       "step's (SyncBatchNorm process_group differs from DDP's) is not "
                       'supported in the captured step')
