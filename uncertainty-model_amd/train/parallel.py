"""Data-parallel wrapping of the model (reference parallel_main.py:156-158).

One process per GPU; BatchNorm layers become ``torch.nn.SyncBatchNorm``
(the umamd BN path recognises them and all-reduces its f64 partial sums
instead of torch's all_gather + host sync, functional.BNSync), and the model
is wrapped in DistributedDataParallel, whose gradient all-reduce runs on
RCCL ('nccl' backend) over xGMI, overlapped with the backward pass.

``gradient_as_bucket_view`` keeps each ``.grad`` a view into its all-reduce
bucket, so the reduced gradient is not copied back and the fused Adam reads
it in place.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch.nn import Module, SyncBatchNorm
from torch.nn.parallel import DistributedDataParallel


def data_parallel(model: Module, device_index: Optional[int] = None,
                  process_group=None, bucket_cap_mb: float = 25.0,
                  sync_bn: bool = True, stream=None) -> DistributedDataParallel:
    """``stream``: the HIP stream the training step will be captured on
    (train.graph.CapturedTrainStep, train.train's captured loop).  DDP keeps
    the parameters' AccumulateGrad nodes alive and each remembers the stream
    it was created on, so DDP is constructed under that stream (a new one by
    default for a device model) and the stream is recorded on the wrapper as
    ``_umamd_stream``."""
    if sync_bn:  # torch only accepts SyncBatchNorm under DDP for device modules
        model = SyncBatchNorm.convert_sync_batchnorm(model, process_group)
    kwargs = dict(process_group=process_group, bucket_cap_mb=bucket_cap_mb,
                  gradient_as_bucket_view=True)
    if device_index is not None:
        kwargs['device_ids'] = [device_index]
    p = next(model.parameters(), None)
    on_device = p is not None and p.is_cuda
    if stream is None and on_device:
        cur = torch.cuda.current_stream(p.device)
        # already under a side stream (the caller's capture stream): use it
        stream = cur if cur != torch.cuda.default_stream(p.device) \
            else torch.cuda.Stream(device=p.device)
    if stream is None:
        return DistributedDataParallel(model, **kwargs)
    cur = torch.cuda.current_stream()
    stream.wait_stream(cur)
    with torch.cuda.stream(stream):
        ddp = DistributedDataParallel(model, **kwargs)
    cur.wait_stream(stream)
    ddp._umamd_stream = stream
    return ddp


def count_sync_bn(model: Module) -> int:
    return sum(isinstance(m, SyncBatchNorm) for m in model.modules())


def is_data_parallel(model: Module) -> bool:
    return isinstance(model, DistributedDataParallel)


def unwrap(model: Module) -> Module:
    return model.module if isinstance(model, DistributedDataParallel) else model


__all__ = ['data_parallel', 'count_sync_bn', 'is_data_parallel', 'unwrap', 'torch']
