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
                  sync_bn: bool = True) -> DistributedDataParallel:
    if sync_bn:  # torch only accepts SyncBatchNorm under DDP for device modules
        model = SyncBatchNorm.convert_sync_batchnorm(model, process_group)
    kwargs = dict(process_group=process_group, bucket_cap_mb=bucket_cap_mb,
                  gradient_as_bucket_view=True)
    if device_index is not None:
        kwargs['device_ids'] = [device_index]
    return DistributedDataParallel(model, **kwargs)


def count_sync_bn(model: Module) -> int:
    return sum(isinstance(m, SyncBatchNorm) for m in model.modules())


def is_data_parallel(model: Module) -> bool:
    return isinstance(model, DistributedDataParallel)


def unwrap(model: Module) -> Module:
    return model.module if isinstance(model, DistributedDataParallel) else model


__all__ = ['data_parallel', 'count_sync_bn', 'is_data_parallel', 'unwrap', 'torch']
