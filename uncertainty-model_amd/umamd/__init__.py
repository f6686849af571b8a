"""umamd: MI355X (gfx950) HIP kernels + autograd glue for the
depth+uncertainty training step.  ``import umamd`` does not touch the GPU;
the HIP library is loaded on first kernel call (no CPU fallback)."""
import os

import torch

from . import _lib  # noqa: F401

_DTYPES = {'fp32': torch.float32, 'float32': torch.float32, 'f32': torch.float32,
           'bf16': torch.bfloat16, 'bfloat16': torch.bfloat16}


def default_dtype() -> torch.dtype:
    """Compute dtype of new models: env UMAMD_DTYPE in {fp32, bf16}; fp32 default
    (reference precision).  bf16 keeps f32 master weights, f32 BN statistics,
    f32 loss stack and f32 warp coordinates."""
    return _DTYPES[os.environ.get('UMAMD_DTYPE', 'fp32').lower()]


def resolve_dtype(d) -> torch.dtype:
    if d is None:
        return default_dtype()
    if isinstance(d, torch.dtype):
        return d
    return _DTYPES[str(d).lower()]
