"""Layout plumbing between the reference's NCHW module interface and the
NHWC tensors the kernels use.  An NHWC-contiguous tensor permuted to NCHW is
a channels_last tensor, so these are zero-copy in the common case."""
import torch

from . import functional as U


def compute_dtype_of(t: torch.Tensor) -> torch.dtype:
    return t.dtype if t.dtype in (torch.float32, torch.bfloat16) else torch.float32


def to_nhwc(x: torch.Tensor, dtype: torch.dtype = None) -> torch.Tensor:
    """logical [N,C,H,W] -> NHWC [N,H,W,Cp] (Cp = ceil8(C))."""
    dtype = dtype or compute_dtype_of(x)
    N, C, H, W = x.shape
    v = x.permute(0, 2, 3, 1)
    if C % 8 == 0 and v.is_contiguous() and v.dtype == dtype:
        return v
    if C % 8 == 0:
        return v.to(dtype).contiguous()
    return U.image_to_nhwc(x, dtype)


def to_nchw(x_nhwc: torch.Tensor, C: int = None) -> torch.Tensor:
    """NHWC [N,H,W,Cp] -> logical NCHW view (channels_last memory)."""
    v = x_nhwc.permute(0, 3, 1, 2)
    if C is not None and C != v.shape[1]:
        v = v[:, :C]
    return v
