"""RandomlyConnectedModel (reference model/model.py:8-23), HIP-backed.

``forward(image [B,3,H,W] f32, scale)`` returns four disparity/uncertainty
maps (train) or the full-resolution one (eval), as float32 tensors of logical
shape [B,4,h,w] in channels-last memory.  The compute dtype is float32 by
default (reference precision) or bfloat16 (``dtype='bf16'`` or
UMAMD_DTYPE=bf16): activations and conv operands in bf16, f32 accumulation,
f32 master weights, f32 BN statistics, f32 disparity heads and loss.
"""
import torch
import torch.nn as nn
from torch import Tensor

import umamd
from umamd import functional as U
from umamd import packer as P

from .decoder import DepthDecoder, DecoderOut
from .encoder import RandomEncoder


class RandomlyConnectedModel(nn.Module):
    def __init__(self, encoder: dict, decoder: dict, dtype=None) -> None:
        super().__init__()
        self.encoder = RandomEncoder(**encoder)
        self.decoder = DepthDecoder(**decoder)
        self.compute_dtype = umamd.resolve_dtype(dtype)
        self._packer = P.WeightPacker()  # packed conv weights, one refresh launch per forward
        self._stats = U.StatArena()      # BN statistics slots, one zero fill per forward

    def forward(self, image: Tensor, scale: float = 1) -> DecoderOut:
        _, _, h, w = image.shape
        if h % 32 or w % 32:
            raise ValueError(f'image size {h}x{w}: height and width must be multiples of 32')
        x = U.image_to_nhwc(image, self.compute_dtype)
        with P.scope(self._packer), U.stat_scope(self._stats, x.device), U.grad_slots():
            feats = self.encoder._fwd(x)
            disps = self.decoder._fwd(x, *feats, scale=float(scale))
        disps = tuple(d.permute(0, 3, 1, 2) for d in disps)  # logical NCHW, NHWC memory
        return disps if self.training else disps[0]


Model = RandomlyConnectedModel
