"""EfficientAttention (reference model/layers/attention.py:7-76).

Same constructor, parameters (keys/queries/values/reprojection 1x1 convs) and
state_dict names; the forward runs ``umamd.functional.attention_block``: one
QKV GEMM on MFMA, the per-head linear-attention core and the reprojection
GEMM with the residual fused into its epilogue.
"""
import torch.nn as nn
from torch import Tensor

from umamd import functional as U
from umamd.layout import to_nhwc, to_nchw


class EfficientAttention(nn.Module):
    def __init__(self, image_channels: int, key_channels: int,
                 value_channels: int, head_size: int) -> None:
        super().__init__()
        if not (image_channels == key_channels == value_channels):
            raise NotImplementedError('umamd EfficientAttention: image/key/value channels '
                                      'must be equal (as in every reference config)')
        self.image_channels = image_channels
        self.key_channels = key_channels
        self.value_channels = value_channels
        self.head_size = head_size
        self.key_channels_per_head = key_channels // head_size
        self.value_channels_per_head = value_channels // head_size
        self.keys = nn.Conv2d(image_channels, key_channels, 1)
        self.queries = nn.Conv2d(image_channels, key_channels, 1)
        self.values = nn.Conv2d(image_channels, value_channels, 1)
        self.reprojection = nn.Conv2d(value_channels, image_channels, 1)

    def _fwd(self, x_nhwc: Tensor) -> Tensor:
        return U.attention_block(x_nhwc, self)

    def forward(self, x: Tensor) -> Tensor:
        return to_nchw(self._fwd(to_nhwc(x)))
