"""DepthDecoder (reference model/decoder.py:11-62): five DecoderStages wired
with the encoder skips; train mode returns (disp1..disp4), eval disp1."""
from typing import List, Tuple, Union

import torch
import torch.nn as nn
from torch import Tensor

from umamd.layout import to_nhwc, to_nchw

from .layers.decoder import DecoderStage

DecoderOut = Union[Tuple[Tensor, ...], Tensor]


class DepthDecoder(nn.Module):
    def __init__(self, layers: List[dict]) -> None:
        super().__init__()
        self.layers = nn.ModuleList()
        for layer_config in layers:
            self.layers.append(DecoderStage(**layer_config))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.xavier_uniform_(m.weight)

    def _fwd(self, left_image: Tensor, *feature_maps: Tensor, scale: float = 1):
        """NHWC in, f32 NHWC disparities out (disp1 full resolution first)."""
        f1, f2, f3, f4, x4 = feature_maps
        out5, skip5, _ = self.layers[0]._fwd(x4, f4, x4, None, scale)
        out4, skip4, disp4 = self.layers[1]._fwd(out5, f3, skip5, None, scale)
        out3, skip3, disp3 = self.layers[2]._fwd(out4, f2, skip4, disp4, scale)
        out2, skip2, disp2 = self.layers[3]._fwd(out3, f1, skip3, disp3, scale)
        _, _, disp1 = self.layers[4]._fwd(out2, left_image, skip2, disp2, scale)
        return disp1, disp2, disp3, disp4

    def forward(self, left_image: Tensor, *feature_maps: Tensor,
                scale: float = 1) -> DecoderOut:
        dt = feature_maps[0].dtype
        dt = dt if dt in (torch.float32, torch.bfloat16) else torch.float32
        disps = self._fwd(to_nhwc(left_image, dt), *[to_nhwc(f, dt) for f in feature_maps],
                          scale=scale)
        disps = tuple(to_nchw(d) for d in disps)
        return disps if self.training else disps[0]
