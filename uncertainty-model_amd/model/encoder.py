"""RandomEncoder (reference model/encoder.py:9-53): five EncoderStages in
sequence, Xavier-uniform init on every Conv2d (:38-40)."""
from typing import List, Optional, Tuple

import torch.nn as nn
from torch import Tensor

from umamd.layout import to_nhwc, to_nchw

from .layers.encoder import EncoderStage


class RandomEncoder(nn.Module):
    def __init__(self, layers: List[dict], load_graph: Optional[str] = None,
                 nodes: int = 5, seed: int = 42) -> None:
        super().__init__()
        self.layers = nn.ModuleList()
        for i, layer_config in enumerate(layers):
            self.layers.append(EncoderStage(**layer_config, stage=(i + 1), nodes=nodes,
                                            seed=seed, load_graph=load_graph))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.xavier_uniform_(m.weight)

    def _fwd(self, x: Tensor) -> Tuple[Tensor, ...]:
        encodings = []
        for layer in self.layers:
            x = layer._fwd(x)
            encodings.append(x)
        return tuple(encodings)

    def forward(self, x: Tensor) -> Tuple[Tensor, ...]:
        return tuple(to_nchw(e) for e in self._fwd(to_nhwc(x)))
