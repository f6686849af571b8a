"""RandomDiscriminator (reference model/discriminator.py:13-86), HIP-backed.

Same constructor kwargs (config.yml ``discriminator``), module names and
state_dict keys as the reference: EncoderStages over the image pyramid
(stage i sees cat(previous features, pyramid level i)), a final EncoderStage
and Linear(linear_in_features, 1) + sigmoid.  The stages run on the encoder
kernels on NHWC activations; the channel concat is the decoder's one-launch
concat, the flatten + Linear + sigmoid one small head kernel whose weight
indexing follows the reference's NCHW ``view`` (umamd.discfn).
"""
from typing import List, Optional

import torch
import torch.nn as nn
from torch import Tensor

import umamd
from umamd import discfn as D
from umamd import functional as U
from umamd import packer as P
from umamd._lib import CAT_COPY
from umamd.layout import to_nchw

from .layers.encoder import EncoderStage

ImagePyramid = List[Tensor]


class RandomDiscriminator(nn.Module):
    def __init__(self, layers: List[dict], final_conv: dict, linear_in_features: int,
                 load_graph: Optional[str] = None, nodes: int = 5, seed: int = 42,
                 dtype=None) -> None:
        super().__init__()
        self.layers = nn.ModuleList()
        for i, layer_config in enumerate(layers):
            self.layers.append(EncoderStage(**layer_config, stage=(i + 1), nodes=nodes, seed=seed,
                                            load_graph=load_graph))
        self.conv = EncoderStage(**final_conv, stage=(len(self.layers) + 1), nodes=nodes,
                                 seed=seed, load_graph=load_graph)
        self.linear = nn.Linear(linear_in_features, 1)
        self.compute_dtype = umamd.resolve_dtype(dtype)
        self._packer = P.WeightPacker()

    def _features(self, pyramid: ImagePyramid) -> List[Tensor]:
        """NHWC feature maps of the stages (reference :53-76)."""
        feats = []
        out = None
        for i, (images, layer) in enumerate(zip(pyramid, self.layers)):
            img = D.image_to_nhwc(images, self.compute_dtype)
            if i == 0:
                x = img
            else:
                N, H, W, _ = out.shape
                x, segs = U.concat([U.CatSource(out, CAT_COPY, out.shape[-1]),
                                    U.CatSource(img, CAT_COPY, images.shape[1])],
                                   N, H, W, self.compute_dtype)
                if segs is not None:
                    raise NotImplementedError('umamd RandomDiscriminator: stage widths must be '
                                              'multiples of 8')
            out = layer._fwd(x)
            feats.append(out)
        return feats

    def features(self, pyramid: ImagePyramid) -> ImagePyramid:
        with P.scope(self._packer):
            return [to_nchw(f) for f in self._features(pyramid)]

    def forward(self, pyramid: ImagePyramid) -> Tensor:
        with P.scope(self._packer):
            feature = self._features(pyramid)[-1]
            out = self.conv._fwd(feature)
        return D.disc_head(out, self.linear)
