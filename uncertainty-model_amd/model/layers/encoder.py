"""Encoder layers (reference model/layers/encoder.py:1-262), HIP-backed.

Module names, constructor kwargs, parameters and state_dict keys follow the
reference exactly; forwards run the umamd kernels on NHWC activations:

* ``ConvELUBlock``  zero-pad + Conv2d + BatchNorm2d(train) + ELU as one
  autograd node (implicit-GEMM conv with BN partial sums in the epilogue).
* ``NodeBlock``     sigmoid-weighted predecessor merge with the reference's
  index mapping (F3: inputs 0 and 1 both use mean_weight[0]).
* ``GraphBlock``    DAG evaluation in id order; multiple output nodes are
  averaged out of place (the reference's in-place sum breaks autograd, F4).
* ``EncoderStage``  GraphBlock -> EfficientAttention.
"""
import os
import os.path
from typing import Optional, Tuple, Union

import torch
import torch.nn as nn
from torch import Tensor

from umamd import functional as U
from umamd._lib import PAD_ZERO
from umamd.layout import to_nhwc, to_nchw

from .attention import EfficientAttention
from .. import graph as g
from ..graph import Node

KernelSize = Union[int, Tuple[int, int]]
StrideSize = Union[int, Tuple[int, int]]


class ConvELUBlock(nn.Module):
    """Zero-padding -> Conv2d -> BatchNorm2d -> ELU (reference :21-52)."""

    def __init__(self, in_channels: int, out_channels: int,
                 kernel_size: KernelSize, stride: StrideSize) -> None:
        super().__init__()
        self.layers = nn.Sequential(
            nn.Conv2d(in_channels, out_channels, kernel_size, stride),
            nn.BatchNorm2d(out_channels),
            nn.ELU(inplace=True))
        padding_size = (kernel_size - 1) // 2
        self.padding = tuple([padding_size] * 4)

    def _fwd(self, x: Tensor) -> Tensor:
        return U.conv_bn_elu(x, self.layers[0], self.layers[1], self.padding[0], PAD_ZERO)

    def forward(self, x: Tensor) -> Tensor:
        return to_nchw(self._fwd(to_nhwc(x)))


class NodeBlock(nn.Module):
    """One graph node: weighted merge of its inputs, then ConvELUBlock
    (reference :55-127).  Input nodes convolve with stride 2."""

    def __init__(self, node: Node, in_channels: int, out_channels: int,
                 kernel_size: KernelSize) -> None:
        super().__init__()
        self.numberof_inputs = len(node.inputs)
        initial_means = torch.ones(self.numberof_inputs)
        self.mean_weight = nn.Parameter(initial_means) \
            if self.numberof_inputs > 1 else None
        if node.node_type == 'input':
            stride = 2
        else:
            in_channels = out_channels
            stride = 1
        self.convolution = ConvELUBlock(in_channels, out_channels, kernel_size, stride=stride)

    @staticmethod
    def weight_index(n_inputs: int):
        """Reference merge (:116-123): input 0 -> w[0], input i>=1 -> w[i-1]."""
        return [0] + list(range(n_inputs - 1))

    def _fwd(self, *inputs: Tensor) -> Tensor:
        if self.numberof_inputs > 1:
            for x in inputs[1:]:
                if x.shape != inputs[0].shape:
                    raise NotImplementedError('umamd NodeBlock: inputs of different sizes '
                                              '(reflect resize, reference :92-113) are not '
                                              'produced by any Watts-Strogatz stage graph')
            out = U.merge(inputs, self.mean_weight, self.weight_index(len(inputs)))
        else:
            out = inputs[0]
        return self.convolution._fwd(out)

    def forward(self, *inputs: Tensor) -> Tensor:
        return to_nchw(self._fwd(*[to_nhwc(x) for x in inputs]))


class GraphBlock(nn.Module):
    """All NodeBlocks of one random graph (reference :130-198)."""

    def __init__(self, graph, in_channels: int, out_channels: int,
                 kernel_size: KernelSize) -> None:
        super().__init__()
        self.nodes, self.in_nodes, self.out_nodes = g.get_graph_info(graph)
        self.node_blocks = nn.ModuleList()
        for node in self.nodes:
            self.node_blocks.append(NodeBlock(node, in_channels, out_channels, kernel_size))

    def _fwd(self, x: Tensor) -> Tensor:
        if U._STAGE_FN:  # the whole block as one autograd node (umamd.functional.GraphBlockFn)
            return U.graph_block(x, self)
        results = {idx: self.node_blocks[idx]._fwd(x) for idx in self.in_nodes}
        for idx, node in enumerate(self.nodes):
            if idx in self.in_nodes:
                continue
            inputs = [results[i] for i in node.inputs]
            results[idx] = self.node_blocks[idx]._fwd(*inputs)
        outs = [results[i] for i in self.out_nodes]
        if len(outs) == 1:
            return outs[0]
        k = len(outs)
        return U.merge(outs, None, [0] * k, [1.0 / k] * k)

    def forward(self, x: Tensor) -> Tensor:
        return to_nchw(self._fwd(to_nhwc(x)))


class EncoderStage(nn.Module):
    """GraphBlock + EfficientAttention (reference :201-262)."""

    def __init__(self, in_channels: int, out_channels: int,
                 kernel_size: KernelSize, stage: int, heads: int = 8,
                 nodes: int = 5, p: float = 0.75, k: int = 4,
                 seed: Optional[int] = None,
                 load_graph: Optional[str] = None,
                 save_graph: Optional[str] = None) -> None:
        super().__init__()
        if load_graph is not None:
            filepath = os.path.join(load_graph, f'stage_{stage}.gpickle')
            graph = g.load_graph(filepath)
        else:
            graph = g.build_graph(nodes, k, p, seed=(stage * seed))
            if save_graph is not None:
                directory_path = os.path.join(save_graph, f'nodes_{nodes}_seed_{seed}')
                os.makedirs(directory_path, exist_ok=True)
                g.save_graph(graph, os.path.join(directory_path, f'stage_{stage}.gpickle'))
        self.layers = nn.Sequential(
            GraphBlock(graph, in_channels, out_channels, kernel_size),
            EfficientAttention(out_channels, out_channels, out_channels, heads))

    def _fwd(self, x: Tensor) -> Tensor:
        return self.layers[1]._fwd(self.layers[0]._fwd(x))

    def forward(self, x: Tensor) -> Tensor:
        return to_nchw(self._fwd(to_nhwc(x)))
