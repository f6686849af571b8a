"""Decoder layers (reference model/layers/decoder.py:1-249), HIP-backed.

Same classes, kwargs, parameters and state_dict keys.  ``DecoderStage``
runs on NHWC activations:

  cat1  = [feature_map | bilinear_x2(skip) * gate_prev]      (um_concat_build)
  u1, s = ConvELU(1x1)+BN -> SE gate s = sigmoid(W2 relu(W1 mean(u1)))
  x_up  = PixelShuffle(ConvELU3x3reflect+BN(x))               (folded into cat2)
  cat2  = [x_up | u1 * s | bilinear_x2(disp_prev)]
  out   = ConvELU3x3reflect+BN(cat2);  disp = scale * sigmoid(Conv3x3reflect(out))

The SE product u1 * s is never materialised: it is applied as a per-(n,c)
gate wherever the skip is read (here and in the next stage's cat1).
"""
from typing import Optional, Tuple, Union

import torch
import torch.nn as nn
from torch import Tensor

from umamd import functional as U
from umamd._lib import CAT_COPY, CAT_PSHUF, CAT_UP2, PAD_REFLECT, PAD_ZERO
from umamd.layout import to_nhwc, to_nchw

KernelSize = Union[int, Tuple[int, int]]


class ConvLayer(nn.Module):
    """(Reflection|Zero)Pad2d(1)? -> Conv2d -> Sigmoid? (reference :11-52)."""

    def __init__(self, in_channels: int, out_channels: int,
                 padding: bool = True, reflection: bool = True,
                 sigmoid: bool = False, kernel_size: KernelSize = 3) -> None:
        super().__init__()
        if padding:
            self.padding = nn.ReflectionPad2d(1) if reflection else nn.ZeroPad2d(1)
        else:
            self.padding = None
        self.layers = nn.Sequential(
            nn.Conv2d(in_channels, out_channels, kernel_size=kernel_size),
            nn.Sigmoid() if sigmoid else nn.Identity())

    def pad_args(self):
        if self.padding is None:
            return 0, PAD_ZERO
        mode = PAD_REFLECT if isinstance(self.padding, nn.ReflectionPad2d) else PAD_ZERO
        return 1, mode


class ConvELUBlock(nn.Module):
    """ConvLayer -> BatchNorm2d? -> ELU (reference :55-87)."""

    def __init__(self, in_channels: int, out_channels: int,
                 padding: bool = True, kernel_size: KernelSize = 3,
                 batch_norm: bool = False) -> None:
        super().__init__()
        self.layers = nn.Sequential(
            ConvLayer(in_channels, out_channels, padding=padding, kernel_size=kernel_size),
            nn.BatchNorm2d(out_channels) if batch_norm else nn.Identity(),
            nn.ELU(inplace=True))

    def _fwd(self, x: Tensor, se: Optional['SELayer'] = None, segs=None):
        conv_layer = self.layers[0]
        pad, mode = conv_layer.pad_args()
        bn = self.layers[1] if isinstance(self.layers[1], nn.modules.batchnorm._BatchNorm) \
            else None
        return U.conv_bn_elu(x, conv_layer.layers[0], bn, pad, mode, se=se, segs=segs)

    def forward(self, x: Tensor) -> Tensor:
        return to_nchw(self._fwd(to_nhwc(x)))


class SELayer(nn.Module):
    """Squeeze-excitation (reference :90-136).  The HIP path supports fc=True
    (the reference default and the only configured variant)."""

    def __init__(self, channels: int, reduction: int = 16, fc: bool = True) -> None:
        super().__init__()
        self.fc = fc
        self.channels_reduced = channels // reduction
        self.squeeze = nn.AdaptiveAvgPool2d(1)
        self.excite = nn.Sequential(
            nn.Linear(channels, self.channels_reduced, bias=False)
            if fc else nn.Conv2d(channels, self.channels_reduced, kernel_size=1, stride=1,
                                 bias=True),
            nn.ReLU(inplace=True),
            nn.Linear(self.channels_reduced, channels, bias=False)
            if fc else nn.Conv2d(self.channels_reduced, channels, kernel_size=1, stride=1,
                                 bias=True),
            nn.Sigmoid())
        if not fc:
            raise NotImplementedError('umamd SELayer: only fc=True is implemented')


class DecoderStage(nn.Module):
    """One decoder stage (reference :139-249)."""
    DecoderOut = Tuple[Tensor, Tensor, Optional[Tensor]]

    def __init__(self, in_channels: int, feature_in_channels: int,
                 skip_in_channels: int, upsample_channels: int,
                 out_channels: int, skip_out_channels: int,
                 disp_channels: int = 2, batch_norm: bool = True,
                 fc: bool = True, scale: int = 2, concat_disp: bool = True,
                 calculate_disp: bool = True) -> None:
        super().__init__()
        if scale != 2:
            raise NotImplementedError('umamd DecoderStage: only scale=2 is implemented')
        self.scale = scale
        self.calculate_disp = calculate_disp
        self.concat_disp = concat_disp
        self.feature_in_channels = feature_in_channels
        self.skip_in_channels = skip_in_channels
        self.upsample_channels = upsample_channels
        self.skip_out_channels = skip_out_channels
        self.disp_channels = disp_channels
        self.upsample = nn.Sequential(
            ConvELUBlock(in_channels, upsample_channels * int(scale ** 2),
                         batch_norm=batch_norm),
            nn.PixelShuffle(upscale_factor=self.scale))
        self.squeeze_excite = nn.Sequential(
            ConvELUBlock(feature_in_channels + skip_in_channels, skip_out_channels,
                         kernel_size=1, batch_norm=True, padding=False),
            SELayer(channels=skip_out_channels, fc=fc))
        iconv_in_channels = upsample_channels + skip_out_channels
        iconv_in_channels += disp_channels if concat_disp else 0
        self.iconv = ConvELUBlock(iconv_in_channels, out_channels, batch_norm=batch_norm)
        self.disp = ConvLayer(out_channels, disp_channels, sigmoid=True) \
            if self.calculate_disp else None

    def _fwd(self, x: Tensor, feature_map: Tensor, skip, disparity: Optional[Tensor] = None,
             scale: float = 1.0):
        """NHWC forward.  ``skip`` is an NHWC tensor or a (tensor, gate) pair;
        ``disparity`` is the previous stage's f32 NHWC [N,h,w,dc] output.
        Returns (out, (u1, gate), disp)."""
        N, H, W, _ = feature_map.shape
        dtype = x.dtype
        skip_t, skip_g = skip if isinstance(skip, tuple) else (skip, None)
        se_block = self.squeeze_excite[0]
        if U._SKIP_CONV and isinstance(se_block.layers[1], nn.modules.batchnorm._BatchNorm) \
                and se_block.layers[0].padding is None \
                and tuple(se_block.layers[0].layers[0].kernel_size) == (1, 1):
            # 1x1 conv of cat(feature_map, up2(skip)) with the skip half at
            # the skip's resolution (umamd.functional.SkipConvFn)
            u1, gate = U.skip_conv_bn_elu(feature_map, skip_t, skip_g,
                                          se_block.layers[0].layers[0], se_block.layers[1],
                                          self.squeeze_excite[1], self.feature_in_channels,
                                          self.skip_in_channels)
        else:
            cat1, segs1 = U.concat([U.CatSource(feature_map, CAT_COPY, self.feature_in_channels),
                                    U.CatSource(skip_t, CAT_UP2, self.skip_in_channels, skip_g)],
                                   N, H, W, dtype)
            u1, gate = se_block._fwd(cat1, se=self.squeeze_excite[1], segs=segs1)
        xu = self.upsample[0]._fwd(x)  # [N, H/2, W/2, 4*Cu]; pixel shuffle folded into cat2
        srcs = [U.CatSource(xu, CAT_PSHUF, self.upsample_channels),
                U.CatSource(u1, CAT_COPY, self.skip_out_channels, gate)]
        if self.concat_disp:
            srcs.append(U.CatSource(disparity, CAT_UP2, self.disp_channels))
        cat2, segs2 = U.concat(srcs, N, H, W, dtype)
        out = self.iconv._fwd(cat2, segs=segs2)
        disp = U.disp_head(out, self.disp.layers[0], scale) if self.calculate_disp else None
        return out, (u1, gate), disp

    def forward(self, x: Tensor, feature_map: Tensor, skip: Tensor,
                disparity: Optional[Tensor] = None,
                scale: Optional[float] = 1.0) -> DecoderOut:
        dt = x.dtype if x.dtype in (torch.float32, torch.bfloat16) else torch.float32
        d = to_nhwc(disparity, torch.float32) if disparity is not None else None
        out, (u1, gate), disp = self._fwd(to_nhwc(x, dt), to_nhwc(feature_map, dt),
                                          to_nhwc(skip, dt), d, scale)
        skip_out = to_nchw(u1) * gate.to(u1.dtype)[:, :, None, None]
        return to_nchw(out), skip_out, (to_nchw(disp) if disp is not None else None)
