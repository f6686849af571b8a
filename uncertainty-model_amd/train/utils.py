"""Training utilities (reference train/utils.py), HIP-backed where they are on
the hot path:

  scale_pyramid        utils.py:27-50   -> um_pyramid (every level, one launch)
  reconstruct(+L/R)    utils.py:65-109  -> um_warp / um_warp_bwd
  reconstruct_pyramid  utils.py:112-135 -> um_recon_pyramid (one launch; tagged
                                           for the fused loss)
  l1_loss, detach_pyramid, concatenate_pyramids, adjust_disparity,
  adjust_learning_rate, prepare_state_dict: host-side, same semantics.
"""
from typing import Callable, List, OrderedDict, Union

import numpy as np
import torch
from torch import Tensor
from torch.optim import Optimizer

from umamd import lossfn as LF

Device = Union[torch.device, str]
ImagePyramid = List[Tensor]
LRAdjuster = Callable[[Optimizer, int, float, bool], None]
ScaleAdjuster = Callable[[int], float]
Loss = List[float]


def l1_loss(x: Tensor, y: Tensor) -> Tensor:
    """Mean absolute difference (utils.py:22-24)."""
    return (x - y).abs().mean()


def scale_pyramid(x: Tensor, scales: int) -> ImagePyramid:
    """Bilinear (align_corners=True) resizes of x to H/2^i x W/2^i."""
    return LF.scale_pyramid(x, scales)


def detach_pyramid(pyramid: ImagePyramid) -> ImagePyramid:
    return [layer.detach().clone() for layer in pyramid]


def reconstruct(disparity: Tensor, opposite_image: Tensor) -> Tensor:
    """Warp ``opposite_image`` by ``disparity`` (grid_sample semantics of
    utils.py:77-97, including the non-identity linspace base grid, F6)."""
    return LF.reconstruct(disparity, opposite_image, 1.0)


def reconstruct_left_image(left_disparity: Tensor, right_image: Tensor) -> Tensor:
    return LF.reconstruct(left_disparity, right_image, -1.0)


def reconstruct_right_image(right_disparity: Tensor, left_image: Tensor) -> Tensor:
    return LF.reconstruct(right_disparity, left_image, 1.0)


def reconstruct_pyramid(disparities: ImagePyramid, pyramid: ImagePyramid) -> ImagePyramid:
    return LF.reconstruct_pyramid(disparities, pyramid)


def concatenate_pyramids(a: ImagePyramid, b: ImagePyramid) -> ImagePyramid:
    return [torch.cat((x, y), 0) for x, y in zip(a, b)]


def adjust_disparity(epoch: int, m: float = 0.02, c: float = 0.0,
                     step: float = 0.2, offset: float = 0.1,
                     min_scale: float = 0.3, max_scale: float = 1.0) -> float:
    """Quantised linear disparity-scale schedule (utils.py:143-174)."""
    scale = ((epoch + 1) * m) + c
    scale = (round((scale + offset) / step) * step) - offset
    return np.clip(scale, min_scale, max_scale)


def prepare_state_dict(state_dict: OrderedDict) -> dict:
    """Strip the DDP ``module.`` prefix (utils.py:328-330)."""
    return {k.replace('module.', ''): v for k, v in state_dict.items()}


def adjust_learning_rate(optimiser: Optimizer, epoch: int, lr: float,
                         finetune: bool = False) -> None:
    """lr / 2 after 30 epochs, / 4 after 40 or when fine-tuning (utils.py:333-353)."""
    if epoch > 40 or finetune:
        target = lr / 4
    elif epoch > 30:
        target = lr / 2
    else:
        target = lr
    for group in optimiser.param_groups:
        group['lr'] = target


def run_discriminator(*args, **kwargs):
    raise NotImplementedError('umamd: adversarial training (run_discriminator, reference '
                              'train/utils.py:248-273) is not implemented yet')
