"""Training utilities (reference train/utils.py), HIP-backed where they are on
the hot path:

  scale_pyramid        utils.py:27-50   -> um_pyramid (every level, one launch)
  reconstruct(+L/R)    utils.py:65-109  -> um_warp / um_warp_bwd
  reconstruct_pyramid  utils.py:112-135 -> um_recon_pyramid (one launch; tagged
                                           for the fused loss)
  l1_loss, detach_pyramid, concatenate_pyramids, adjust_disparity,
  adjust_learning_rate, prepare_state_dict: host-side, same semantics.
"""
from typing import Callable, List, Optional, OrderedDict, Union

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


def run_discriminator(image_pyramid: ImagePyramid, recon_pyramid: ImagePyramid,
                      discriminator, disc_loss_function, batch_size: int) -> Tensor:
    """Discriminator predictions on real (label 1) and detached reconstructed
    (label 0) pyramids and its loss / 2 (reference :248-273)."""
    recon_pyramid = detach_pyramid(recon_pyramid)
    pyramid = concatenate_pyramids(image_pyramid, recon_pyramid)
    predictions = discriminator(pyramid)
    labels = torch.zeros_like(predictions)
    labels[:batch_size] = 1
    return disc_loss_function(predictions, labels) / 2


# ------------------------------------------------ visualisation (host) ----
# reference train/utils.py:177-245,276-325 and the torchvision.utils
# make_grid / save_image they rely on (torchvision is not in this image)
def to_heatmap(x: Tensor, device: Device = 'cpu', inverse: bool = False,
               colour_map: str = 'inferno') -> Tensor:
    """Single-channel image -> RGB heatmap (reference :177-199)."""
    import matplotlib.pyplot as plt
    image = x.squeeze(0).detach().float().cpu().numpy()
    image = 1 - image if inverse else image
    heatmap = plt.get_cmap(colour_map)(image)[:, :, :3]
    return torch.from_numpy(heatmap).to(device).permute(2, 0, 1)


def combine_disparity(left: Tensor, right: Tensor, device: Device = 'cpu',
                      alpha: float = 20, beta: float = 0.05) -> Tensor:
    """Monodepth2-style blind-spot blend of the two views (reference :202-245)."""
    left_disp = left.detach().cpu().numpy()
    right_disp = right.detach().cpu().numpy()
    mean_disp = (left_disp + right_disp) / 2
    _, height, width = mean_disp.shape
    xv, _ = np.meshgrid(np.linspace(0, 1, width), np.linspace(0, 1, height))
    left_mask = 1 - np.clip(alpha * (xv - beta), 0, 1)
    right_mask = np.fliplr(left_mask)
    mean_mask = 1 - (left_mask + right_mask)
    combined = (right_mask * left_disp) + (left_mask * right_disp) + (mean_mask * mean_disp)
    return torch.from_numpy(combined).to(device)


def make_grid(tensor: Tensor, nrow: int = 8, padding: int = 2, pad_value: float = 0.0) -> Tensor:
    """torchvision.utils.make_grid (no normalisation) for a [B,C,H,W] batch."""
    t = tensor.detach()
    if t.dim() == 3:
        t = t.unsqueeze(0)
    if t.shape[1] == 1:
        t = t.repeat(1, 3, 1, 1)
    nmaps = t.shape[0]
    xmaps = min(nrow, nmaps)
    ymaps = (nmaps + xmaps - 1) // xmaps
    height, width = t.shape[2] + padding, t.shape[3] + padding
    grid = t.new_full((t.shape[1], height * ymaps + padding, width * xmaps + padding), pad_value)
    k = 0
    for y in range(ymaps):
        for x in range(xmaps):
            if k >= nmaps:
                break
            grid[:, y * height + padding:(y + 1) * height, x * width + padding:(x + 1) * width] = t[k]
            k += 1
    return grid


def save_image(tensor: Tensor, fp: str) -> None:
    """torchvision.utils.save_image of a [C,H,W] image in [0, 1]."""
    from PIL import Image
    grid = make_grid(tensor) if tensor.dim() == 4 else tensor.detach()
    arr = grid.float().mul(255).add_(0.5).clamp_(0, 255).permute(1, 2, 0).to('cpu', torch.uint8)
    Image.fromarray(arr.numpy()).save(fp)


def get_comparison(image: Tensor, prediction: Tensor, extra: Optional[Tensor],
                   add_scaled: bool = False, device: Device = 'cpu') -> Tensor:
    """Grid of the stereo images, disparity heatmaps and an extra pair (reference :276-325)."""
    image, prediction = image.detach().float().cpu(), prediction.detach().float().cpu()
    left_image, right_image = torch.split(image, [3, 3], dim=0)
    left_pred, right_pred = torch.split(prediction, [1, 1], dim=0)
    min_pred, max_pred = prediction.min(), prediction.max()
    scaled_left_pred = (left_pred - min_pred) / (max_pred - min_pred)
    scaled_right_pred = (right_pred - min_pred) / (max_pred - min_pred)
    left_pred = to_heatmap(left_pred).float()
    right_pred = to_heatmap(right_pred).float()
    if extra is not None:
        extra = extra.detach().float().cpu()
        extra_split = [3, 3] if extra.size(0) == 6 else [1, 1]
        left_extra, right_extra = torch.split(extra, extra_split, dim=0)
        if extra.size(0) == 2:
            left_extra = to_heatmap(left_extra).float()
            right_extra = to_heatmap(right_extra).float()
    images = torch.stack((left_image, right_image, left_pred, right_pred))
    if add_scaled:
        images = torch.cat((images, to_heatmap(scaled_left_pred).float().unsqueeze(0),
                            to_heatmap(scaled_right_pred).float().unsqueeze(0)))
    if extra is not None:
        images = torch.cat((images, left_extra.unsqueeze(0), right_extra.unsqueeze(0)))
    return make_grid(images, nrow=2).to(device)
