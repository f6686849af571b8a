"""Evaluation loop (reference train/evaluate.py:25-196).

Same signature, metrics and logging as the reference.  The per-batch work runs
on the HIP path: the eval-mode model, the two reconstructions, the 11x11
gaussian SSIM (torchmetrics semantics, umamd.evalfn.ssim), the image error
map (WeightedSSIMLoss.image_error with alpha = 1) and the AUSE/AURG
sparsification curves.  Comparison images (save_comparisons) are host-side
visualisation, written only for the first batch when a directory is given.
"""
import os.path
from typing import Optional, Tuple

import torch
from torch.nn import Module
from torch.utils.data import DataLoader

from umamd import evalfn as EF

from . import sparsification as spars
from . import utils as u
from .loss import WeightedSSIMLoss
from .utils import Device

try:
    import tqdm
except ImportError:  # pragma: no cover
    tqdm = None


def save_comparisons(image, disparity, uncertainty, recon, error, directory: str,
                     epoch_number: Optional[int] = None, is_final: bool = True,
                     device: Device = 'cpu') -> None:
    """prediction.png / disparity.png / uncertainty.png (reference :25-63)."""
    prediction_image = u.get_comparison(image, disparity, uncertainty, add_scaled=False,
                                        device=device)
    disparity_image = u.get_comparison(image, disparity, recon, add_scaled=True, device=device)
    uncertainty_image = u.get_comparison(image, uncertainty, error, add_scaled=True,
                                         device=device)
    dirname = 'final' if is_final else f'epoch_{epoch_number:03}'
    epoch_directory = os.path.join(directory, dirname)
    os.makedirs(epoch_directory, exist_ok=True)
    print(f'Saving comparisons to:\n\t{epoch_directory}')
    u.save_image(prediction_image, os.path.join(epoch_directory, 'prediction.png'))
    u.save_image(disparity_image, os.path.join(epoch_directory, 'disparity.png'))
    u.save_image(uncertainty_image, os.path.join(epoch_directory, 'uncertainty.png'))


@torch.no_grad()
def evaluate_model(model: Module, loader: DataLoader,
                   save_evaluation_to: Optional[str] = None,
                   epoch_number: Optional[int] = None,
                   scale: int = 4, is_final: bool = True,
                   kernel_size: int = 11,
                   no_pbar: bool = False,
                   device: Device = 'cpu',
                   rank: int = 0) -> Tuple[float, float]:
    running_left_ssim = running_right_ssim = running_ause = running_aurg = 0
    average_left_ssim = average_right_ssim = average_ause = average_aurg = None
    batch_size = loader.batch_size if loader.batch_size is not None else len(loader)
    description = 'Evaluation'
    tepoch = tqdm.tqdm(loader, description, unit='batch', disable=(no_pbar or rank > 0)) \
        if tqdm is not None else loader
    # alpha one: L1 has zero weight (reference :123-124)
    ssim_loss = WeightedSSIMLoss(alpha=1)
    model.eval()
    for i, image_pair in enumerate(tepoch):
        left = image_pair['left'].to(device)
        right = image_pair['right'].to(device)
        images = torch.cat([left, right], dim=1)
        prediction = model(left, scale)
        disparity, uncertainty = torch.split(prediction, [2, 2], dim=1)
        left_disp, right_disp = torch.split(disparity, [1, 1], dim=1)
        left_recon = u.reconstruct_left_image(left_disp, right)
        right_recon = u.reconstruct_right_image(right_disp, left)
        left_ssim = EF.ssim(left_recon, left, kernel_size=kernel_size, reduction='sum',
                            data_range=1.0)
        right_ssim = EF.ssim(right_recon, right, kernel_size=kernel_size, reduction='sum',
                             data_range=1.0)
        recon = torch.cat((left_recon, right_recon), dim=1)
        # the reference interpolates the error map to (H, W): it already is
        error = ssim_loss.image_error(images, recon)
        oracle_spars = spars.curve(error, error, device=device)
        pred_spars = spars.curve(error, uncertainty, device=device)
        random_spars = spars.random_curve(error, device=device)
        ause = spars.ause(oracle_spars, pred_spars)
        aurg = spars.aurg(pred_spars, random_spars)
        if rank > 0:
            continue
        running_left_ssim += left_ssim.item()
        average_left_ssim = running_left_ssim / ((i + 1) * batch_size)
        running_right_ssim += right_ssim.item()
        average_right_ssim = running_right_ssim / ((i + 1) * batch_size)
        running_ause += ause.item()
        average_ause = running_ause / (i + 1)
        running_aurg += aurg.item()
        average_aurg = running_aurg / (i + 1)
        if tqdm is not None and hasattr(tepoch, 'set_postfix'):
            tepoch.set_postfix(left=average_left_ssim, right=average_right_ssim,
                               ause=average_ause, aurg=average_aurg, scale=scale)
        if save_evaluation_to is not None and i == 0:
            save_comparisons(images[0], disparity[0], uncertainty[0], recon[0], error[0],
                             save_evaluation_to, epoch_number, is_final, device)
    if no_pbar and rank == 0:
        print(f'{description}:'
              f'\n\tleft ssim: {average_left_ssim:.2f}'
              f'\n\tright ssim: {average_right_ssim:.2f}'
              f'\n\tause: {average_ause:.2f}'
              f'\n\taurg: {average_aurg:.2f}'
              f'\n\tdisparity scale: {scale:.2f}')
    average_ssim = (average_left_ssim, average_right_ssim)
    average_spars = (average_ause, average_aurg)
    return average_ssim, average_spars
