"""Loss functions (reference train/loss.py), HIP-backed.

``TukraUncertaintyLoss.forward`` (reference :512-568) runs the fused umamd
loss stack: ONE forward launch over every scale (the six loss terms, reduced
on the device) and ONE backward launch producing d(total)/d(prediction) for
all four channels of every scale, including the WSSIM term's path through
the warp, both L-R consistency terms (with the scatter into the warped
disparity), the edge-aware smoothness and the reprojection-error NLL.

The sub-loss modules keep the reference's names and constructor kwargs so
configs and attribute access (``loss.wssim.previous_image_error``,
``loss.predictive_error.loss_type``...) work; the sub-losses are evaluated
inside the fused kernels, not through their own ``forward``.
"""
from typing import Optional

import torch
import torch.nn as nn
from torch import Tensor
from torch.nn import Module
from torch.nn.parallel import DistributedDataParallel

from umamd import discfn as DF
from umamd import lossfn as LF
from umamd import packer as P

from .utils import ImagePyramid


class _FusedOnly(nn.Module):
    def forward(self, *args, **kwargs):
        raise NotImplementedError(
            f'umamd: {type(self).__name__} is evaluated inside TukraUncertaintyLoss\'s fused '
            f'HIP kernels; a standalone forward is not implemented')


class WeightedSSIMLoss(_FusedOnly):
    """SSIM/L1 photometric error (reference :15-151)."""

    def __init__(self, alpha: float = 0.85, k1: float = 0.01, k2: float = 0.03) -> None:
        super().__init__()
        if k1 != 0.01 or k2 != 0.03:
            raise NotImplementedError('umamd WeightedSSIMLoss: k1/k2 are compiled in (0.01, 0.03)')
        self.alpha = alpha
        self.k1 = k1 ** 2
        self.k2 = k2 ** 2
        self.pool = nn.AvgPool2d(kernel_size=3, stride=1)
        self._previous_image_error = None

    @property
    def previous_image_error(self) -> Tensor:
        """Error map [B,2,h,w] of the last scale evaluated (reference :38-41)."""
        return self._previous_image_error

    def image_error(self, images: Tensor, recon: Tensor) -> Tensor:
        """Per-pixel alpha*DSSIM(upsampled) + (1-alpha)*L1, channel mean per
        view -> [B,2,H,W] (reference :96-131); no gradient (evaluation)."""
        if torch.is_grad_enabled() and (images.requires_grad or recon.requires_grad):
            raise NotImplementedError('umamd WeightedSSIMLoss.image_error has no autograd '
                                      '(training evaluates it inside TukraUncertaintyLoss)')
        return LF.image_error(images, recon, self.alpha)


class ConsistencyLoss(_FusedOnly):
    """L-R consistency (reference :154-188)."""


class SmoothnessLoss(_FusedOnly):
    """Edge-aware smoothness (reference :191-264)."""


def _disc_module(disc: Module) -> Module:
    # discriminator methods are reached through .module under DDP (reference :294-299)
    return disc.module if isinstance(disc, DistributedDataParallel) else disc


class PerceptualLoss(nn.Module):
    """Discriminator feature reconstruction L1 (reference :267-305): sum over
    the discriminator stages of mean |features(image) - features(recon)|,
    on the NHWC feature maps (one fused L1 launch per stage)."""

    def forward(self, image_pyramid: ImagePyramid, recon_pyramid: ImagePyramid,
                disc: Module) -> Tensor:
        d = _disc_module(disc)
        with P.scope(d._packer):
            image_maps = d._features(image_pyramid)
            recon_maps = d._features(recon_pyramid)
        perceptual_loss = 0
        for image_map, recon_map in zip(image_maps, recon_maps):
            perceptual_loss = perceptual_loss + DF.l1_mean(image_map, recon_map)
        return perceptual_loss


class GeneratorLoss(nn.Module):
    """Loss of failing to convince the discriminator (reference :308-337):
    ``self.adversarial`` (MSE or BCE) of the discriminator's predictions on
    the reconstructions against ones."""

    def __init__(self, loss: str = 'mse') -> None:
        super().__init__()
        self.adversarial = nn.MSELoss() if loss == 'mse' else nn.BCELoss()

    def forward(self, recon_pyramid: ImagePyramid, discriminator: Module) -> Tensor:
        predictions = discriminator(recon_pyramid)
        labels = torch.ones_like(predictions)
        return self.adversarial(predictions, labels)


class ReprojectionErrorLoss(_FusedOnly):
    """Uncertainty loss (reference :340-434)."""

    def __init__(self, loss_type: str = 'l1', smoothness_weight: float = 1.0,
                 consistency_weight: float = 1.0, pooling: bool = False) -> None:
        super().__init__()
        if loss_type not in ('l1', 'bayesian', 'log_bayesian'):
            raise ValueError('Loss must be either "l1", "bayesian" or "log_bayesian".')
        if pooling:
            raise NotImplementedError('umamd ReprojectionErrorLoss: pooling=True is not '
                                      'implemented (every reference config uses False)')
        self.loss_type = loss_type
        self.smoothness_weight = smoothness_weight
        self.consistency_weight = consistency_weight
        self.smoothness = SmoothnessLoss() if smoothness_weight > 0 else None
        self.consistency = ConsistencyLoss() if consistency_weight > 0 else None
        self.pool = nn.Identity()


class TukraUncertaintyLoss(nn.Module):
    """Total loss of the uncertainty model (reference :437-568)."""

    def __init__(self, wssim_weight: float = 1.0, consistency_weight: float = 1.0,
                 smoothness_weight: float = 1.0, adversarial_weight: float = 0.85,
                 predictive_error_weight: float = 1.0, perceptual_weight: float = 0.05,
                 wssim_alpha: float = 0.85, perceptual_start: int = 5,
                 adversarial_loss_type: str = 'mse',
                 error_loss_config: Optional[dict] = None) -> None:
        super().__init__()
        self.wssim = WeightedSSIMLoss(wssim_alpha)
        self.consistency = ConsistencyLoss()
        self.smoothness = SmoothnessLoss()
        self.adversarial = GeneratorLoss(adversarial_loss_type)
        self.perceptual = PerceptualLoss()
        self.predictive_error = ReprojectionErrorLoss(**(error_loss_config or {}))
        self.perceptual_start = perceptual_start
        self.wssim_weight = wssim_weight
        self.consistency_weight = consistency_weight
        self.smoothness_weight = smoothness_weight
        self.adversarial_weight = adversarial_weight
        self.perceptual_weight = perceptual_weight
        self.predictive_error_weight = predictive_error_weight
        self.last_terms: Optional[Tensor] = None

    def _cfg(self):
        pe = self.predictive_error
        return {'alpha': float(self.wssim.alpha), 'loss_type': LF.LOSS_TYPES[pe.loss_type],
                'esw': float(pe.smoothness_weight), 'ecw': float(pe.consistency_weight),
                'w_wssim': float(self.wssim_weight), 'w_cons': float(self.consistency_weight),
                'w_smooth': float(self.smoothness_weight),
                'w_err': float(self.predictive_error_weight)}

    def forward(self, image_pyramid: ImagePyramid, predictions: ImagePyramid,
                recon_pyramid: ImagePyramid, epoch: Optional[int] = None,
                discriminator: Optional[Module] = None):
        for p, im, r in zip(predictions, image_pyramid, recon_pyramid):
            tag = getattr(r, '_umamd_recon', None)
            if tag is None or tag != (id(p), id(im)):
                raise ValueError('TukraUncertaintyLoss (umamd): recon_pyramid must be '
                                 'train.utils.reconstruct_pyramid(predictions, image_pyramid) '
                                 '(the fused kernels re-derive that warp and differentiate '
                                 'through it)')
        pending = [r for r in recon_pyramid if getattr(r, '_umamd_pending', False)]
        if pending and len(pending) != len(recon_pyramid):
            raise ValueError('TukraUncertaintyLoss (umamd): partly deferred recon_pyramid')
        disp_loss, error_loss, terms, emap = LF.tukra_loss(
            self._cfg(), list(predictions), list(image_pyramid),
            list(recon_pyramid) if pending else None)
        self.wssim._previous_image_error = emap
        self.last_terms = terms  # [disp, error, wssim, consistency, smoothness, error-term]
        if discriminator is not None:
            # adversarial terms (reference :552-564); the recon pyramid carries
            # the gradient back to the disparities through the warp adjoint
            adversarial_loss = self.adversarial(recon_pyramid, discriminator)
            disp_loss = disp_loss + adversarial_loss * self.adversarial_weight
            if epoch is not None and epoch >= self.perceptual_start:
                perceptual_loss = self.perceptual(image_pyramid, recon_pyramid, discriminator)
                disp_loss = disp_loss + perceptual_loss * self.perceptual_weight
        return disp_loss, error_loss
