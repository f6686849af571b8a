"""Functional CPU restatement of the reference loss stack -- TEST ORACLE.

Reference anchors (train/utils.py, train/loss.py):
  l1_loss                 utils.py:22-24
  scale_pyramid           utils.py:27-50
  reconstruct (+L/R)      utils.py:65-109 (F6: not identity at d=0)
  reconstruct_pyramid     utils.py:112-135
  WeightedSSIM            loss.py:15-151
  Consistency             loss.py:154-188
  Smoothness              loss.py:191-264
  ReprojectionError       loss.py:340-434 (F5 argument order)
  Tukra total             loss.py:512-568
"""
from __future__ import annotations

from typing import Dict, List

import torch
import torch.nn.functional as F


def l1_loss(x, y):
    return (x - y).abs().mean()


def scale_pyramid(x, scales):
    h, w = x.shape[-2:]
    return [F.interpolate(x, size=(h // 2 ** i, w // 2 ** i), mode='bilinear',
                          align_corners=True) for i in range(scales)]


def reconstruct(disparity, opposite):
    """grid_sample warp with the reference's linspace(0,1) base grid
    (utils.py:77-97): sample x = j*W/(W-1) - 0.5 + d*W, y = i*H/(H-1) - 0.5."""
    b, _, h, w = opposite.shape
    xb = torch.linspace(0, 1, w).repeat(b, h, 1).type_as(opposite)
    yb = torch.linspace(0, 1, h).repeat(b, w, 1).transpose(1, 2).type_as(opposite)
    flow = torch.stack((xb + disparity.squeeze(1), yb), dim=3) * 2 - 1
    return F.grid_sample(opposite, flow, mode='bilinear', padding_mode='zeros',
                         align_corners=False)


def reconstruct_left(dl, right):
    return reconstruct(-dl, right)


def reconstruct_right(dr, left):
    return reconstruct(dr, left)


def reconstruct_pyramid(disps, pyramid):
    out = []
    for d, im in zip(disps, pyramid):
        out.append(torch.cat([reconstruct_left(d[:, 0:1], im[:, 3:6]),
                              reconstruct_right(d[:, 1:2], im[:, 0:3])], 1))
    return out


# ------------------------------------------------------------------ terms --
def _pool(x):
    return F.avg_pool2d(x, 3, 1)


def dssim(x, y, c1=0.01 ** 2, c2=0.03 ** 2):
    mx, my = _pool(x), _pool(y)
    sx = _pool(x * x) - mx * mx
    sy = _pool(y * y) - my * my
    sxy = _pool(x * y) - mx * my
    ssim = ((2 * mx * my + c1) * (2 * sxy + c2)) / ((mx * mx + my * my + c1) * (sx + sy + c2))
    return torch.clamp((1 - ssim) / 2, 0, 1)


def image_error(images, recon, alpha=0.85):
    """Per-pixel weighted SSIM/L1 error, 2 channels (loss.py:96-131)."""
    h, w = images.shape[-2:]
    l1 = (images - recon).abs()
    ss = torch.cat((dssim(images[:, 0:3], recon[:, 0:3]),
                    dssim(images[:, 3:6], recon[:, 3:6])), 1)
    ss = F.interpolate(ss, size=(h, w), mode='bilinear', align_corners=True)
    tot = alpha * ss + (1 - alpha) * l1
    return torch.cat((tot[:, 0:3].mean(1, keepdim=True), tot[:, 3:6].mean(1, keepdim=True)), 1)


def wssim_loss(images, recon, alpha=0.85):
    e = image_error(images, recon, alpha)
    return (e[:, 0:1] + e[:, 1:2]).mean(), e


def consistency_loss(disp, images=None):
    """F5: the first argument is both the compared map and the shift."""
    images = disp if images is None else images
    ld, rd = disp[:, 0:1], disp[:, 1:2]
    li, ri = images[:, 0:1], images[:, 1:2]
    return l1_loss(ld, reconstruct_left(ld, ri)) + l1_loss(rd, reconstruct_right(rd, li))


def _grad_x(x):
    x = F.pad(x, (0, 1, 0, 0), mode='replicate')
    return x[:, :, :, :-1] - x[:, :, :, 1:]


def _grad_y(x):
    x = F.pad(x, (0, 0, 0, 1), mode='replicate')
    return x[:, :, :-1, :] - x[:, :, 1:, :]


def _smooth_err(d, im):
    wx = torch.exp(-_grad_x(im).abs().mean(1, keepdim=True))
    wy = torch.exp(-_grad_y(im).abs().mean(1, keepdim=True))
    return (_grad_x(d) * wx).abs() + (_grad_y(d) * wy).abs()


def smoothness_loss(disp, images):
    return (_smooth_err(disp[:, 0:1], images[:, 0:3]) +
            _smooth_err(disp[:, 1:2], images[:, 3:6])).mean()


def error_loss(pred, images, err, loss_type='l1', smoothness_weight=0.0,
               consistency_weight=0.5, pooling=False):
    """ReprojectionErrorLoss.forward (loss.py:405-434)."""
    err = err.detach().clone()
    if pooling:
        pred, images, err = _pool(pred), _pool(images), _pool(err)
    disp, unc = pred[:, 0:2], pred[:, 2:4]
    if loss_type == 'bayesian':
        loss = (err / unc + torch.log(unc)).mean()
    elif loss_type == 'log_bayesian':
        loss = (err / torch.exp(-unc) + unc).mean() / 2
    elif loss_type == 'l1':
        loss = l1_loss(unc, err)
    else:
        raise ValueError(loss_type)
    if smoothness_weight > 0:
        loss = loss + smoothness_loss(unc, images) * smoothness_weight
    if consistency_weight > 0:
        loss = loss + consistency_loss(unc, disp) * consistency_weight
    return loss


def total_loss(pyramid, preds, recon, cfg: Dict) -> tuple:
    """TukraUncertaintyLoss.forward without a discriminator (loss.py:512-568).
    Returns (disp_loss, error_loss, terms) where terms holds the per-term sums."""
    alpha = cfg.get('wssim_alpha', 0.85)
    ecfg = dict(cfg.get('error_loss_config') or {})
    terms = {'wssim': 0., 'consistency': 0., 'smoothness': 0., 'error': 0.}
    for i, (im, p, rc) in enumerate(zip(pyramid, preds, recon)):
        disp = p[:, 0:2]
        w, e = wssim_loss(im, rc, alpha)
        terms['wssim'] = terms['wssim'] + w
        terms['consistency'] = terms['consistency'] + consistency_loss(disp)
        terms['smoothness'] = terms['smoothness'] + smoothness_loss(disp, im) / 2 ** i
        terms['error'] = terms['error'] + error_loss(p, im, e, **ecfg)
    disp_loss = terms['wssim'] * cfg.get('wssim_weight', 1.0) \
        + terms['consistency'] * cfg.get('consistency_weight', 1.0) \
        + terms['smoothness'] * cfg.get('smoothness_weight', 1.0)
    err_loss = terms['error'] * cfg.get('predictive_error_weight', 1.0)
    return disp_loss, err_loss, terms


def adjust_disparity(epoch, m=0.02, c=0.0, step=0.2, offset=0.1, min_scale=0.3,
                     max_scale=1.0):
    """utils.py:143-174."""
    s = (epoch + 1) * m + c
    s = round((s + offset) / step) * step - offset
    return float(min(max(s, min_scale), max_scale))


def adjust_learning_rate_value(epoch, lr, finetune=False):
    """utils.py:333-353 (returns the value instead of mutating groups)."""
    if epoch > 40 or finetune:
        return lr / 4
    if epoch > 30:
        return lr / 2
    return lr
