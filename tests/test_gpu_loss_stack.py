"""Loss-stack launches beyond the reference goldens (test_gpu_model.py holds
the golden checks): the deferred reconstruction written by the fused loss
forward, the reconstruct / reconstruct_pyramid adjoint w.r.t. the disparity
(adversarial path), WeightedSSIMLoss.image_error, and the fused kernels at
sizes whose tiles do not divide the image (ragged edges) against the CPU
oracle.  Marked gpu."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import loss as OL

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _cfg(lt='bayesian'):
    return {'wssim_weight': 1.0, 'consistency_weight': 1.0, 'smoothness_weight': 1.0,
            'adversarial_weight': 0.85, 'perceptual_weight': 0.05, 'predictive_error_weight': 1.0,
            'wssim_alpha': 0.85, 'perceptual_start': 5, 'adversarial_loss_type': 'mse',
            'error_loss_config': {'loss_type': lt, 'smoothness_weight': 0.3,
                                  'consistency_weight': 0.5, 'pooling': False}}


def _inputs(N, H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    imgs = torch.rand(N, 6, H, W, generator=g)
    preds = [(0.02 + 0.2 * torch.rand(N, 4, H >> i, W >> i, generator=g)) for i in range(4)]
    return imgs, preds


@pytest.mark.parametrize('shape', [(2, 64, 128), (1, 40, 72), (3, 24, 104)])
def test_deferred_recon_and_ragged_tiles(shape):
    """The fused loss at sizes that leave partial forward/backward tiles and
    partial scatter strips; deferred recon == eager recon == oracle."""
    import train.utils as u
    from train.loss import TukraUncertaintyLoss
    from umamd import lossfn as LF
    N, H, W = shape
    imgs, preds = _inputs(N, H, W)
    cfg = _cfg()
    lf = TukraUncertaintyLoss(**cfg)
    pyr = u.scale_pyramid(imgs.to(DEV), 4)
    pd = [p.to(DEV).requires_grad_(True) for p in preds]
    eager = [r.clone() for r in u.reconstruct_pyramid(pd, pyr)]
    with LF.deferred_recon():
        rec = u.reconstruct_pyramid(pd, pyr)
    dl, el = lf(pyr, pd, rec, 0, None)
    for a, b in zip(rec, eager):
        assert _rel(a, b) < 1e-6
    # oracle (fp64 CPU)
    pyr_c = OL.scale_pyramid(imgs.double(), 4)
    pc = [p.double().requires_grad_(True) for p in preds]
    rc = OL.reconstruct_pyramid(pc, pyr_c)
    for a, b in zip(rec, rc):
        assert _rel(a, b) < 1e-5
    ocfg = dict(cfg)
    dlc, elc, _ = OL.total_loss(pyr_c, pc, rc, ocfg)
    assert abs(float(dl) / float(dlc) - 1) < 1e-4
    assert abs(float(el) / float(elc) - 1) < 1e-4
    (dl + 0.5 * el).backward()
    (dlc + 0.5 * elc).backward()
    for i in range(4):
        ref = pc[i].grad
        err = float((pd[i].grad.double().cpu() - ref).norm() / ref.norm())
        assert err < 4e-3, (i, err)  # warp cell flips


def test_reconstruct_adjoint_matches_grid_sample():
    """reconstruct() and reconstruct_pyramid() backward (the adversarial
    terms' path into the disparities) vs torch autograd of the oracle warp."""
    import train.utils as u
    imgs, preds = _inputs(2, 32, 64, seed=3)
    pd = [p.to(DEV).requires_grad_(True) for p in preds]
    pyr = u.scale_pyramid(imgs.to(DEV), 4)
    rec = u.reconstruct_pyramid(pd, pyr)
    gs = [torch.randn(r.shape) for r in rec]
    sum((r * g.to(DEV)).sum() for r, g in zip(rec, gs)).backward()
    pc = [p.double().requires_grad_(True) for p in preds]
    rc = OL.reconstruct_pyramid(pc, OL.scale_pyramid(imgs.double(), 4))
    sum((r * g.double()).sum() for r, g in zip(rc, gs)).backward()
    for i in range(4):
        assert _rel(pd[i].grad[:, :2], pc[i].grad[:, :2]) < 1e-3
        assert float(pd[i].grad[:, 2:].abs().max()) == 0.0
    # the single-view warp
    d = pd[0][:, :1].detach().clone().requires_grad_(True)
    im = pyr[0][:, 3:6]
    out = u.reconstruct_left_image(d, im)
    g = torch.randn(out.shape)
    (out * g.to(DEV)).sum().backward()
    dc = d.detach().double().cpu().requires_grad_(True)
    oc = OL.reconstruct_left(dc, im.double().cpu())
    (oc * g.double()).sum().backward()
    assert _rel(d.grad, dc.grad) < 1e-3


@pytest.mark.parametrize('alpha', [0.85, 1.0])
def test_image_error(alpha):
    from train.loss import WeightedSSIMLoss
    g = torch.Generator().manual_seed(5)
    imgs = torch.rand(2, 6, 40, 72, generator=g)
    rec = (imgs + 0.1 * torch.randn(imgs.shape, generator=g)).clamp(0, 1)
    got = WeightedSSIMLoss(alpha).image_error(imgs.to(DEV), rec.to(DEV))
    ref = OL.image_error(imgs.double(), rec.double(), alpha)
    assert _rel(got, ref) < 1e-5


def test_loss_full_size_properties():
    """BASELINE config-2 loss shape (B=8, 256x512): finite terms, the
    deferred recon equals the eager one, gradients finite and linear in the
    upstream gradient."""
    import train.utils as u
    from train.loss import TukraUncertaintyLoss
    from umamd import lossfn as LF
    imgs, preds = _inputs(8, 256, 512, seed=7)
    lf = TukraUncertaintyLoss(**_cfg())
    pyr = u.scale_pyramid(imgs.to(DEV), 4)
    pd = [p.to(DEV).requires_grad_(True) for p in preds]
    with LF.deferred_recon():
        rec = u.reconstruct_pyramid(pd, pyr)
    dl, el = lf(pyr, pd, rec, 0, None)
    eager = u.reconstruct_pyramid(pd, pyr)
    for a, b in zip(rec, eager):
        assert _rel(a, b) < 1e-6
    assert torch.isfinite(lf.last_terms).all()
    g1 = torch.autograd.grad(dl + el, pd, retain_graph=True)
    g2 = torch.autograd.grad(2.0 * dl + 2.0 * el, pd)
    for a, b in zip(g1, g2):
        assert torch.isfinite(a).all()
        assert _rel(2.0 * a, b) < 1e-6


def _smooth_preds(N, H, W, seed, noisy_right=False):
    """disparities that vary by well under a pixel of shift between
    neighbours (the row-owned scatter's increasing-tap path); with
    noisy_right the right half of every row is per-pixel noise (the atomic
    fallback path) in the same launch"""
    g = torch.Generator().manual_seed(seed)
    out = []
    for i in range(4):
        h, w = H >> i, W >> i
        yy = torch.linspace(0, 1, h).view(1, 1, h, 1)
        xx = torch.linspace(0, 1, w).view(1, 1, 1, w)
        base = 0.05 + 0.1 * torch.rand(N, 4, 1, 1, generator=g)
        p = base + 0.02 * torch.sin(6.0 * xx + 3.0 * yy + torch.rand(N, 4, 1, 1, generator=g))
        if noisy_right:
            p = p.expand(N, 4, h, w).clone()
            p[..., w // 2:] = 0.02 + 0.2 * torch.rand(N, 4, h, w - w // 2, generator=g)
        out.append(p.expand(N, 4, h, w).contiguous())
    return out


def _loss_grads(imgs, preds, cfg):
    import train.utils as u
    from train.loss import TukraUncertaintyLoss
    from umamd import lossfn as LF
    lf = TukraUncertaintyLoss(**cfg)
    pyr = u.scale_pyramid(imgs.to(DEV), 4)
    pd = [p.to(DEV).requires_grad_(True) for p in preds]
    with LF.deferred_recon():
        rec = u.reconstruct_pyramid(pd, pyr)
    dl, el = lf(pyr, pd, rec, 0, None)
    (dl + 0.5 * el).backward()
    return dl, el, [p.grad.detach().clone() for p in pd]


@pytest.mark.parametrize('shape', [(2, 64, 128), (1, 40, 72), (2, 32, 200)])
@pytest.mark.parametrize('noisy_right', [False, True])
def test_row_scatter_vs_oracle(shape, noisy_right):
    """loss backward (the strip-owned consistency scatter completing the
    fused forward's gradient partials) against the f64 oracle, smooth and
    per-pixel-noise disparities, ragged widths (72, 200: partial tiles)"""
    N, H, W = shape
    g = torch.Generator().manual_seed(11)
    imgs = torch.rand(N, 6, H, W, generator=g)
    preds = _smooth_preds(N, H, W, 12, noisy_right)
    cfg = _cfg()
    dl, el, gr = _loss_grads(imgs, preds, cfg)
    pyr_c = OL.scale_pyramid(imgs.double(), 4)
    pc = [p.double().requires_grad_(True) for p in preds]
    rc = OL.reconstruct_pyramid(pc, pyr_c)
    dlc, elc, _ = OL.total_loss(pyr_c, pc, rc, dict(cfg))
    assert abs(float(dl) / float(dlc) - 1) < 1e-4
    assert abs(float(el) / float(elc) - 1) < 1e-4
    (dlc + 0.5 * elc).backward()
    for i in range(4):
        ref = pc[i].grad
        err = float((gr[i].double().cpu() - ref).norm() / ref.norm())
        assert err < 4e-3, (i, err)  # warp cell flips


@pytest.mark.parametrize('noisy_right', [False, True])
@pytest.mark.parametrize('loss_type', ['l1', 'bayesian', 'log_bayesian'])
def test_fused_loss_matches_two_pass_full_size(noisy_right, loss_type):
    """BASELINE config-2 shape: the fused forward (loss terms + gradient
    partials in one tile pass, um_loss_fwd gpart) and its one-launch backward
    against the plain forward kernel and the two-launch backward (a second
    backward through the same graph has no partials left): the same values
    up to the summation order"""
    import train.utils as u
    from train.loss import TukraUncertaintyLoss
    from umamd import lossfn as LF
    g = torch.Generator().manual_seed(21)
    imgs = torch.rand(8, 6, 256, 512, generator=g)
    preds = _smooth_preds(8, 256, 512, 22, noisy_right)
    lf = TukraUncertaintyLoss(**_cfg(loss_type))
    pyr = u.scale_pyramid(imgs.to(DEV), 4)
    pd = [p.to(DEV).requires_grad_(True) for p in preds]
    with LF.deferred_recon():
        rec = u.reconstruct_pyramid(pd, pyr)
    dl, el = lf(pyr, pd, rec, 0, None)
    terms = lf.last_terms.clone()
    eager = u.reconstruct_pyramid(pd, pyr)
    for a, b in zip(rec, eager):
        assert _rel(a, b) < 1e-6
    g_fused = torch.autograd.grad(dl + 0.5 * el, pd, retain_graph=True)
    g_plain = torch.autograd.grad(dl + 0.5 * el, pd)
    with torch.no_grad():
        pdd = [p.detach() for p in pd]
        dl0, el0 = lf(pyr, pdd, u.reconstruct_pyramid(pdd, pyr), 0, None)
    assert abs(float(dl) / float(dl0) - 1) < 1e-6
    assert abs(float(el) / float(el0) - 1) < 1e-6
    assert _rel(terms, lf.last_terms) < 1e-6
    for a, b in zip(g_fused, g_plain):
        assert torch.isfinite(a).all()
        assert _rel(a, b) < 1e-5
