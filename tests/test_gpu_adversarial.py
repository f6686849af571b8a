"""Adversarial path (BASELINE config 3; reference model/discriminator.py,
train/loss.py:267-337, train/utils.py:248-273, train/train.py:107-152) on
the HIP kernels against reference-generated goldens (make_goldens.py
adversarial: B=2, 64x128, formula weights; the discriminator's Linear is
sized to the 64x128 feature map).  Marked gpu."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, REPO
from test_gpu_model import _cfg, _model, _rel, _pre_bn_bias

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _z():
    return np.load(os.path.join(GOLDEN, 'adversarial.npz'))


def _disc(z, dtype='fp32'):
    import model as M
    from oracle import graph as og, step as OS
    dcfg = json.loads(str(z['disc_cfg']))
    dcfg['load_graph'] = os.path.join(REPO, 'graphs', 'nodes_5_seed_42')
    graphs = [og.load_json(os.path.join(REPO, 'graphs', 'nodes_5_seed_42', f'stage_{s}.json'))
              for s in range(1, len(dcfg['layers']) + 2)]
    d = M.RandomDiscriminator(**dcfg, dtype=dtype)
    d.load_state_dict(OS.formula_state_dict(OS.disc_param_specs(dcfg, graphs)))
    return d.to(DEV).train()


def _pyr(z):
    import train.utils as u
    left = torch.from_numpy(z['left']).to(DEV)
    right = torch.from_numpy(z['right']).to(DEV)
    return left, right, u.scale_pyramid(torch.cat([left, right], 1), 4)


def test_discriminator_forward_and_features():
    z = _z()
    d = _disc(z)
    _, _, pyr = _pyr(z)
    with torch.no_grad():
        prob = d(pyr)
    assert _rel(prob, z['prob_images']) < 1e-3
    d2 = _disc(z)
    with torch.no_grad():
        feats = d2.features(pyr)
    for i, f in enumerate(feats):
        assert abs(float(f.double().sum()) / float(z[f'feat{i}_sum']) - 1) < 1e-3, i
        assert abs(float(f.double().abs().sum()) / float(z[f'feat{i}_abssum']) - 1) < 1e-4, i


def test_generator_perceptual_losses_and_gradients():
    import train.utils as u
    from train.loss import GeneratorLoss, PerceptualLoss
    z = _z()
    d = _disc(z)
    _, _, pyr = _pyr(z)
    preds = [torch.from_numpy(z[f'pred{i}']).to(DEV).requires_grad_(True) for i in range(4)]
    recon = u.reconstruct_pyramid(preds, pyr)
    gen = GeneratorLoss('mse')(recon, d)
    per = PerceptualLoss()(pyr, recon, d)
    assert abs(float(gen) / float(z['generator_loss']) - 1) < 1e-3
    assert abs(float(per) / float(z['perceptual_loss']) - 1) < 1e-3
    g = torch.autograd.grad(gen * 0.85 + per * 0.05, preds)
    for i in range(4):
        ref = torch.from_numpy(z[f'adv_grad{i}']).double()
        err = float((g[i].double().cpu() - ref).norm() / ref.norm())
        assert err < 2e-2, (i, err)  # warp cell flips through a deep network


def test_run_discriminator_loss_and_gradients():
    import train.utils as u
    z = _z()
    d = _disc(z)
    _, _, pyr = _pyr(z)
    preds = [torch.from_numpy(z[f'pred{i}']).to(DEV) for i in range(4)]
    recon = u.reconstruct_pyramid(preds, pyr)
    dl = u.run_discriminator(pyr, recon, d, torch.nn.BCELoss(), 2)
    dl.backward()
    assert abs(float(dl) / float(z['disc_loss']) - 1) < 1e-3
    bad = []
    for k, p in d.named_parameters():
        if _pre_bn_bias(k.replace('layers.', 'encoder.layers.', 1)) or \
                (k.endswith('.bias') and 'convolution.layers.0.' in k) or k.endswith('keys.bias'):
            continue
        ref, got = float(z[f'disc_gradnorm/{k}']), float(p.grad.double().norm())
        if abs(got - ref) > 2e-2 * ref + 1e-6:
            bad.append((k, got, ref))
    assert not bad, bad[:8]


def test_adversarial_train_steps():
    """Two steps of the reference's adversarial loop body (model step with
    the discriminator clone's generator + perceptual terms, then the
    discriminator step), batch index 0 and 1 with perceptual_start 1."""
    from copy import deepcopy
    from train.loss import TukraUncertaintyLoss
    from train.train import train_step
    from umamd.optim import Adam
    z = _z()
    cfg = _cfg()
    cfg['loss']['error_loss_config']['loss_type'] = 'bayesian'
    cfg['loss']['perceptual_start'] = 1
    m = _model(cfg).train()
    d = _disc(z)
    clone = deepcopy(d)
    lf = TukraUncertaintyLoss(**cfg['loss'])
    opt, dopt = Adam(m.parameters(), 1e-4), Adam(d.parameters(), 1e-4)
    left, right, _ = _pyr(z)
    for i in range(2):
        dl, el, dsl = train_step(m, left, right, lf, opt, 0.3, 4, i, d, clone, dopt,
                                 torch.nn.BCELoss())
        if i % 10 == 0:
            clone.load_state_dict(d.state_dict())
        got = [float(dl), float(el), float(dsl)]
        ref = [float(z[f'step_disp_{i}']), float(z[f'step_err_{i}']), float(z[f'step_disc_{i}'])]
        rel = [abs(a / b - 1) for a, b in zip(got, ref)]
        print(f'adversarial step {i}: got {got} ref {ref} rel {rel}')
        # step 0: same weights in.  Step 1 follows one Adam step, lr*sign(g):
        # gradient elements within noise of zero (the adversarial gradient
        # reaches the disparities through the warp) flip their
        # update, and the bayesian NLL at small sigma (error loss ~1.6e3 here)
        # amplifies that: 3e-2 on the error loss, 5e-3 on the others
        if i == 0:
            assert all(r < 1e-3 for r in rel), (i, got, ref)
            # the updates themselves: Adam's first step is lr*sign(g), so a
            # gradient element within summation noise of zero moves +-lr
            # either way -- allow two such flips (2 * 2lr) per tensor
            for pre, mod in (('model', m), ('disc', d)):
                for k, v in mod.state_dict().items():
                    key = f'{pre}_sum/{k}'
                    if key not in z.files or _pre_bn_bias(k) or (
                            pre == 'disc' and (k.endswith('keys.bias') or (
                                k.endswith('.bias') and 'convolution.layers.0.' in k))):
                        continue
                    tol = 1e-4 * float(z[f'{pre}_abs/{k}']) + 2 * 2 * 1e-4
                    assert abs(float(v.double().sum()) - float(z[key])) <= tol, key
        else:
            # one Adam step later the reference's own error loss jumped from
            # 14 to 1.6e3 (bayesian NLL at collapsing sigma): the step is
            # ill-conditioned, and the sign flips above move it by percents;
            # only agreement to within 10 % is meaningful here
            assert all(r < 0.1 for r in rel), (i, got, ref)


def test_adversarial_bf16_runs():
    """bf16 discriminator + model step: finite losses and gradients."""
    from copy import deepcopy
    from train.loss import TukraUncertaintyLoss
    from train.train import train_step
    from umamd.optim import Adam
    z = _z()
    cfg = _cfg()
    m = _model(cfg, 'bf16').train()
    d = _disc(z, 'bf16')
    lf = TukraUncertaintyLoss(**cfg['loss'])
    left, right, _ = _pyr(z)
    dl, el, dsl = train_step(m, left, right, lf, Adam(m.parameters(), 1e-4), 0.3, 4, 5, d,
                             deepcopy(d), Adam(d.parameters(), 1e-4), torch.nn.BCELoss())
    torch.cuda.synchronize()
    assert all(torch.isfinite(t) for t in (dl, el, dsl))
    for k, p in d.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), k


def test_adversarial_config3_full_size():
    """BASELINE config 3 shape (config 2 + discriminator: B=8, 256x512,
    bayesian, bf16, config.yml's discriminator with its 32768-feature head):
    one adversarial step past perceptual_start -- finite losses and gradients
    on both networks, and the bf16 disparity/error losses within the bf16 bar
     of an fp32 step from the same weights."""
    from copy import deepcopy
    import model as M
    from test_gpu_model import _uniform_pair
    from train.loss import TukraUncertaintyLoss
    from train.train import train_step
    from umamd.optim import Adam
    cfg = _cfg()
    dcfg = dict(cfg['discriminator'])
    dcfg['load_graph'] = os.path.join(REPO, dcfg['load_graph'])
    left, right = _uniform_pair(8, 256, 512, seed=7)
    left, right = left.to(DEV), right.to(DEV)
    torch.manual_seed(0)
    d16 = M.RandomDiscriminator(**dcfg, dtype='bf16').to(DEV).train()
    d32 = M.RandomDiscriminator(**dcfg, dtype='fp32').to(DEV).train()
    d32.load_state_dict(d16.state_dict())
    m16 = _model(cfg, 'bf16').train()
    m32 = _model(cfg, 'fp32').train()
    res = []
    for m, d in ((m16, d16), (m32, d32)):
        lf = TukraUncertaintyLoss(**cfg['loss'])
        dl, el, dsl = train_step(m, left, right, lf, Adam(m.parameters(), 1e-4), 0.3, 4, 5, d,
                                 deepcopy(d), Adam(d.parameters(), 1e-4), torch.nn.BCELoss())
        torch.cuda.synchronize()
        assert all(torch.isfinite(t) for t in (dl, el, dsl))
        for net in (m, d):
            for k, p in net.named_parameters():
                assert p.grad is not None and torch.isfinite(p.grad).all(), k
        res.append((float(dl), float(el), float(dsl)))
    (a16, e16, _), (a32, e32, _) = res
    assert abs(a16 / a32 - 1) < 2e-2 and abs(e16 / e32 - 1) < 3e-2, res
