"""Evaluation path on the GPU (reference train/evaluate.py, train/
sparsification.py): the gaussian SSIM against the oracle's torchmetrics
restatement (parity unpinned: torchmetrics is absent), the sparsification
curves against the reference-generated golden, and evaluate_model end to end.
Marked gpu."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import evaluate as OE

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def test_sparsification_curve_matches_reference():
    import train.sparsification as S
    z = np.load(os.path.join(GOLDEN, 'sparsification.npz'))
    err = torch.from_numpy(z['err']).to(DEV)
    unc = torch.from_numpy(z['unc']).to(DEV)
    oc = S.curve(err, err, device=DEV)
    pc = S.curve(err, unc, device=DEV)
    assert torch.allclose(oc.cpu(), torch.from_numpy(z['oracle_curve']), rtol=1e-5, atol=1e-6)
    assert torch.allclose(pc.cpu(), torch.from_numpy(z['pred_curve']), rtol=1e-5, atol=1e-6)
    assert abs(float(S.ause(oc, pc)) - float(z['ause'])) < 1e-5
    rc = S.random_curve(err, device=DEV)  # random: statistical only
    assert torch.isfinite(rc).all() and abs(float(rc[0]) - 1.0) < 1e-5


@pytest.mark.parametrize('shape', [(2, 3, 64, 128), (1, 3, 37, 90)])
def test_gaussian_ssim(shape):
    from umamd import evalfn as EF
    g = torch.Generator().manual_seed(1)
    x = torch.rand(shape, generator=g)
    y = (x + 0.2 * torch.randn(shape, generator=g)).clamp(0, 1)
    got = EF.ssim(y.to(DEV), x.to(DEV), reduction='none')
    ref = OE.ssim_gauss(y.double(), x.double(), reduction='none')
    assert float((got.double().cpu() - ref).abs().max()) < 1e-5
    s = EF.ssim(x.to(DEV), x.to(DEV), reduction='sum')
    assert abs(float(s) - shape[0]) < 1e-5  # identical images: SSIM 1


def test_evaluate_model_end_to_end(tmp_path):
    """evaluate_model over a 2-batch loader of synthetic pairs at 64x128:
    SSIMs and AUSE against an oracle evaluation of the same predictions."""
    import yaml
    import model as M
    import train.utils as u
    from oracle import loss as OL, model as OM, step as OS
    from train.evaluate import evaluate_model
    repo = os.path.dirname(GOLDEN.rstrip('/').rsplit('/', 1)[0])
    with open(os.path.join(repo, 'config.yml')) as f:
        cfg = yaml.safe_load(f)
    cfg['model']['encoder']['load_graph'] = os.path.join(repo, 'graphs/nodes_5_seed_42')
    graphs = OM.load_stage_graphs(cfg['model']['encoder'])
    sd = OS.formula_state_dict(OS.param_specs(cfg['model'], graphs))
    m = M.RandomlyConnectedModel(**cfg['model']).to(DEV)
    m.load_state_dict(sd)
    g = torch.Generator().manual_seed(3)
    data = [{'left': torch.rand(2, 3, 64, 128, generator=g),
             'right': torch.rand(2, 3, 64, 128, generator=g)} for _ in range(2)]

    class Loader(list):
        batch_size = 2
    (ls, rs), (au, ag) = evaluate_model(m, Loader(data), str(tmp_path), epoch_number=1, scale=0.3,
                                        no_pbar=True, device=DEV)
    assert os.path.exists(tmp_path / 'final' / 'prediction.png')
    # oracle evaluation of the same model/inputs (deterministic parts)
    P = {k: v.clone() for k, v in sd.items()}
    left_s = right_s = ause_s = 0.0
    for b in data:
        left, right = b['left'], b['right']
        with torch.no_grad():
            pred = OM.model_forward(left, P, cfg['model'], graphs, 0.3, training=False)
        dl, dr = pred[:, 0:1], pred[:, 1:2]
        lrec, rrec = OL.reconstruct_left(dl, right), OL.reconstruct_right(dr, left)
        left_s += float(OE.ssim_gauss(lrec, left))
        right_s += float(OE.ssim_gauss(rrec, right))
        err = OL.image_error(torch.cat([left, right], 1), torch.cat([lrec, rrec], 1), 1.0)
        ause_s += float(OE.ause(OE.curve(err, err), OE.curve(err, pred[:, 2:4])))
    assert abs(ls - left_s / 4) < 1e-3 and abs(rs - right_s / 4) < 1e-3, (ls, left_s / 4)
    assert abs(au - ause_s / 2) < 2e-3, (au, ause_s / 2)
    assert np.isfinite(ag)
