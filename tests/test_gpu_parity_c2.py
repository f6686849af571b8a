"""Parity at the benchmarked size and by gradient DIRECTION.

* step goldens (64x128 bayesian / l1, config 1): step-0 gradients of the fp32
  HIP path against the reference's Rademacher sketches (tests/_parity.py);
* BASELINE config 2 at full size (B=8, 256x512, bayesian): the fp32 HIP step
  against the CPU oracle on the same inputs and formula weights --
  disparities of all 4 scales, both loss scalars and every full gradient
  (||g - g_ref|| / ||g_ref||) -- and against the reference's own step 0 and
  10-step loss trajectory (tests/golden/traj_c2.npz, made by importing the
  reference: the BASELINE metric's "loss delta vs ref");
* the drop-in loop: train.train.train_model over a synthetic loader, graph
  replay (one capture per disparity scale, an eager step for the ragged last
  batch) against the same loop stepped eagerly.

Tolerances (stated per check below): fp32 build vs reference 1e-3 rel on
disparities and loss scalars; gradients 2e-2 rel-norm (F9: the
warp-dependent terms alone carry 4e-3 fp32-vs-fp64 noise), 0.1 for the l1
loss (its NLL gradient is sign(sigma - e): the reference's own fp32 vs fp64
differ by up to 5.5e-2 rel-norm on weights, see _l1_tol).
"""
import os

import numpy as np
import pytest
import torch

from _parity import grad_worst, rel_norm, sketch_worst
from conftest import GOLDEN
from test_gpu_model import DEV, _cfg, _model, _z

pytestmark = pytest.mark.gpu


def _l1_tol(k):
    """l1 error loss: its NLL gradient is sign(sigma - e), so every upstream
    gradient inherits sign flips of near-tie pixels.  The reference's own
    math in fp32 vs fp64 (the oracle, same inputs) differs by up to 5.5e-2
    rel-norm on weights at config 1 (decoder.2 disp head) and 0.12 on an SE
    weight (step_l1), so l1 directions are held to about twice that noise;
    the bayesian loss keeps 2e-2."""
    return 0.3 if ('excite' in k or k.endswith('mean_weight')) else 0.12


@pytest.mark.parametrize('name,lt', [('step_bayesian.npz', 'bayesian'), ('step_l1.npz', 'l1'),
                                     ('step_c1_l1.npz', 'l1')])
def test_step0_gradient_directions(name, lt):
    """fp32 HIP step-0 gradients vs the reference's sketches (direction)."""
    import train.utils as u
    from train.loss import TukraUncertaintyLoss
    z = _z(name)
    cfg = _cfg()
    cfg['loss']['error_loss_config']['loss_type'] = lt
    m = _model(cfg).train()
    lf = TukraUncertaintyLoss(**cfg['loss'])
    left = torch.from_numpy(z['left']).to(DEV)
    right = torch.from_numpy(z['right']).to(DEV)
    pyr = u.scale_pyramid(torch.cat([left, right], 1), 4)
    d = m(left, float(z['scale']) if 'scale' in z.files else 0.3)
    dl, el = lf(pyr, d, u.reconstruct_pyramid(d, pyr), 0, None)
    (dl + el).backward()
    grads = {k: p.grad for k, p in m.named_parameters()}
    worst = sketch_worst(grads, z, 2e-2, _l1_tol if lt == 'l1' else None)
    print(f'{name}: worst sketch ratio {worst}')
    assert worst[0] < 1, worst


def _c2_inputs():
    from oracle import step as OS
    z = _z('traj_c2.npz')
    b, h, w = [int(v) for v in z['shape']]
    return z, OS.bench_inputs(b, h, w)


def test_config2_fp32_step_vs_oracle_and_reference():
    """C2 full size: HIP fp32 step 0 vs the oracle (full tensors) and vs the
    reference golden (loss scalars, disparity sums, gradient sketches)."""
    import train.utils as u
    from oracle import model as OM, step as OS
    from train.loss import TukraUncertaintyLoss
    z, (left, right) = _c2_inputs()
    cfg = _cfg()
    cfg['loss']['error_loss_config']['loss_type'] = 'bayesian'
    m = _model(cfg).train()
    lf = TukraUncertaintyLoss(**cfg['loss'])
    lg, rg = left.to(DEV), right.to(DEV)
    pyr = u.scale_pyramid(torch.cat([lg, rg], 1), 4)
    d = m(lg, 0.3)
    dl, el = lf(pyr, d, u.reconstruct_pyramid(d, pyr), 0, None)
    (dl + el).backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu() for k, p in m.named_parameters()}
    disps = [t.detach().cpu() for t in d]
    # the reference's own step 0 (golden)
    assert abs(float(dl) / float(z['disp_loss_0']) - 1) < 1e-3
    assert abs(float(el) / float(z['error_loss_0']) - 1) < 1e-3
    for i in range(4):
        assert abs(float(disps[i].double().sum()) / float(z[f'step0_disp{i}_sum']) - 1) < 1e-4
    ref3 = torch.from_numpy(z['step0_disp3'])
    assert float((disps[3] - ref3).abs().max() / ref3.abs().max()) < 1e-3
    ws = sketch_worst(grads, z, 2e-2)
    print('C2 sketch worst', ws)
    assert ws[0] < 1, ws
    # the oracle on the box's CPU, same inputs and weights: full tensors
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    graphs = OM.load_stage_graphs(cfg['model']['encoder'])
    P = OS.formula_state_dict(OS.param_specs(cfg['model'], graphs))
    out = OS.train_step(P, left, right, 0.3, cfg['model'], cfg['loss'], graphs, {})
    assert abs(float(dl) / out['disp_loss'] - 1) < 1e-3
    assert abs(float(el) / out['error_loss'] - 1) < 1e-3
    for i in range(4):
        r = out['disps'][i]
        assert float((disps[i] - r).abs().max() / r.abs().max()) < 1e-3, i
    gw = grad_worst(grads, out['grads'], 2e-2)
    print('C2 full-gradient worst', gw)
    assert gw[0] < 1, gw
    rels = sorted((rel_norm(grads[k], g), k) for k, g in out['grads'].items()
                  if not k.endswith('mean_weight') and not k.endswith('.bias'))
    print('C2 median weight-gradient rel-norm', rels[len(rels) // 2])


def _trajectory(dtype, steps):
    from oracle import model as OM, step as OS
    from train.graph import CapturedTrainStep
    from train.loss import TukraUncertaintyLoss
    from umamd.optim import Adam
    _, (left, right) = _c2_inputs()
    cfg = _cfg()
    cfg['loss']['error_loss_config']['loss_type'] = 'bayesian'
    m = _model(cfg, dtype).train()
    lf = TukraUncertaintyLoss(**cfg['loss'])
    opt = Adam(m.parameters(), 1e-4)
    cap = CapturedTrainStep(m, lf, opt, left.to(DEV), right.to(DEV), 0.3, warmup=1)
    out = []
    for _ in range(steps):
        dl, el = cap()
        out.append((float(dl), float(el)))
    del OM, OS
    return out


def test_config2_trajectory_vs_reference():
    """The BASELINE metric's loss delta: 10 captured fp32 steps at C2 against
    the reference's own 10-step trajectory.  Step 0: 1e-3.  Later steps: the
    bayesian error loss falls 28.7 -> 9.6 in 10 steps, and Adam's first
    updates are lr * sign(g), so elements whose gradient is at summation-noise
    level move either way: two eager runs of our own path drift 1e-3..4e-3 by
    steps 5-8 (test_gpu_graph), so later steps are held to 2e-2.
    bf16 (the bench's dtype): step 0 within 1e-3 (disparity loss) and 2e-3
    (error loss; DESIGN §2: 1.25e-3 measured), and over the 10 steps within
    1e-2 AND no further from the reference's fp32 trajectory than the
    reference itself under torch.autocast('cpu', bf16) is (traj_c2_bf16.npz:
    3.9e-3 at step 0, 1.6e-2 over 10 steps on the error loss)."""
    z = _z('traj_c2.npz')
    n = sum(1 for k in z.files if k.startswith('disp_loss_'))
    ref = [(float(z[f'disp_loss_{i}']), float(z[f'error_loss_{i}'])) for i in range(n)]
    got = _trajectory('fp32', n)
    rel = [(abs(a[0] / b[0] - 1), abs(a[1] / b[1] - 1)) for a, b in zip(got, ref)]
    print('fp32 trajectory rel deltas', [(round(x, 6), round(y, 6)) for x, y in rel])
    assert rel[0][0] < 1e-3 and rel[0][1] < 1e-3, rel[0]
    assert max(max(r) for r in rel) < 2e-2, rel
    g16 = _trajectory('bf16', n)
    r16 = [(abs(a[0] / b[0] - 1), abs(a[1] / b[1] - 1)) for a, b in zip(g16, ref)]
    zb = _z('traj_c2_bf16.npz')
    refb = [(float(zb[f'disp_loss_{i}']), float(zb[f'error_loss_{i}'])) for i in range(n)]
    rb = [(abs(a[0] / b[0] - 1), abs(a[1] / b[1] - 1)) for a, b in zip(refb, ref)]
    print('bf16 trajectory rel deltas', [(round(x, 6), round(y, 6)) for x, y in r16])
    print('reference bf16-autocast rel deltas', [(round(x, 6), round(y, 6)) for x, y in rb])
    assert r16[0][0] < 1e-3 and r16[0][1] < 2e-3, r16[0]
    for j in range(2):
        worst, worst_ref = max(r[j] for r in r16), max(r[j] for r in rb)
        assert worst < 1e-2 and worst <= worst_ref, (j, worst, worst_ref)


def test_config2_bf16_disparity_vs_reference():
    """The bench's bf16 build at BASELINE config 2 (B=8, 256x512, formula
    weights, the bench's synthetic pair, scale 0.3, train-mode forward):
    every disparity/uncertainty scale within max(BASELINE.md's bar: 3e-2
    max-abs/max-ref, 1e-2 mean relative; 1.1 x the reference's OWN
    bf16-autocast deviation on this input: disp_c2_bf16.npz, 4.1-4.7e-2 /
    1.2-1.6e-2) of the reference's fp32 disparities.  The fp32 side is our
    fp32 build, pinned to the reference in the same test: its coarsest scale
    against the reference's fp32 map (1e-4) and every scale's sum against
    the reference's (1e-4 of the absolute sum); the coarsest bf16 map is also
    compared with the reference's fp32 map directly."""
    from oracle import step as OS
    from test_gpu_model import disp_bf16_bar, disp_stats
    z = _z('disp_c2_bf16.npz')
    bar = disp_bf16_bar(z)
    b, h, w = (int(v) for v in z['shape'])
    left, _ = OS.bench_inputs(b, h, w)
    left = left.to(DEV)
    cfg = _cfg()
    m32 = _model(cfg).train()
    m16 = _model(cfg, 'bf16').train()
    with torch.no_grad():
        d32 = m32(left, 0.3)
        d16 = m16(left, 0.3)
    ref3 = torch.from_numpy(z['fp32_d3']).to(DEV)
    pin = disp_stats(d32[3], ref3)[0]
    assert pin < 1e-4, pin
    for i in range(4):
        s = float(d32[i].double().sum())
        assert abs(s - float(z[f'fp32_sum_{i}'])) <= 1e-4 * float(z[f'fp32_abssum_{i}']), i
    errs = [disp_stats(d16[i], d32[i]) for i in range(4)]
    direct = disp_stats(d16[3], ref3)
    refdev = [(float(z[f'max_rel_{i}']), float(z[f'mean_rel_{i}'])) for i in range(4)]
    print('bf16 vs reference fp32 (max-abs/max-ref, mean rel) per scale:', errs)
    print('coarsest scale vs the reference map directly:', direct)
    print("reference's own bf16 autocast:", refdev)
    for i in range(4):
        assert errs[i][0] <= bar[i][0] and errs[i][1] <= bar[i][1], (i, errs[i], bar[i])
    assert direct[0] <= bar[3][0] and direct[1] <= bar[3][1], (direct, bar[3])


def test_train_model_graph_replay_matches_eager(monkeypatch):
    """The drop-in loop (reference train/train.py:173-267 via our
    train.train.train_model): 2 epochs over a 7-pair loader (batch 2: three
    full batches and a ragged one) with the disparity scale and the learning
    rate changing at epoch 1.  Graph replay (one capture per scale, the
    ragged batch eager) must give the per-epoch losses of the same loop run
    eagerly (UMAMD_TRAIN_GRAPH=0)."""
    from torch.utils.data import DataLoader
    from train import train as T
    from train.loss import TukraUncertaintyLoss
    from test_gpu_model import _uniform_pair
    cfg = _cfg()
    cfg['loss']['error_loss_config']['loss_type'] = 'l1'
    pairs = []
    for i in range(7):
        left, right = _uniform_pair(1, 64, 128, seed=100 + i)
        pairs.append({'left': left[0], 'right': right[0]})
    res, caps = {}, {}
    for mode in ('graph', 'eager'):
        monkeypatch.setenv('UMAMD_TRAIN_GRAPH', '1' if mode == 'graph' else '0')
        torch.manual_seed(0)
        m = _model(cfg).train()
        lf = TukraUncertaintyLoss(**cfg['loss'])
        loader = DataLoader(pairs, batch_size=2, shuffle=False)
        seen = []
        orig = T._GraphSteps.__call__

        def spy(self, left, right, scale, _orig=orig, _seen=seen):
            out = _orig(self, left, right, scale)
            _seen.append((float(scale), tuple(left.shape), out is not None))
            return out
        monkeypatch.setattr(T._GraphSteps, '__call__', spy)
        losses, _ = T.train_model(m, loader, lf, 2, 1e-4,
                                  adjust_learning_rate=lambda o, e, lr: [
                                      g.__setitem__('lr', lr / (1 + e)) for g in o.param_groups],
                                  adjust_disparity=lambda e: (0.3, 0.5)[e],
                                  device=DEV, no_pbar=True)
        monkeypatch.setattr(T._GraphSteps, '__call__', orig)
        res[mode] = losses
        caps[mode] = seen
    print('graph', res['graph'], 'eager', res['eager'])
    # graph mode: full batches replayed (captures at both scales), ragged eager
    replayed = [s for s in caps['graph'] if s[2]]
    assert {s[0] for s in replayed} == {0.3, 0.5} and len(replayed) == 6, caps['graph']
    assert [s for s in caps['graph'] if not s[2]] == [(0.3, (1, 3, 64, 128), False),
                                                      (0.5, (1, 3, 64, 128), False)]
    assert caps['eager'] == []
    for (dg, ug, _), (de, ue, _) in zip(res['graph'], res['eager']):
        assert abs(dg / de - 1) < 5e-3 and abs(ug / ue - 1) < 5e-3, (res['graph'], res['eager'])
    assert np.isfinite(np.array([r[:2] for r in res['graph']])).all()


def test_train_model_vs_reference_loop(monkeypatch):
    """Our train.train.train_model (graph replay for full batches, the
    ragged last batch eager, the capture redone when the scale moves) against
    the REFERENCE's own train_model run on the same loader
    (tests/golden/train_model.npz: reference train/train.py:173-267, 7 pairs
    at 64x128, batch 2, 2 epochs, disparity scale 0.3 -> 0.5, the reference
    adjust_learning_rate, bayesian, fp32, formula weights): per-epoch losses
    per image within max(1e-3, 2x the reference's own fp32 noise on that
    number): the same reference loop in float64 (epoch_*_f64) moves the
    epoch-0 uncertainty loss by 2.0e-3 and epoch 1's by 3.3e-3 (Adam turns
    summation-order noise in near-zero gradient components into update sign
    flips, and the bayesian e/sigma amplifies them)."""
    from torch.utils.data import DataLoader
    from train import train as T
    from train.loss import TukraUncertaintyLoss
    z = np.load(os.path.join(GOLDEN, 'train_model.npz'))
    cfg = _cfg()
    cfg['loss']['error_loss_config']['loss_type'] = 'bayesian'
    left, right = torch.from_numpy(z['left']), torch.from_numpy(z['right'])
    pairs = [{'left': left[i], 'right': right[i]} for i in range(left.shape[0])]
    loader = DataLoader(pairs, batch_size=2, shuffle=False)
    m = _model(cfg).train()
    lf = TukraUncertaintyLoss(**cfg['loss'])
    seen = []
    orig = T._GraphSteps.__call__

    def spy(self, l_, r_, scale):
        out = orig(self, l_, r_, scale)
        seen.append(out is not None)
        return out
    monkeypatch.setattr(T._GraphSteps, '__call__', spy)
    scales = [float(s) for s in z['scales']]
    losses, _ = T.train_model(m, loader, lf, 2, 1e-4, adjust_disparity=lambda e: scales[e],
                              device=DEV, no_pbar=True)
    assert seen.count(True) == 6 and seen.count(False) == 2, seen  # graph path taken
    for e, (d, u_, _) in enumerate(losses):
        for name, got in (('disp', d), ('unc', u_)):
            ref32, ref64 = float(z[f'epoch_{name}'][e]), float(z[f'epoch_{name}_f64'][e])
            noise = abs(ref32 / ref64 - 1)  # the reference's own fp32 deviation
            r = abs(got / ref32 - 1)
            print(f'epoch {e} {name}: ours {got:.6f} ref fp32 {ref32:.6f} ({r:.2e}) '
                  f'ref f64 {ref64:.6f} (ours {abs(got / ref64 - 1):.2e}, ref fp32 {noise:.2e})')
            assert r < max(1e-3, 2 * noise), (e, name, losses, ref32, ref64)
