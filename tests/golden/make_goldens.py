#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE.

Run in the build container only (needs /root/reference, read-only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py

The reference is imported from /root/reference with a minimal harness
(SURVEY.md 8(c)): stub modules for the absent torchvision/torchmetrics (not on
the loss-math path), and ``model.graph.load_graph`` replaced by a reader of our
JSON adjacency files (pinned equal to the reference gpickles by
tests/test_graph.py) -- nothing from the reference is unpickled.  Weights come
from ``oracle.step.formula_state_dict`` (a deterministic function of the
parameter name and element index) and are loaded with ``load_state_dict``.

Outputs are small .npz files (data only: inputs and expected outputs).  The
oracle is checked against them by tests/test_oracle_goldens.py, and the HIP
build by the GPU parity tests.
"""
from __future__ import annotations

import json
import os
import sys
import types

os.environ['PYTHONDONTWRITEBYTECODE'] = '1'
sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402
import yaml  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'


# ------------------------------------------------------------------ harness --
def _install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    ident = lambda *a, **k: (lambda x: x)  # noqa: E731
    tv = mod('torchvision')
    tv.utils = mod('torchvision.utils', make_grid=lambda *a, **k: None,
                   save_image=lambda *a, **k: None)
    tv.transforms = mod('torchvision.transforms', Resize=ident, ToTensor=ident,
                        RandomHorizontalFlip=ident, Compose=ident)
    tv.transforms.functional = mod('torchvision.transforms.functional')
    tm = mod('torchmetrics')
    tm.functional = mod('torchmetrics.functional',
                        structural_similarity_index_measure=lambda *a, **k: None)


class _Adj:
    def __init__(self, adj):
        self.adj = adj

    def number_of_nodes(self):
        return len(self.adj)

    def neighbors(self, i):
        return iter(self.adj[i])


def _json_graph_loader(path):
    # path = <dir>/stage_{s}.gpickle  ->  repo graphs/<dirname>/stage_{s}.json
    d = os.path.basename(os.path.dirname(path))
    f = os.path.basename(path).replace('.gpickle', '.json')
    with open(os.path.join(REPO, 'graphs', d, f)) as fh:
        return _Adj(json.load(fh)['adj'])


def import_reference():
    _install_stubs()
    sys.path.insert(0, REF)
    import model as ref_model  # noqa: E402
    import model.graph as ref_graph  # noqa: E402
    ref_graph.load_graph = _json_graph_loader
    import train.loss as ref_loss  # noqa: E402
    import train.utils as ref_utils  # noqa: E402
    return ref_model, ref_loss, ref_utils


# ------------------------------------------------------------------- inputs --
def smooth_texture(b, c, h, w, seed=1234, sigma=2.0):
    """Gaussian-blurred U[0,1) noise, renormalised to [0.05, 0.95]."""
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(b, c, h, w, generator=g)
    r = int(3 * sigma)
    t = torch.arange(-r, r + 1, dtype=torch.float32)
    k = torch.exp(-t * t / (2 * sigma * sigma))
    k = k / k.sum()
    x = torch.nn.functional.conv2d(x.reshape(b * c, 1, h, w), k.view(1, 1, 1, -1),
                                   padding=(0, r))
    x = torch.nn.functional.conv2d(x, k.view(1, 1, -1, 1), padding=(r, 0))
    x = x.reshape(b, c, h, w)
    lo = x.amin(dim=(2, 3), keepdim=True)
    hi = x.amax(dim=(2, 3), keepdim=True)
    return 0.05 + 0.9 * (x - lo) / (hi - lo)


def stereo_pair(b, h, w, seed=1234):
    left = smooth_texture(b, 3, h, w, seed)
    g = torch.Generator().manual_seed(seed + 1)
    dfield = smooth_texture(b, 1, h, w, seed + 2, sigma=6.0) * 0.1  # 0..0.1 * W
    del g
    sys.path.insert(0, REPO)
    from oracle import loss as OL  # noqa: E402
    right = OL.reconstruct(dfield, left)  # right sees left shifted by d
    return left.contiguous(), right.contiguous(), dfield


def pred_pyramid(b, h, w, seed, scale=0.3):
    """4-level 4-channel prediction pyramid in (0, scale) like the disp head."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for i in range(4):
        hh, ww = h // 2 ** i, w // 2 ** i
        z = smooth_texture(b, 4, hh, ww, seed + 10 + i, sigma=1.5)
        z = (z - 0.5) * 4 + 0.2 * torch.randn(b, 4, hh, ww, generator=g)
        out.append(scale * torch.sigmoid(z))
    return out


# ------------------------------------------------------------------ goldens --
def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: (v.detach().cpu().numpy() if torch.is_tensor(v)
                                     else np.asarray(v)) for k, v in arrays.items()})
    print(f'wrote {path} ({os.path.getsize(path) / 1024:.1f} KB)')


def gen_warp(ref_utils):
    g = torch.Generator().manual_seed(7)
    arrays = {}
    for tag, (b, h, w) in {'small': (2, 4, 8), 'mid': (2, 32, 64)}.items():
        img = torch.rand(b, 3, h, w, generator=g)
        d = (torch.rand(b, 1, h, w, generator=g) - 0.5) * 0.6
        arrays[f'{tag}_img'] = img
        arrays[f'{tag}_disp'] = d
        arrays[f'{tag}_out'] = ref_utils.reconstruct(d, img)
        arrays[f'{tag}_out_zero'] = ref_utils.reconstruct(torch.zeros_like(d), img)
        arrays[f'{tag}_left'] = ref_utils.reconstruct_left_image(d, img)
        arrays[f'{tag}_right'] = ref_utils.reconstruct_right_image(d, img)
    save('warp.npz', **arrays)


def gen_loss(ref_loss, ref_utils, cfg, b=2, h=32, w=64, grads=True, name='loss.npz'):
    left, right, _ = stereo_pair(b, h, w)
    images = torch.cat([left, right], 1)
    arrays = {'images': images}
    pyr = ref_utils.scale_pyramid(images, 4)
    for i, p in enumerate(pyr):
        arrays[f'pyr{i}'] = p
    for tex, seed in (('smooth', 21), ('rough', 22)):
        preds = pred_pyramid(b, h, w, seed)
        if tex == 'rough':
            g = torch.Generator().manual_seed(99)
            preds = [0.3 * torch.rand(p.shape, generator=g).clamp_min(1e-3) for p in preds]
        for i, p in enumerate(preds):
            arrays[f'{tex}_pred{i}'] = p
        for lt in ('l1', 'bayesian', 'log_bayesian'):
            lcfg = json.loads(json.dumps(cfg['loss']))
            lcfg['error_loss_config']['loss_type'] = lt
            lf = ref_loss.TukraUncertaintyLoss(**lcfg)
            ps = [p.clone().requires_grad_(True) for p in preds]
            recon = ref_utils.reconstruct_pyramid(ps, pyr)
            if lt == 'l1':
                for i, r in enumerate(recon):
                    arrays[f'{tex}_recon{i}'] = r
            dl, el = lf(pyr, ps, recon, 0, None)
            arrays[f'{tex}_{lt}_disp_loss'] = dl.detach()
            arrays[f'{tex}_{lt}_error_loss'] = el.detach()
            if not grads:
                continue
            # separate gradients of the two returned scalars
            ps2 = [p.clone().requires_grad_(True) for p in preds]
            recon2 = ref_utils.reconstruct_pyramid(ps2, pyr)
            dl2, el2 = lf(pyr, ps2, recon2, 0, None)
            gd = torch.autograd.grad(dl2, ps2, retain_graph=True, allow_unused=True)
            ge = torch.autograd.grad(el2, ps2, allow_unused=True)
            for i in range(4):
                arrays[f'{tex}_{lt}_gdisp{i}'] = gd[i] if gd[i] is not None else torch.zeros_like(preds[i])
                arrays[f'{tex}_{lt}_gerr{i}'] = ge[i] if ge[i] is not None else torch.zeros_like(preds[i])
            # per-term values (reference sub-modules, same loop as loss.py:541-550)
            with torch.no_grad():
                t = {'wssim': 0., 'consistency': 0., 'smoothness': 0., 'error': 0.}
                rc = ref_utils.reconstruct_pyramid(preds, pyr)
                for i, (im, p, r) in enumerate(zip(pyr, preds, rc)):
                    d = p[:, :2]
                    t['wssim'] += float(lf.wssim(im, r))
                    t['consistency'] += float(lf.consistency(d))
                    t['smoothness'] += float(lf.smoothness(d, im) / 2 ** i)
                    t['error'] += float(lf.predictive_error(p, im, lf.wssim.previous_image_error))
                    if lt == 'l1':
                        arrays[f'{tex}_err{i}'] = lf.wssim.previous_image_error
                for k, v in t.items():
                    arrays[f'{tex}_{lt}_term_{k}'] = np.float64(v)
    if not grads:
        arrays = {k: v for k, v in arrays.items() if 'recon' not in k
                  and not k.startswith('pyr') and 'err' not in k[-5:]}
    save(name, **arrays)


def _formula_weights(cfg, nodes_dir=None):
    sys.path.insert(0, REPO)
    from oracle import model as OM  # noqa: E402
    from oracle import step as OS  # noqa: E402
    graphs = OM.load_stage_graphs(cfg['model']['encoder'])
    specs = OS.param_specs(cfg['model'], graphs)
    return OS.formula_state_dict(specs), specs


def _ref_model(ref_model, cfg):
    mcfg = json.loads(json.dumps(cfg['model']))
    mcfg['encoder']['load_graph'] = os.path.join(REF, 'graphs', 'nodes_5_seed_42') \
        if mcfg['encoder'].get('nodes', 5) == 5 else \
        os.path.join('/nonexistent', os.path.basename(mcfg['encoder']['load_graph']))
    return ref_model.RandomlyConnectedModel(**mcfg)


def gen_model(ref_model, cfg):
    sd, specs = _formula_weights(cfg)
    m = _ref_model(ref_model, cfg)
    ref_keys = list(m.state_dict().keys())
    assert ref_keys == [s[0] for s in specs], 'state_dict schema mismatch'
    shapes_ok = all(tuple(m.state_dict()[k].shape) == tuple(s[1]) for k, s in zip(ref_keys, specs))
    assert shapes_ok
    m.load_state_dict(sd)
    b, h, w = 2, 64, 128
    left, right, _ = stereo_pair(b, h, w, seed=4321)
    m.train()
    with torch.no_grad():
        d1, d2, d3, d4 = m(left, 0.3)
    arrays = {'left': left, 'train_d1': d1, 'train_d2': d2, 'train_d3': d3, 'train_d4': d4}
    arrays['running_mean_sum'] = sum(v.sum() for k, v in m.state_dict().items()
                                     if k.endswith('running_mean'))
    arrays['running_var_sum'] = sum(v.sum() for k, v in m.state_dict().items()
                                    if k.endswith('running_var'))
    m2 = _ref_model(ref_model, cfg)
    m2.load_state_dict(sd)
    m2.eval()
    with torch.no_grad():
        arrays['eval_d1'] = m2(left[:1], 0.3)
    # encoder features at stage granularity (a localisation aid)
    with torch.no_grad():
        m3 = _ref_model(ref_model, cfg)
        m3.load_state_dict(sd)
        m3.train()
        feats = m3.encoder(left)
        for i, f in enumerate(feats):
            arrays[f'feat{i}_sum'] = f.double().sum()
            arrays[f'feat{i}_abssum'] = f.double().abs().sum()
    arrays['schema'] = np.array(json.dumps([[s[0], list(s[1])] for s in specs]))
    save('model_fwd.npz', **arrays)


def gen_step(ref_model, ref_loss, ref_utils, cfg, loss_type, steps=3, tag=None, b=2, h=64,
             w=128, disp_levels=(0, 1, 2, 3)):
    sd, specs = _formula_weights(cfg)
    m = _ref_model(ref_model, cfg)
    m.load_state_dict(sd)
    m.train()
    lcfg = json.loads(json.dumps(cfg['loss']))
    lcfg['error_loss_config']['loss_type'] = loss_type
    lf = ref_loss.TukraUncertaintyLoss(**lcfg)
    opt = torch.optim.Adam(m.parameters(), 1e-4)
    left, right, _ = stereo_pair(b, h, w, seed=555)
    arrays = {'left': left, 'right': right}
    scale = float(ref_utils.adjust_disparity(0))
    arrays['scale'] = np.float64(scale)
    for step in range(steps):
        images = torch.cat([left, right], 1)
        pyr = ref_utils.scale_pyramid(images, 4)
        opt.zero_grad()
        disps = m(left, scale)
        recon = ref_utils.reconstruct_pyramid(disps, pyr)
        dl, el = lf(pyr, disps, recon, step, None)
        (dl + el).backward()
        if step == 0:
            from oracle import step as OS  # noqa: E402
            for k, p in m.named_parameters():
                arrays[f'gradnorm/{k}'] = p.grad.double().norm()
                arrays[f'sketch/{k}'] = OS.grad_sketch(k, p.grad)
            for i, d in enumerate(disps):
                if i in disp_levels:
                    arrays[f'step0_disp{i}'] = d.detach()
                arrays[f'step0_disp{i}_sum'] = d.detach().double().sum()
                arrays[f'step0_disp{i}_abssum'] = d.detach().double().abs().sum()
        opt.step()
        arrays[f'disp_loss_{step}'] = dl.detach()
        arrays[f'error_loss_{step}'] = el.detach()
        if step == 0:
            for k, v in m.state_dict().items():
                if k.endswith('running_mean') or k.endswith('running_var'):
                    arrays[f'bn/{k}'] = v.clone()
                elif v.is_floating_point():
                    arrays[f'param_sum/{k}'] = v.double().sum()
                    arrays[f'param_abs/{k}'] = v.double().abs().sum()
    save(f'step_{tag or loss_type}.npz', **arrays)


def gen_traj(ref_model, ref_loss, ref_utils, cfg, steps=10, b=8, h=256, w=512):
    """BASELINE config 2 at full size: 10 fp32 steps of the reference loop
    body (train/train.py:116-129, Adam lr 1e-4, scale 0.3) on the bench's own
    synthetic pair (oracle.step.bench_inputs: U[0,1), seed 1234) with formula
    weights -- the "loss delta vs ref" trajectory of the BASELINE metric,
    plus step-0 gradient sketches and disparity sums at this size."""
    from oracle import step as OS  # noqa: E402
    sd, _ = _formula_weights(cfg)
    m = _ref_model(ref_model, cfg)
    m.load_state_dict(sd)
    m.train()
    lcfg = json.loads(json.dumps(cfg['loss']))
    lcfg['error_loss_config']['loss_type'] = 'bayesian'
    lf = ref_loss.TukraUncertaintyLoss(**lcfg)
    opt = torch.optim.Adam(m.parameters(), 1e-4)
    left, right = OS.bench_inputs(b, h, w)
    arrays = {'shape': np.array([b, h, w]), 'seed': np.int64(1234), 'scale': np.float64(0.3)}
    for step in range(steps):
        pyr = ref_utils.scale_pyramid(torch.cat([left, right], 1), 4)
        opt.zero_grad()
        disps = m(left, 0.3)
        recon = ref_utils.reconstruct_pyramid(disps, pyr)
        dl, el = lf(pyr, disps, recon, step, None)
        (dl + el).backward()
        if step == 0:
            for k, p in m.named_parameters():
                arrays[f'gradnorm/{k}'] = p.grad.double().norm()
                arrays[f'sketch/{k}'] = OS.grad_sketch(k, p.grad)
            for i, d in enumerate(disps):
                arrays[f'step0_disp{i}_sum'] = d.detach().double().sum()
                arrays[f'step0_disp{i}_abssum'] = d.detach().double().abs().sum()
            arrays['step0_disp3'] = disps[3].detach()
        opt.step()
        arrays[f'disp_loss_{step}'] = np.float64(float(dl))
        arrays[f'error_loss_{step}'] = np.float64(float(el))
        print(f'traj step {step}: {float(dl):.6f} {float(el):.6f}', flush=True)
    save('traj_c2.npz', **arrays)


def gen_traj_bf16(ref_model, ref_loss, ref_utils, cfg, steps=10, b=8, h=256, w=512):
    """The same 10 config-2 steps as gen_traj, with the reference's forward and
    loss under CPU bf16 autocast (torch.autocast('cpu', torch.bfloat16); the
    backward and Adam as autocast leaves them).  This is the reference's OWN
    bf16 deviation at exactly the bench's workload (weights, pair, scale), the
    yardstick BASELINE.md's bf16 bar was measured with (at other
    weights).  Stores the per-step loss scalars and the step-0 disparity sums."""
    sys.path.insert(0, REPO)
    from oracle import step as OS  # noqa: E402
    sd, _ = _formula_weights(cfg)
    m = _ref_model(ref_model, cfg)
    m.load_state_dict(sd)
    m.train()
    lcfg = json.loads(json.dumps(cfg['loss']))
    lcfg['error_loss_config']['loss_type'] = 'bayesian'
    lf = ref_loss.TukraUncertaintyLoss(**lcfg)
    opt = torch.optim.Adam(m.parameters(), 1e-4)
    left, right = OS.bench_inputs(b, h, w)
    arrays = {'shape': np.array([b, h, w]), 'seed': np.int64(1234), 'scale': np.float64(0.3)}
    for step in range(steps):
        with torch.autocast('cpu', dtype=torch.bfloat16):
            pyr = ref_utils.scale_pyramid(torch.cat([left, right], 1), 4)
            opt.zero_grad()
            disps = m(left, 0.3)
            recon = ref_utils.reconstruct_pyramid(disps, pyr)
            dl, el = lf(pyr, disps, recon, step, None)
        (dl + el).float().backward()
        if step == 0:
            for i, d in enumerate(disps):
                arrays[f'step0_disp{i}_sum'] = d.detach().double().sum()
                arrays[f'step0_disp{i}_abssum'] = d.detach().double().abs().sum()
        opt.step()
        arrays[f'disp_loss_{step}'] = np.float64(float(dl))
        arrays[f'error_loss_{step}'] = np.float64(float(el))
        print(f'traj bf16 step {step}: {float(dl):.6f} {float(el):.6f}', flush=True)
    save('traj_c2_bf16.npz', **arrays)


def disp_bf16_stats(got, ref):
    """(max-abs/max-ref, mean relative) of a disparity/uncertainty map
    against its fp32 counterpart; the same formulas as the GPU tests"""
    g, r = got.double(), ref.double()
    mx = float((g - r).abs().max() / r.abs().max())
    mr = float(((g - r).abs() / r.abs().clamp_min(1e-6)).mean())
    return mx, mr


def gen_disp_bf16(ref_model, cfg, b=8, h=256, w=512):
    """The reference's OWN bf16 disparity deviation at BASELINE config 2
    (B=8, 256x512, formula weights, the bench's synthetic pair, scale 0.3,
    train-mode forward): the model run in fp32 and under
    torch.autocast('cpu', torch.bfloat16), compared per scale by
    max-abs/max-ref and mean relative error (disp_bf16_stats).  Stores the
    per-scale figures, the fp32 and bf16 maps of the coarsest scale
    (8x4x32x64) and the per-scale sums of the fp32 maps.  The GPU test holds
    our bf16 build to max(BASELINE.md's bar, 1.1 x these figures)."""
    sys.path.insert(0, REPO)
    from oracle import step as OS  # noqa: E402
    sd, _ = _formula_weights(cfg)
    m = _ref_model(ref_model, cfg)
    m.load_state_dict(sd)
    m.train()
    left, _ = OS.bench_inputs(b, h, w)
    arrays = {'shape': np.array([b, h, w]), 'seed': np.int64(1234), 'scale': np.float64(0.3)}
    with torch.no_grad():
        d32 = [d.clone() for d in m(left, 0.3)]
        m.load_state_dict(sd)  # the same running statistics before the second forward
        with torch.autocast('cpu', dtype=torch.bfloat16):
            d16 = [d.float().clone() for d in m(left, 0.3)]
    for i, (a, r) in enumerate(zip(d16, d32)):
        mx, mr = disp_bf16_stats(a, r)
        arrays[f'max_rel_{i}'] = np.float64(mx)
        arrays[f'mean_rel_{i}'] = np.float64(mr)
        arrays[f'fp32_sum_{i}'] = r.double().sum()
        arrays[f'fp32_abssum_{i}'] = r.double().abs().sum()
        print(f'disp bf16 scale {i} {tuple(r.shape)}: max-abs/max-ref {mx:.3e}, '
              f'mean rel {mr:.3e}', flush=True)
    arrays['fp32_d3'] = d32[3]
    arrays['bf16_d3'] = d16[3]
    # the same figures on tests/test_gpu_model.py's U[0,1) pair (B=2, 64x128,
    # torch.Generator seed 1234, the left view), the input of its bf16 test
    g = torch.Generator().manual_seed(1234)
    left64 = torch.rand(2, 3, 64, 128, generator=g)
    with torch.no_grad():
        m.load_state_dict(sd)
        u32 = [d.clone() for d in m(left64, 0.3)]
        m.load_state_dict(sd)
        with torch.autocast('cpu', dtype=torch.bfloat16):
            u16 = [d.float().clone() for d in m(left64, 0.3)]
    for i, (a, r) in enumerate(zip(u16, u32)):
        mx, mr = disp_bf16_stats(a, r)
        arrays[f'u64_max_rel_{i}'] = np.float64(mx)
        arrays[f'u64_mean_rel_{i}'] = np.float64(mr)
        print(f'disp bf16 U[0,1) 64x128 scale {i}: max-abs/max-ref {mx:.3e}, mean rel {mr:.3e}',
              flush=True)
    save('disp_c2_bf16.npz', **arrays)


def uniform_pair(b, h, w, seed):
    """tests/test_gpu_model.py's _uniform_pair: U[0,1) left and right views"""
    g = torch.Generator().manual_seed(seed)
    return torch.rand(b, 3, h, w, generator=g), torch.rand(b, 3, h, w, generator=g)


LOSS_BF16_CASES = {  # tag: (config, batch, height, width, seeds)
    'u64': ('config.yml', 2, 64, 128, (99, 100, 101, 102, 103, 104, 105, 106)),
    'c2u': ('config.yml', 8, 256, 512, (99,)),
    'c5u': ('config_nodes10.yml', 8, 512, 1024, (5,)),
}


def gen_loss_bf16(ref_model, ref_loss, ref_utils):
    """The reference's OWN bf16-autocast deviation of the step-0 loss
    scalars (forward + loss, formula weights, bayesian, scale 0.3) on the
    U[0,1) inputs of the GPU tests' bf16 loss checks: per case and seed the
    fp32 and torch.autocast('cpu', bf16) disparity / error losses.  The
    nodes=10 graphs (config 5) run forward only, which the reference can do
    (its in-place output sum breaks only the backward)."""
    arrays = {}
    for tag, (cname, b, h, w, seeds) in LOSS_BF16_CASES.items():
        with open(os.path.join(REPO, cname)) as f:
            cfg = yaml.safe_load(f)
        sd, _ = _formula_weights(cfg)
        m = _ref_model(ref_model, cfg)
        m.train()
        lcfg = json.loads(json.dumps(cfg['loss']))
        lcfg['error_loss_config']['loss_type'] = 'bayesian'
        lf = ref_loss.TukraUncertaintyLoss(**lcfg)
        for seed in seeds:
            left, right = uniform_pair(b, h, w, seed)
            for mode in ('fp32', 'bf16'):
                m.load_state_dict(sd)
                with torch.no_grad(), torch.autocast('cpu', dtype=torch.bfloat16,
                                                     enabled=mode == 'bf16'):
                    pyr = ref_utils.scale_pyramid(torch.cat([left, right], 1), 4)
                    d = m(left, 0.3)
                    dl, el = lf(pyr, d, ref_utils.reconstruct_pyramid(d, pyr), 0, None)
                arrays[f'{tag}_{seed}_{mode}'] = np.array([float(dl), float(el)])
            a, r = arrays[f'{tag}_{seed}_bf16'], arrays[f'{tag}_{seed}_fp32']
            print(f'loss bf16 {tag} seed {seed}: rel disp {abs(a[0] / r[0] - 1):.3e} '
                  f'error {abs(a[1] / r[1] - 1):.3e}', flush=True)
    save('loss_bf16.npz', **arrays)


def train_model_pairs():
    """7 smooth stereo pairs at 64x128 (a ragged last batch at batch 2)"""
    left, right, _ = stereo_pair(7, 64, 128, seed=2468)
    return left, right


def gen_train_model(ref_model, ref_loss, ref_utils, cfg):
    """The reference's own epoch loop, train/train.py:173-267: train_model
    over a DataLoader of 7 pairs (batch 2, so a ragged last batch), 2 epochs,
    the disparity scale moving 0.3 -> 0.5 between them (adjust_disparity
    passed in, as train_model allows), the reference adjust_learning_rate,
    bayesian loss, fp32, formula weights.  Stores the per-epoch losses per
    image, and the reference adjust_learning_rate over epochs 0..45 (plain
    and finetune)."""
    from torch.utils.data import DataLoader
    import train.train as ref_train  # noqa: E402
    sd, _ = _formula_weights(cfg)
    m = _ref_model(ref_model, cfg)
    m.load_state_dict(sd)
    lcfg = json.loads(json.dumps(cfg['loss']))
    lcfg['error_loss_config']['loss_type'] = 'bayesian'
    lf = ref_loss.TukraUncertaintyLoss(**lcfg)
    left, right = train_model_pairs()
    ds = [{'left': left[i], 'right': right[i]} for i in range(left.shape[0])]
    loader = DataLoader(ds, batch_size=2, shuffle=False)
    scales = [0.3, 0.5]
    losses, _ = ref_train.train_model(m, loader, lf, epochs=2, learning_rate=1e-4,
                                      adjust_disparity=lambda e: scales[e], no_pbar=True)
    arrays = {'left': left, 'right': right, 'scales': np.array(scales),
              'epoch_disp': np.array([l[0] for l in losses]),
              'epoch_unc': np.array([l[1] for l in losses])}
    opt = torch.optim.Adam([torch.zeros(1, requires_grad=True)], 1e-4)
    for ft in (False, True):
        lrs = []
        for e in range(46):
            ref_utils.adjust_learning_rate(opt, e, 1e-4, finetune=ft)
            lrs.append(opt.param_groups[0]['lr'])
        arrays['lr_finetune' if ft else 'lr'] = np.array(lrs)
    print('train_model epochs:', losses, flush=True)
    # the same loop in float64: the reference's own fp32 noise on these
    # per-epoch losses (Adam turns summation-order noise in near-zero
    # gradient components into update sign flips), the scale of the bar
    torch.set_default_dtype(torch.float64)
    try:
        m64 = _ref_model(ref_model, cfg)
        m64.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in sd.items()})
        ds64 = [{'left': left[i].double(), 'right': right[i].double()}
                for i in range(left.shape[0])]
        losses64, _ = ref_train.train_model(m64, DataLoader(ds64, batch_size=2, shuffle=False),
                                            lf, epochs=2, learning_rate=1e-4,
                                            adjust_disparity=lambda e: scales[e], no_pbar=True)
    finally:
        torch.set_default_dtype(torch.float32)
    arrays['epoch_disp_f64'] = np.array([l[0] for l in losses64])
    arrays['epoch_unc_f64'] = np.array([l[1] for l in losses64])
    print('train_model epochs (f64):', losses64, flush=True)
    save('train_model.npz', **arrays)


def gen_nodes10(ref_model, cfg10):
    sd, specs = _formula_weights(cfg10)
    m = _ref_model(ref_model, cfg10)
    assert list(m.state_dict().keys()) == [s[0] for s in specs]
    m.load_state_dict(sd)
    m.train()
    left, _, _ = stereo_pair(1, 64, 128, seed=777)
    with torch.no_grad():
        d = m(left, 0.3)
    save('nodes10_fwd.npz', left=left, train_d1=d[0], train_d4=d[3],
         schema=np.array(json.dumps([[s[0], list(s[1])] for s in specs])))


def gen_transforms():
    """The reference's RandomFlip / RandomAugment decision and arithmetic
    logic (train/transforms.py:44-129) on seeded numpy RNG draws.  torchvision
    is absent: RandomHorizontalFlip(1) is stubbed by a tensor flip, which is
    torchvision's tensor semantics."""
    tv = sys.modules['torchvision.transforms']
    tv.RandomHorizontalFlip = lambda p: (lambda x: x.flip(-1))
    import importlib
    import train.transforms as ref_t  # noqa: E402
    importlib.reload(ref_t)
    g = torch.Generator().manual_seed(99)
    left = torch.rand(3, 24, 40, generator=g)
    right = torch.rand(3, 24, 40, generator=g)
    flip = ref_t.RandomFlip(0.5)
    aug = ref_t.RandomAugment(0.5, gamma=(0.8, 1.2), brightness=(0.5, 2.0), colour=(0.8, 1.2))
    np.random.seed(2024)
    arrays = {'left': left, 'right': right}
    for i in range(12):
        out = aug(flip({'left': left.clone(), 'right': right.clone()}))
        arrays[f'left{i}'] = out['left']
        arrays[f'right{i}'] = out['right']
    save('transforms.npz', **arrays)


def gen_sparsification():
    """train/sparsification.py curves on synthetic error / uncertainty maps
    (the deterministic parts: the oracle and predicted curves, AUSE; the
    random curve is recorded for its seed only)."""
    import train.sparsification as ref_s  # noqa: E402
    g = torch.Generator().manual_seed(7)
    b, h, w = 2, 40, 72
    err = torch.rand(b, 2, h, w, generator=g) ** 2
    unc = (err + 0.3 * torch.rand(b, 2, h, w, generator=g)).clamp_min(0)
    oracle = ref_s.curve(err, err)
    pred = ref_s.curve(err, unc)
    save('sparsification.npz', err=err, unc=unc, oracle_curve=oracle, pred_curve=pred,
         ause=ref_s.ause(oracle, pred))


def disc_setup(cfg, h, w):
    """discriminator config for an h x w input (linear_in_features follows
    the final map: C * h/32 * w/32) and its formula weights"""
    sys.path.insert(0, REPO)
    from oracle import graph as og  # noqa: E402
    from oracle import step as OS  # noqa: E402
    dcfg = json.loads(json.dumps(cfg['discriminator']))
    dcfg['linear_in_features'] = dcfg['final_conv']['out_channels'] * (h // 32) * (w // 32)
    nstages = len(dcfg['layers']) + 1
    graphs = [og.load_json(os.path.join(REPO, 'graphs', 'nodes_5_seed_42', f'stage_{s}.json'))
              for s in range(1, nstages + 1)]
    return dcfg, OS.formula_state_dict(OS.disc_param_specs(dcfg, graphs))


def gen_adversarial(ref_model, ref_loss, ref_utils, cfg):
    """RandomDiscriminator forward/features, GeneratorLoss, PerceptualLoss,
    run_discriminator (model/discriminator.py, train/loss.py:267-337,
    train/utils.py:248-273) and two adversarial training steps
    (train/train.py:112-152) at B=2, 64x128 with formula weights."""
    b, h, w = 2, 64, 128
    dcfg, dsd = disc_setup(cfg, h, w)
    rcfg = json.loads(json.dumps(dcfg))
    rcfg['load_graph'] = os.path.join(REF, 'graphs', 'nodes_5_seed_42')
    disc = ref_model.RandomDiscriminator(**rcfg)
    assert list(disc.state_dict().keys()) == list(dsd.keys()), 'disc schema'
    disc.load_state_dict(dsd)
    disc.train()
    left, right, _ = stereo_pair(b, h, w, seed=808)
    pyr = ref_utils.scale_pyramid(torch.cat([left, right], 1), 4)
    preds = [p.requires_grad_(True) for p in pred_pyramid(b, h, w, seed=909)]
    recon = ref_utils.reconstruct_pyramid(preds, pyr)
    arrays = {'left': left, 'right': right, 'disc_cfg': np.array(json.dumps(dcfg))}
    for i, p in enumerate(preds):
        arrays[f'pred{i}'] = p.detach()
    with torch.no_grad():
        d2 = ref_model.RandomDiscriminator(**rcfg)
        d2.load_state_dict(dsd)
        d2.train()
        arrays['prob_images'] = d2(pyr)
        for i, f in enumerate(d2.features(pyr)):
            arrays[f'feat{i}_sum'] = f.double().sum()
            arrays[f'feat{i}_abssum'] = f.double().abs().sum()
    gen = ref_loss.GeneratorLoss('mse')(recon, disc)
    per = ref_loss.PerceptualLoss()(pyr, recon, disc)
    arrays['generator_loss'] = gen.detach()
    arrays['perceptual_loss'] = per.detach()
    g = torch.autograd.grad(gen * 0.85 + per * 0.05, preds)
    for i, gi in enumerate(g):
        arrays[f'adv_grad{i}'] = gi
    d3 = ref_model.RandomDiscriminator(**rcfg)
    d3.load_state_dict(dsd)
    d3.train()
    dl = ref_utils.run_discriminator(pyr, recon, d3, torch.nn.BCELoss(), b)
    dl.backward()
    arrays['disc_loss'] = dl.detach()
    for k, p in d3.named_parameters():
        arrays[f'disc_gradnorm/{k}'] = p.grad.double().norm()
    # two adversarial training steps (reference train_one_epoch body)
    from copy import deepcopy
    sd, _ = _formula_weights(cfg)
    m = _ref_model(ref_model, cfg)
    m.load_state_dict(sd)
    m.train()
    lcfg = json.loads(json.dumps(cfg['loss']))
    lcfg['error_loss_config']['loss_type'] = 'bayesian'
    lcfg['perceptual_start'] = 1  # the perceptual term from batch 1 on
    lf = ref_loss.TukraUncertaintyLoss(**lcfg)
    d4 = ref_model.RandomDiscriminator(**rcfg)
    d4.load_state_dict(dsd)
    d4.train()
    opt = torch.optim.Adam(m.parameters(), 1e-4)
    dopt = torch.optim.Adam(d4.parameters(), 1e-4)
    clone = deepcopy(d4)
    for i in range(2):
        images = torch.cat([left, right], 1)
        pyr = ref_utils.scale_pyramid(images, 4)
        opt.zero_grad()
        disps = m(left, 0.3)
        rec = ref_utils.reconstruct_pyramid(disps, pyr)
        dl_, el_ = lf(pyr, disps, rec, i, clone)
        (dl_ + el_).backward()
        opt.step()
        dopt.zero_grad()
        dsl = ref_utils.run_discriminator(pyr, rec, d4, torch.nn.BCELoss(), b)
        dsl.backward()
        dopt.step()
        if i % 10 == 0:
            clone.load_state_dict(d4.state_dict())
        arrays[f'step_disp_{i}'] = dl_.detach()
        arrays[f'step_err_{i}'] = el_.detach()
        arrays[f'step_disc_{i}'] = dsl.detach()
        if i == 0:  # parameters after the first model and discriminator updates
            for pre, mod in (('model', m), ('disc', d4)):
                for k, v in mod.state_dict().items():
                    if v.is_floating_point():
                        arrays[f'{pre}_sum/{k}'] = v.double().sum()
                        arrays[f'{pre}_abs/{k}'] = v.double().abs().sum()
    save('adversarial.npz', **arrays)


def main():
    ref_model, ref_loss, ref_utils = import_reference()
    torch.set_num_threads(8)
    with open(os.path.join(REPO, 'config.yml')) as f:
        cfg = yaml.safe_load(f)
    with open(os.path.join(REPO, 'config_nodes10.yml')) as f:
        cfg10 = yaml.safe_load(f)
    which = sys.argv[1:] or ['warp', 'loss', 'model', 'step', 'nodes10', 'c1', 'transforms',
                             'sparsification', 'adversarial', 'traj', 'train_model']
    if 'warp' in which:
        gen_warp(ref_utils)
    if 'loss' in which:
        gen_loss(ref_loss, ref_utils, cfg)
        gen_loss(ref_loss, ref_utils, cfg, 2, 64, 128, grads=False, name='loss_64x128.npz')
    if 'model' in which:
        gen_model(ref_model, cfg)
    if 'step' in which:
        gen_step(ref_model, ref_loss, ref_utils, cfg, 'bayesian')
        gen_step(ref_model, ref_loss, ref_utils, cfg, 'l1', steps=1)
    if 'nodes10' in which:
        gen_nodes10(ref_model, cfg10)
    if 'traj' in which:  # BASELINE config 2, full size (slow: ~1 min on 8 cores)
        gen_traj(ref_model, ref_loss, ref_utils, cfg)
    if 'traj_bf16' in which:  # the reference's own bf16-autocast deviation at config 2
        gen_traj_bf16(ref_model, ref_loss, ref_utils, cfg)
    if 'loss_bf16' in which:  # the reference's own bf16-autocast loss deviations
        gen_loss_bf16(ref_model, ref_loss, ref_utils)
    if 'disp_bf16' in which:  # the reference's own bf16-autocast disparity deviation at C2
        gen_disp_bf16(ref_model, cfg)
    if 'train_model' in which:  # the reference's epoch loop (ragged batch, scale change)
        gen_train_model(ref_model, ref_loss, ref_utils, cfg)
    if 'c1' in which:  # BASELINE config 1: 128x256, batch 2, l1 error loss, one step
        gen_step(ref_model, ref_loss, ref_utils, cfg, 'l1', steps=1, tag='c1_l1', b=2, h=128,
                 w=256, disp_levels=(2, 3))
    if 'transforms' in which:
        gen_transforms()
    if 'sparsification' in which:
        gen_sparsification()
    if 'adversarial' in which:
        gen_adversarial(ref_model, ref_loss, ref_utils, cfg)


if __name__ == '__main__':
    main()
