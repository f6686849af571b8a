"""Kernel-level parity: each umamd autograd op (HIP) vs a plain-PyTorch fp32
CPU reference of the same op, forward and backward.  Marked gpu."""
import math

import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _nhwc(x):  # NCHW cpu -> NHWC device
    return x.permute(0, 2, 3, 1).contiguous().to(DEV)


def _nchw(x):
    return x.detach().permute(0, 3, 1, 2).float().cpu()


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


CONV_CASES = [
    # (Cin, Cout, k, stride, pad_mode, H, W)
    (8, 32, 7, 2, 'zero', 16, 24),
    (32, 32, 7, 1, 'zero', 12, 20),
    (32, 64, 5, 2, 'zero', 16, 16),
    (64, 64, 3, 1, 'zero', 8, 12),
    (40, 48, 3, 1, 'reflect', 10, 14),
    (24, 40, 1, 1, 'zero', 6, 10),
    (16, 8, 3, 1, 'reflect', 4, 6),
    # small-M deep layers: split-K partials + epilogue kernel (fwd and dgrad)
    (256, 512, 3, 1, 'zero', 4, 6),
    (128, 96, 3, 1, 'reflect', 6, 10),
    (64, 32, 5, 1, 'zero', 3, 5),
    # stride-2 data gradient by parity classes: odd sizes, split-K classes
    (64, 128, 3, 2, 'zero', 9, 11),
    (256, 512, 3, 2, 'zero', 7, 9),
    (32, 64, 5, 2, 'zero', 13, 15),
]


# shapes the halo-tiled direct conv takes (bf16, stride 1, "same" padding,
# P % 8 == 0, Q % 32 == 0, K <= 64); the tile-count threshold is lowered so
# these small images use it (forward + zero-pad data gradient)
HALO_CASES = [
    (32, 32, 7, 1, 'zero', 16, 32),
    (64, 64, 5, 1, 'zero', 8, 64),
    (40, 48, 3, 1, 'reflect', 8, 32),
    (64, 16, 3, 1, 'zero', 16, 32),
    (8, 32, 3, 1, 'reflect', 8, 64),
    # one-chunk 3x3 (32 input channels): resident weights when halo_res_kb
    # allows (forward and data gradient)
    (32, 32, 3, 1, 'zero', 16, 64),
    (32, 64, 3, 1, 'reflect', 8, 64),
    # wider outputs (halo_max_nc): 96- and 128-wide 3x3 column blocks, column
    # grids of 96 / 64 (5x5, 7x7) blocks
    (168, 128, 3, 1, 'reflect', 8, 32),
    (64, 96, 3, 1, 'zero', 8, 32),
    (88, 160, 3, 1, 'zero', 8, 32),
    (32, 88, 5, 1, 'zero', 8, 32),
    (96, 72, 7, 1, 'zero', 8, 32),
]


@pytest.mark.parametrize('case', HALO_CASES)
@pytest.mark.parametrize('pf2,res', [(0, 0), (1, 0), (0, 48)])
@pytest.mark.parametrize('hgrid', [0, 1, 3])
def test_conv_bn_elu_halo(case, pf2, res, hgrid):
    """the halo kernel forced on; weight modes: tap rows streamed (res 0),
    two rows ahead (pf2, knob halo_pf2), or -- 3x3 whose weights fit res KB
    (knob halo_res_kb) -- resident in LDS for persistent workgroups; hgrid >
    0: at most that many workgroups per column block, so each takes several
    tiles and prefetches the next one's halo (knob halo_grid); forward, BN
    statistics and data gradient"""
    from umamd._lib import lib
    knobs = {b'halo_min_tiles': 1, b'halo_pf2': pf2, b'halo_res_kb': res, b'halo_grid': hgrid}
    old = {k: lib().um_set_tuning(k, v) for k, v in knobs.items()}
    try:
        test_conv_bn_elu(case, torch.bfloat16)
    finally:
        for k, v in old.items():
            lib().um_set_tuning(k, v)


@pytest.mark.parametrize('case', HALO_CASES)
def test_conv_bn_elu_halo_persist_slots(case):
    """persistent halo workgroups (2 per column block) with the BN statistics
    in f64 slots: each tile adds its own slot rows"""
    from umamd import functional as U
    from umamd._lib import lib
    old = lib().um_set_tuning(b'halo_min_tiles', 1)
    old_g = lib().um_set_tuning(b'halo_grid', 2)
    try:
        test_conv_bn_elu(case, torch.bfloat16, arena=U.StatArena())
    finally:
        lib().um_set_tuning(b'halo_min_tiles', old)
        lib().um_set_tuning(b'halo_grid', old_g)


@pytest.mark.parametrize('case', CONV_CASES)
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_conv_bn_elu_slots(case, dtype):
    """BN statistics as f64 atomics into slots (the model-forward path):
    same bars as the partial-row reductions, with the halo kernel forced on
    for bf16 so its slot epilogue is covered too"""
    from umamd import functional as U
    from umamd._lib import lib
    old = lib().um_set_tuning(b'halo_min_tiles', 1)
    try:
        test_conv_bn_elu(case, dtype, arena=U.StatArena())
    finally:
        lib().um_set_tuning(b'halo_min_tiles', old)


@pytest.mark.parametrize('case', CONV_CASES)
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_conv_bn_elu(case, dtype, arena=None):
    import contextlib
    from umamd import functional as U
    from umamd._lib import PAD_REFLECT, PAD_ZERO
    Cin, Cout, k, stride, mode, H, W = case
    N = 2
    pad = (k - 1) // 2
    conv = nn.Conv2d(Cin, Cout, k, stride)
    bn = nn.BatchNorm2d(Cout)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    x = torch.randn(N, Cin, H, W)
    # CPU reference
    xr = x.clone().requires_grad_(True)
    cr, br = nn.Conv2d(Cin, Cout, k, stride), nn.BatchNorm2d(Cout)
    cr.load_state_dict(conv.state_dict())
    br.load_state_dict(bn.state_dict())
    xp = F.pad(xr, (pad,) * 4, mode='reflect' if mode == 'reflect' else 'constant')
    yr = F.elu(br(cr(xp)))
    g = torch.randn_like(yr)
    (yr * g).sum().backward()
    # HIP
    cd, bd = conv.to(DEV), bn.to(DEV)
    xd = _nhwc(x).to(dtype).requires_grad_(True)
    with U.stat_scope(arena, DEV) if arena is not None else contextlib.nullcontext():
        yd = U.conv_bn_elu(xd, cd, bd, pad, PAD_REFLECT if mode == 'reflect' else PAD_ZERO)
    (yd.float() * _nhwc(g)).sum().backward()
    tol = 1e-4 if dtype == torch.float32 else 5e-2
    assert _rel(_nchw(yd), yr) < tol
    assert _rel(_nchw(xd.grad), xr.grad) < tol * 5
    assert _rel(cd.weight.grad, cr.weight.grad) < tol * 5
    assert _rel(bd.weight.grad, br.weight.grad) < tol * 5
    assert _rel(bd.bias.grad, br.bias.grad) < tol * 5
    # the conv bias before a training-mode BN: true gradient 0; the closed
    # form (um_bn_bwd_stats_coeffs) and torch's reduction of dy are both
    # rounding noise far below the weight gradient's scale
    wscale = float(cr.weight.grad.abs().max())
    assert float(cd.bias.grad.abs().max()) < 1e-3 * wscale
    assert float(cr.bias.grad.abs().max()) < 1e-3 * wscale
    assert _rel(bd.running_mean, br.running_mean) < tol
    assert _rel(bd.running_var, br.running_var) < tol
    assert int(bd.num_batches_tracked) == 1


def test_conv_first_layer_padded_channels():
    """3-channel image -> 8-channel NHWC pad; weight packed with Creal=3."""
    from umamd import functional as U
    from umamd._lib import PAD_ZERO
    conv = nn.Conv2d(3, 32, 7, 2)
    bn = nn.BatchNorm2d(32)
    x = torch.rand(2, 3, 32, 64)
    yr = F.elu(bn(conv(F.pad(x, (3,) * 4))))
    xd = U.image_to_nhwc(x.to(DEV), torch.float32)
    yd = U.conv_bn_elu(xd, conv.to(DEV), bn.to(DEV), 3, PAD_ZERO)
    assert _rel(_nchw(yd), yr) < 1e-4


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_merge(dtype):
    from umamd import functional as U
    w = torch.tensor([0.3, -0.7, 1.1, 0.2])
    xs = [torch.randn(2, 4, 6, 16) for _ in range(4)]
    wr = w.clone().requires_grad_(True)
    xr = [x.clone().requires_grad_(True) for x in xs]
    ref = torch.sigmoid(wr[0]) * xr[0]
    for i, x in enumerate(xr[1:]):
        ref = ref + torch.sigmoid(wr[i]) * x
    g = torch.randn_like(ref)
    (ref * g).sum().backward()
    wd = w.to(DEV).requires_grad_(True)
    xd = [x.to(DEV).to(dtype).requires_grad_(True) for x in xs]
    out = U.merge(xd, wd, [0, 0, 1, 2])
    (out.float() * g.to(DEV)).sum().backward()
    tol = 1e-6 if dtype == torch.float32 else 2e-2
    assert _rel(out, ref) < tol
    assert _rel(wd.grad, wr.grad) < tol * 10
    assert wd.grad[3].item() == 0.0  # F3: last weight never used
    for a, b in zip(xd, xr):
        assert _rel(a.grad, b.grad) < tol


@pytest.mark.parametrize('C,H,W', [(32, 16, 32), (64, 8, 8), (512, 2, 4), (256, 4, 8),
                                   (32, 20, 30), (128, 12, 16), (64, 40, 72),
                                   # the MFMA heads (d = 16/32/64) at the encoder's
                                   # stage 3-5 sizes and at ragged pixel counts
                                   (128, 32, 64), (256, 16, 32), (512, 8, 16), (256, 9, 13),
                                   (512, 5, 7), (128, 3, 50)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_attention_block(C, H, W, dtype):
    from oracle.model import efficient_attention
    from umamd import functional as U
    import importlib
    att = importlib.import_module('model.layers.attention').EfficientAttention(C, C, C, 8)
    x = torch.randn(2, C, H, W)
    P = {k: v.clone().requires_grad_(True) for k, v in att.state_dict().items()}
    xr = x.clone().requires_grad_(True)
    yr = efficient_attention(xr, P, '', 8)
    g = torch.randn_like(yr)
    (yr * g).sum().backward()
    ad = att.to(DEV)
    xd = _nhwc(x).to(dtype).requires_grad_(True)
    yd = U.attention_block(xd, ad)
    (yd.float() * _nhwc(g)).sum().backward()
    tol = 1e-4 if dtype == torch.float32 else 5e-2
    # bf16 output: one rounding of the stored activation is up to 2^-8 of
    # the largest value, so the forward bar is ~2.5 ulp there
    assert _rel(_nchw(yd), yr) < (tol / 10 if dtype == torch.float32 else 1e-2)
    assert _rel(_nchw(xd.grad), xr.grad) < tol
    for name in ('keys', 'queries', 'values', 'reprojection'):
        for t in ('weight', 'bias'):
            ref = P[f'{name}.{t}'].grad
            got = getattr(getattr(ad, name), t).grad
            if name == 'keys' and t == 'bias':
                # softmax over pixels is shift invariant: true gradient 0
                assert got.abs().max() < tol * (1 + ref.abs().max())
                continue
            assert _rel(got, ref) < tol, (name, t)


def _decoder_stage_case(cfg, N, h, w, with_gate, with_disp):
    import importlib
    from oracle.model import decoder_stage
    DS = importlib.import_module('model.layers.decoder').DecoderStage
    st = DS(**cfg)
    for m in st.modules():
        if isinstance(m, nn.BatchNorm2d):
            with torch.no_grad():
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    x = torch.randn(N, cfg['in_channels'], h // 2, w // 2)
    f = torch.randn(N, cfg['feature_in_channels'], h, w)
    sk = torch.randn(N, cfg['skip_in_channels'], h // 2, w // 2)
    gate = torch.rand(N, cfg['skip_in_channels']) if with_gate else None
    d = 0.3 * torch.rand(N, cfg.get('disp_channels', 2), h // 2, w // 2) if with_disp else None
    return st, x, f, sk, gate, d


@pytest.mark.parametrize('with_gate,with_disp,fC', [(False, False, 256), (True, True, 64),
                                                      (True, True, 3)])
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('skip_conv', [True, False])
def test_decoder_stage(with_gate, with_disp, fC, dtype, skip_conv, monkeypatch):
    """skip_conv: the squeeze-excite 1x1 conv with the skip half at the
    skip's resolution (SkipConvFn) or over the materialised full-size concat"""
    from oracle.model import decoder_stage
    from umamd import functional as U
    monkeypatch.setattr(U, '_SKIP_CONV', skip_conv)
    cfg = dict(in_channels=64, feature_in_channels=fC, skip_in_channels=64,
               upsample_channels=16, out_channels=32, skip_out_channels=32,
               concat_disp=with_disp, calculate_disp=True, disp_channels=4)
    N, h, w = 2, 16, 24
    st, x, f, sk, gate, d = _decoder_stage_case(cfg, N, h, w, with_gate, with_disp)
    P = {k: v.clone() for k, v in st.state_dict().items()}
    for k in P:
        if P[k].is_floating_point() and 'running' not in k:
            P[k].requires_grad_(True)
    xr, fr, skr = [t.clone().requires_grad_(True) for t in (x, f, sk)]
    dr = d.clone().requires_grad_(True) if d is not None else None
    gr = gate.clone().requires_grad_(True) if gate is not None else None
    skin = skr * gr[:, :, None, None] if gate is not None else skr
    out_r, skip_r, disp_r = decoder_stage(xr, fr, skin, dr, 0.3, P, '', cfg, True)
    go, gs, gd = torch.randn_like(out_r), torch.randn_like(skip_r), torch.randn_like(disp_r)
    ((out_r * go).sum() + (skip_r * gs).sum() + (disp_r * gd).sum()).backward()

    from umamd.functional import image_to_nhwc
    sd = st.to(DEV)
    xd = _nhwc(x).to(dtype).requires_grad_(True)
    fd = image_to_nhwc(f.to(DEV), dtype) if fC % 8 else _nhwc(f).to(dtype)
    fd.requires_grad_(fC % 8 == 0)
    skd = _nhwc(sk).to(dtype).requires_grad_(True)
    gated = gate.to(DEV).requires_grad_(True) if gate is not None else None
    dd = _nhwc(d).requires_grad_(True) if d is not None else None
    out_d, (u1, s), disp_d = sd._fwd(xd, fd, (skd, gated) if gated is not None else skd, dd,
                                     0.3)
    skip_d = u1.float() * s[:, None, None, :]
    ((out_d.float() * _nhwc(go)).sum() + (skip_d * _nhwc(gs)).sum() +
     (disp_d * _nhwc(gd)).sum()).backward()
    t = 1e-3 if dtype == torch.float32 else 1e-1
    assert _rel(_nchw(out_d), out_r) < t / 10
    assert _rel(_nchw(skip_d), skip_r) < t / 10
    assert _rel(_nchw(disp_d), disp_r) < t / 10
    assert _rel(_nchw(xd.grad), xr.grad) < t
    assert _rel(_nchw(skd.grad), skr.grad) < t
    if fC % 8 == 0:
        assert _rel(_nchw(fd.grad), fr.grad) < t
    if dd is not None:
        assert _rel(_nchw(dd.grad), dr.grad) < t
    if gated is not None:
        assert _rel(gated.grad, gr.grad) < t
    sdict = dict(sd.named_parameters())
    for k, v in P.items():
        if not (v.is_floating_point() and 'running' not in k) or v.grad is None:
            continue
        got = sdict[k].grad
        if k.endswith('layers.0.layers.0.bias') and 'disp' not in k:
            continue  # pre-BN bias: true gradient 0
        assert got is not None, k
        assert _rel(got, v.grad) < 2 * t, k


def test_pyramid_and_warp_goldens():
    from conftest import GOLDEN
    import os
    from umamd import lossfn as LF
    z = np.load(os.path.join(GOLDEN, 'loss.npz'))
    imgs = torch.from_numpy(z['images']).to(DEV)
    pyr = LF.scale_pyramid(imgs, 4)
    for i in range(4):
        assert _rel(pyr[i], torch.from_numpy(z[f'pyr{i}'])) < 1e-6
    w = np.load(os.path.join(GOLDEN, 'warp.npz'))
    for tag in ('small', 'mid'):
        img = torch.from_numpy(w[f'{tag}_img']).to(DEV)
        d = torch.from_numpy(w[f'{tag}_disp']).to(DEV)
        assert _rel(LF.reconstruct(d, img, 1.0), torch.from_numpy(w[f'{tag}_out'])) < 1e-5
        assert _rel(LF.reconstruct(0 * d, img, 1.0), torch.from_numpy(w[f'{tag}_out_zero'])) < 1e-5
        assert _rel(LF.reconstruct(d, img, -1.0), torch.from_numpy(w[f'{tag}_left'])) < 1e-5


def test_adam_matches_torch():
    from umamd.optim import Adam
    ps = [torch.randn(37, 5), torch.randn(10000), torch.randn(3)]
    gs = [[torch.randn_like(p) for p in ps] for _ in range(3)]
    pr = [p.clone().requires_grad_(True) for p in ps]
    pd = [p.clone().to(DEV).requires_grad_(True) for p in ps]
    o1 = torch.optim.Adam(pr, 1e-3)
    o2 = Adam(pd, 1e-3)
    for step in range(3):
        for p, g in zip(pr, gs[step]):
            p.grad = g.clone()
        for p, g in zip(pd, gs[step]):
            p.grad = g.clone().to(DEV)
        o1.step()
        o2.step()
    for a, b in zip(pd, pr):
        assert _rel(a, b) < 1e-6


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('case', [(8, 32, 7, 2, 64, 128), (32, 32, 7, 1, 32, 64),
                                  (64, 64, 3, 1, 32, 64)])
def test_conv_large(dtype, case):
    from umamd import functional as U
    from umamd._lib import PAD_ZERO
    Cin, Cout, k, stride, H, W = case
    conv = nn.Conv2d(Cin, Cout, k, stride)
    bn = nn.BatchNorm2d(Cout)
    x = torch.rand(2, Cin, H, W)
    xr = x.clone().requires_grad_(True)
    cr, br = nn.Conv2d(Cin, Cout, k, stride), nn.BatchNorm2d(Cout)
    cr.load_state_dict(conv.state_dict())
    br.load_state_dict(bn.state_dict())
    yr = F.elu(br(cr(F.pad(xr, ((k - 1) // 2,) * 4))))
    g = torch.randn_like(yr)
    (yr * g).sum().backward()
    cd, bd = conv.to(DEV), bn.to(DEV)
    xd = _nhwc(x).to(dtype).requires_grad_(True)
    yd = U.conv_bn_elu(xd, cd, bd, (k - 1) // 2, PAD_ZERO)
    (yd.float() * _nhwc(g)).sum().backward()
    errs = [_rel(_nchw(yd), yr), _rel(_nchw(xd.grad), xr.grad), _rel(cd.weight.grad, cr.weight.grad),
            _rel(cd.bias.grad, cr.bias.grad) if cr.bias.grad.abs().max() > 1e-3 else 0.0]
    print(f'conv_large {case} {dtype}: y {errs[0]:.3e} dx {errs[1]:.3e} dw {errs[2]:.3e}')
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    assert errs[0] < tol and errs[1] < tol * 2 and errs[2] < tol * 2, errs


# weight gradient against torch (f64 CPU) for the shapes the halo-tiled kernel
# covers (bf16, Q >= 32): 7x7/5x5 encoder convs incl. stride 2, 3x3 reflect
# decoder convs incl. the 4-channel disparity head, and a K=128 conv
@pytest.mark.parametrize('case', [
    (32, 32, 7, 1, 'zero', 12, 70),
    (8, 32, 7, 2, 'zero', 20, 72),
    (64, 64, 5, 1, 'zero', 9, 40),
    (32, 64, 5, 2, 'zero', 16, 66),
    (48, 32, 3, 1, 'reflect', 10, 36),
    (32, 8, 3, 1, 'reflect', 7, 64),
    (64, 128, 3, 1, 'reflect', 6, 33),
    # transposed-read implicit GEMM (K > 32, not halo-tiled)
    (168, 128, 3, 1, 'reflect', 8, 16),
    (256, 512, 3, 1, 'zero', 4, 8),
    (32, 96, 1, 1, 'zero', 12, 40),
    (128, 256, 3, 2, 'zero', 9, 17),
    # 1x1 VALU streaming pass (K, C in {8..64}, K*C <= 512; the rest on the
    # MFMA tiles), ragged pixel counts
    (8, 32, 1, 1, 'zero', 32, 64),
    (64, 32, 1, 1, 'zero', 16, 40),
    (32, 32, 1, 1, 'zero', 9, 17),
    (16, 8, 1, 1, 'zero', 5, 7),
    (32, 64, 1, 1, 'zero', 10, 30),
    (64, 64, 1, 1, 'zero', 8, 24),
])
def test_wgrad(case):
    from umamd import functional as U
    from umamd._lib import PAD_REFLECT, PAD_ZERO, query
    C, K, R, st, mode, H, W = case
    N = 2
    pad = (R - 1) // 2
    g = torch.Generator().manual_seed(7)
    x = torch.rand(N, C, H, W, generator=g) - 0.5
    xp = F.pad(x.double(), (pad,) * 4, mode='reflect' if mode == 'reflect' else 'constant')
    P = (H + 2 * pad - R) // st + 1
    Q = (W + 2 * pad - R) // st + 1
    dy = torch.randn(N, K, P, Q, generator=g)
    xb = x.to(torch.bfloat16)
    dyb = dy.to(torch.bfloat16)
    xpb = F.pad(xb.double(), (pad,) * 4, mode='reflect' if mode == 'reflect' else 'constant')
    ref = torch.nn.grad.conv2d_weight(xpb, (K, C, R, R), dyb.double(), stride=st)
    pm = PAD_REFLECT if mode == 'reflect' else PAD_ZERO
    got = U._conv_wgrad(_nhwc(xb).to(DEV), _nhwc(dyb).to(DEV), K, K, C, R, st, pad, pm)
    splits = query('um_conv_wgrad_splits', 1, N, H, W, C, C, K, R, st, pad, pm, P, Q, K)
    err = _rel(got, ref)
    print(f'wgrad {case}: splits {splits} rel {err:.3e}')
    assert err < 1e-4, err


# slab reduction of the large 3x3..7x7 weights (>= 256K elements: the LDS-
# transposed kernel with contiguous dW stores) against torch, with padded
# K / C, a segment map (concat input) and accumulate
@pytest.mark.parametrize('case', [(3, 64, 60, 3, 512, 500, None), (2, 32, 32, 5, 256, 256, None),
                                  (5, 24, 24, 7, 200, 200, None),
                                  (2, 48, 40, 3, 640, 600, [(0, 0, 300), (300, 320, 300)])])
@pytest.mark.parametrize('accumulate', [0, 1])
def test_wgrad_reduce_large(case, accumulate):
    from umamd import functional as U
    from umamd._lib import call, ptr
    splits, K, Kreal, R, C, Creal, segs = case
    g = torch.Generator().manual_seed(8)
    slabs = torch.randn(splits, K, R, R, C, generator=g).to(DEV)
    dw0 = torch.randn(Kreal, Creal, R, R, generator=g).to(DEV)
    dw = dw0.clone()
    n, a0, b0, l0 = U._seg_arrays(segs)
    call('um_conv_wgrad_reduce_seg', ptr(slabs), splits, K, Kreal, R, C, Creal, ptr(dw),
         accumulate, n, a0, b0, l0)
    torch.cuda.synchronize()
    ref = slabs.double().sum(0)[:Kreal].permute(0, 3, 1, 2).cpu()  # [Kreal][C][R][R]
    exp = dw0.double().cpu().clone() if accumulate else torch.full_like(dw0.double().cpu(), float('nan'))
    for src0, dst0, ln in (segs or [(0, 0, Creal)]):
        part = ref[:, dst0:dst0 + ln]
        exp[:, src0:src0 + ln] = part + (exp[:, src0:src0 + ln] if accumulate else 0)
    assert torch.allclose(dw.double().cpu(), exp, rtol=1e-5, atol=1e-5)


# the side stream's batched bias gradients (um_colsum_batch: one partial-row
# pass + one f64 finish per flush) against the per-bias reduction
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_colsum_batch_matches_per_bias(dtype):
    from umamd import functional as U
    from umamd import overlap
    g = torch.Generator().manual_seed(11)
    shapes = [(2, 64, 128, 32), (2, 16, 32, 768), (1, 8, 16, 1536), (2, 128, 256, 8),
              (3, 5, 7, 64)] * 6
    ys = [torch.randn(*sh, generator=g).to(dtype).to(DEV) for sh in shapes]
    refs = [y.double().sum(dim=(0, 1, 2)).float() for y in ys]
    with overlap.WgradStream(batch=len(ys)):
        outs = [U._colsum_grad(y, y.shape[-1]) for y in ys]
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        assert torch.allclose(o, r, rtol=1e-5, atol=1e-4), float((o - r).abs().max())


# the decoder skip conv's feature-map half (um_conv2d_fwd_up2): y = W fm +
# bias + up2(z) with the BN statistics slots taken on the sum, f32 y and the
# bf16 build's y (UM_Y_ACT: the accumulating GEMM's statistics in the staged
# 16-byte row store), against f64 torch on the same operands
@pytest.mark.parametrize('case', [(2, 64, 128, 8, 32), (2, 32, 64, 32, 64), (1, 16, 24, 16, 32),
                                  (2, 128, 64, 8, 16)])
@pytest.mark.parametrize('yact', [False, True])
def test_conv_fwd_up2_slots(case, yact):
    from umamd import functional as U
    from umamd import _lib as L
    from umamd._lib import call, ptr
    N, H, W, Cf, K = case
    h, w = H // 2, W // 2
    g = torch.Generator().manual_seed(5)
    fm = torch.rand(N, H, W, Cf, generator=g).to(torch.bfloat16).to(DEV)
    ydt = torch.bfloat16 if yact else torch.float32
    z = torch.randn(N, h, w, K, generator=g).to(ydt).to(DEV)
    wt = torch.randn(K, Cf, 1, 1, generator=g).to(DEV)
    bias = torch.randn(K, generator=g).to(DEV)
    wf, _ = U._pack(wt, Cf, torch.bfloat16)
    y = torch.empty(N, H, W, K, dtype=ydt, device=DEV)
    slots = torch.zeros(L.STAT_SLOTS * K * 2 + 1, dtype=torch.float64, device=DEV)
    call('um_conv2d_fwd_up2', L.UM_BF16 | (L.Y_ACT if yact else 0), N, H, W, Cf, Cf, ptr(fm),
         ptr(wf), ptr(bias), K, H, W, ptr(y), K, L.EPI_STAT_SLOTS, ptr(slots), ptr(z), h, w, K)
    torch.cuda.synchronize()
    wq = wt.to(torch.bfloat16).double()[:, :, 0, 0]
    ref = torch.einsum('nhwc,kc->nhwk', fm.double(), wq) + bias.double()
    up = F.interpolate(z.double().permute(0, 3, 1, 2), scale_factor=2, mode='bilinear',
                       align_corners=True).permute(0, 2, 3, 1)
    ref = ref + up
    tol = 2e-2 if yact else 1e-5
    assert _rel(y.double(), ref) < tol
    st = slots[:L.STAT_SLOTS * K * 2].view(L.STAT_SLOTS, K, 2).sum(0)
    s1, s2 = ref.sum(dim=(0, 1, 2)), (ref * ref).sum(dim=(0, 1, 2))
    scale1 = ref.abs().sum(dim=(0, 1, 2))
    # bf16 y: the statistics are of bf16(W fm + bias) + bf16(up2 z), the
    # reference of the exact sum (two 2^-9 roundings per element)
    stol = 1e-3 if yact else 1e-4
    assert float(((st[:, 0] - s1).abs() / scale1).max()) < stol
    assert float(((st[:, 1] - s2).abs() / s2).max()) < stol
    assert float(slots[-1]) == N * H * W


# the decoder's second concat: the upsample conv's output pixel-shuffled
# (PixelShuffle(2), source [N][h][w][4C] -> [N][2h][2w][C]) next to a gated
# copy source, bf16 and f32, odd source sizes, against torch pixel_shuffle +
# cat; and the adjoint of the shuffled source
@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float32])
@pytest.mark.parametrize('h,w,C', [(4, 8, 16), (5, 7, 32), (3, 33, 8), (16, 32, 64)])
def test_pshuf_concat(dtype, h, w, C):
    from umamd import functional as U
    from umamd._lib import CAT_COPY, CAT_PSHUF
    N, C2 = 2, 24
    torch.manual_seed(h + w + C)
    up = torch.randn(N, 4 * C, h, w)
    cp = torch.randn(N, C2, 2 * h, 2 * w)
    gate = torch.rand(N, C2)
    upq, cpq = up.to(dtype).float(), cp.to(dtype).float()
    ref = torch.cat([F.pixel_shuffle(upq, 2), cpq * gate[:, :, None, None]], 1)
    ud = _nhwc(upq).to(dtype).requires_grad_(True)
    cd = _nhwc(cpq).to(dtype)
    y, _ = U.concat([U.CatSource(ud, CAT_PSHUF, C), U.CatSource(cd, CAT_COPY, C2, gate.to(DEV))],
                    N, 2 * h, 2 * w, dtype)
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-6
    assert _rel(_nchw(y[..., :C + C2].float()), ref) < tol
    assert torch.equal(_nchw(y[..., :C].float()).cpu(), F.pixel_shuffle(upq, 2))
    go = torch.randn(N, 2 * h, 2 * w, y.shape[-1], device=DEV)
    (y.float() * go).sum().backward()
    gref = F.pixel_unshuffle(go[..., :C].permute(0, 3, 1, 2).cpu(), 2)
    assert _rel(_nchw(ud.grad.float()), gref) < tol


# x2 bilinear (align_corners=True) upsample of a concat source: forward and
# the adjoint (branch-free 6x6 window for low-res sides >= 4, general path
# below), with and without an SE gate, against torch
@pytest.mark.parametrize('h,w', [(4, 5), (5, 7), (8, 33), (2, 3), (16, 16)])
@pytest.mark.parametrize('gated', [False, True])
@pytest.mark.parametrize('C', [16, 4])  # 4: the disparity sources' 4-channel adjoint kernel
def test_up2_concat_adjoint(h, w, gated, C):
    from umamd import functional as U
    from umamd._lib import CAT_UP2
    N = 2
    x = torch.randn(N, C, h, w, dtype=torch.float64)
    gate = torch.rand(N, C, dtype=torch.float64) if gated else None
    xr = x.clone().requires_grad_(True)
    gr = gate.clone().requires_grad_(True) if gated else None
    src = xr * gr[:, :, None, None] if gated else xr
    yr = F.interpolate(src, scale_factor=2, mode='bilinear', align_corners=True)
    go = torch.randn_like(yr)
    (yr * go).sum().backward()
    xd = _nhwc(x.float()).requires_grad_(True)
    gd = gate.float().to(DEV).requires_grad_(True) if gated else None
    y, _ = U.concat([U.CatSource(xd, CAT_UP2, C, gd)], N, 2 * h, 2 * w, torch.float32)
    y = y[..., :C]  # the concat pads its channels to a multiple of 8
    (y.float() * _nhwc(go.float())).sum().backward()
    assert _rel(_nchw(y), yr) < 1e-5
    assert _rel(_nchw(xd.grad), xr.grad) < 1e-5
    if gated:
        assert _rel(gd.grad, gr.grad) < 1e-5


# data gradient through the 48/96/160-wide tiles (NC = the conv's input
# channels: the decoder-concat counts 40/88/160/168/320), against f64 torch on
# the same bf16/f32 operands, with each shape checked under the odd-width tile
# and under the 64/128-wide tile it replaces (UMAMD_IG_ODD_BN = 0), with the
# 64x64 deep-layer plan switched off so the 128-row plan is taken.
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('case', [(40, 32, 3, 2, 96, 128), (88, 64, 3, 2, 128, 128),
                                  (168, 128, 3, 2, 128, 128), (160, 64, 1, 2, 128, 128),
                                  (320, 256, 3, 2, 64, 96), (72, 32, 1, 2, 128, 160)])
def test_dgrad_odd_tiles(dtype, case):
    from umamd import functional as U
    from umamd._lib import PAD_ZERO, lib
    C, K, R, N, H, W = case
    pad = (R - 1) // 2
    g = torch.Generator().manual_seed(11)
    w = (torch.rand(K, C, R, R, generator=g) - 0.5) * 0.2
    dy = torch.randn(N, K, H, W, generator=g)
    wq = w.to(dtype).double()
    dyq = dy.to(dtype).double()
    ref = torch.nn.grad.conv2d_input((N, C, H, W), wq, dyq, padding=pad)
    _, wT = U._pack(w.to(DEV), C, dtype, wf=False)
    outs = []
    for odd in (1, 0):
        old = lib().um_set_tuning(b'odd_bn', odd)
        old_h = lib().um_set_tuning(b'halo', 0)
        old_s = lib().um_set_tuning(b'small', 0)
        try:
            dx = U._conv_dgrad(_nhwc(dy).to(dtype), wT, (N, H, W, C), K, R, 1, pad, PAD_ZERO)
            torch.cuda.synchronize()
        finally:
            lib().um_set_tuning(b'odd_bn', old)
            lib().um_set_tuning(b'halo', old_h)
            lib().um_set_tuning(b'small', old_s)
        outs.append(_nchw(dx))
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    for o in outs:
        assert _rel(o, ref) < tol, _rel(o, ref)
    assert _rel(outs[0], outs[1]) < tol


# reflect-pad data gradient: the zero-pad transposed conv over all pixels
# (halo / LDS-DMA / register paths) plus the border-list fold GEMM that adds
# the mirrored taps' gradient, against f64 autograd through F.pad(reflect) on
# the same quantised operands; tiny images (every row a fold row), odd widths,
# accumulate into an existing dx
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('case', [
    (48, 32, 3, 2, 32, 64, False),    # halo path (NC <= 64, 8x32 tiles)
    (32, 8, 3, 2, 40, 64, False),     # disparity-head shape (K = 8)
    (168, 128, 3, 2, 16, 32, False),  # 64x64 LDS-DMA tiles
    (88, 64, 3, 2, 24, 40, True),     # 96-wide register tiles, accumulate
    (64, 64, 3, 1, 3, 5, False),      # H = 3: rows 1 and H-2 coincide
    (32, 16, 3, 1, 2, 7, True),       # H = 2: both rows fold
    (320, 256, 3, 2, 8, 16, False),   # split-K
    (88, 64, 3, 2, 8, 64, True),      # split form on the 96-wide halo blocks
])
@pytest.mark.parametrize('border_valu', [0, 2])
def test_dgrad_reflect(dtype, case, border_valu):
    """border_valu: the split form's reflect fold as the VALU border pass
    (2: every shape) or as the register GEMM's border-list mode (0)"""
    from umamd import functional as U
    from umamd._lib import PAD_REFLECT, lib
    C, K, R, N, H, W, accumulate = case
    pad = 1
    g = torch.Generator().manual_seed(5)
    w = (torch.rand(K, C, R, R, generator=g) - 0.5) * 0.2
    dy = torch.randn(N, K, H, W, generator=g)
    dx0 = torch.randn(N, C, H, W, generator=g) if accumulate else None
    wq = w.to(dtype).double()
    dyq = dy.to(dtype).double()
    x = torch.zeros(N, C, H, W, dtype=torch.float64, requires_grad=True)
    y = F.conv2d(F.pad(x, (pad,) * 4, mode='reflect'), wq)
    y.backward(dyq)
    ref = x.grad + (dx0.to(dtype).double() if accumulate else 0)
    _, wT = U._pack(w.to(DEV), C, dtype, wf=False)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    # default plan, the halo kernel wherever it applies, then the one-pass
    # fold, the split form and the padded form (zero-pad transposed conv onto
    # the padded input + reflect fold pass) forced
    for hmin, snc, pd in ((256, 64, 1), (1, 64, 1), (256, 0, 0), (256, 4096, 1), (256, 64, 2),
                          (1, 64, 2)):
        old = lib().um_set_tuning(b'halo_min_tiles', hmin)
        old_s = lib().um_set_tuning(b'fold_split_nc', snc)
        old_p = lib().um_set_tuning(b'pad_dgrad', pd)
        old_b = lib().um_set_tuning(b'border_valu', border_valu)
        try:
            dx = _nhwc(dx0).to(dtype).contiguous() if accumulate else None
            out = U._conv_dgrad(_nhwc(dy).to(dtype), wT, (N, H, W, C), K, R, 1, pad, PAD_REFLECT,
                                dx=dx, accumulate=accumulate)
            torch.cuda.synchronize()
        finally:
            lib().um_set_tuning(b'halo_min_tiles', old)
            lib().um_set_tuning(b'fold_split_nc', old_s)
            lib().um_set_tuning(b'pad_dgrad', old_p)
            lib().um_set_tuning(b'border_valu', old_b)
        err = _rel(_nchw(out), ref)
        print(f'dgrad_reflect {case} {dtype} halo_min_tiles={hmin} fold_split_nc={snc} '
              f'pad_dgrad={pd}: rel {err:.3e}')
        assert err < tol, err


# 64x64 LDS-DMA main loop with 3 stages (several blocks per CU) and with 6
# stages (grids of <= glds_deep_blocks blocks, one 96 KB block per CU), split
# and unsplit, row- and column-major tile order, forward and data gradient,
# against f64 torch on the same bf16 operands
@pytest.mark.parametrize('case', [(256, 256, 3, 2, 16, 32), (128, 128, 3, 8, 16, 32),
                                  (512, 512, 3, 2, 8, 16), (128, 192, 1, 4, 16, 32)])
@pytest.mark.parametrize('deep', [3, 6])
@pytest.mark.parametrize('split_below', [0, 256])
@pytest.mark.parametrize('xcd_col', [0, 2])
def test_glds_stage_depth(case, deep, split_below, xcd_col):
    from umamd import functional as U
    from umamd._lib import PAD_ZERO, lib
    C, K, R, N, H, W = case
    pad = (R - 1) // 2
    dtype = torch.bfloat16
    g = torch.Generator().manual_seed(5)
    w = (torch.rand(K, C, R, R, generator=g) - 0.5) * 0.2
    x = torch.randn(N, C, H, W, generator=g)
    dy = torch.randn(N, K, H, W, generator=g)
    wq, xq, dyq = (t.to(dtype).double() for t in (w, x, dy))
    ref_y = F.conv2d(xq, wq, padding=pad)
    ref_dx = torch.nn.grad.conv2d_input((N, C, H, W), wq, dyq, padding=pad)
    wf, wT = U._pack(w.to(DEV), C, dtype)
    knobs = {b'glds_deep': deep, b'glds_deep_blocks': 1024, b'glds_split_below': split_below,
             b'halo': 0, b'xcd_col': xcd_col}
    old = {k: lib().um_set_tuning(k, v) for k, v in knobs.items()}
    try:
        y = U._conv_fwd(_nhwc(x).to(dtype), wf, None, K, R, 1, pad, PAD_ZERO,
                        out_dtype=torch.float32)
        dx = U._conv_dgrad(_nhwc(dy).to(dtype), wT, (N, H, W, C), K, R, 1, pad, PAD_ZERO)
        torch.cuda.synchronize()
    finally:
        for k, v in old.items():
            lib().um_set_tuning(k, v)
    assert _rel(_nchw(y), ref_y) < 1e-5
    assert _rel(_nchw(dx), ref_dx) < 1e-2


# 8-channel GEMM operands with 4 taps packed per 32-deep k-step (knob
# tappack 3, default) and without (0): the 7x7 stride-2 first conv (C = 8
# after the 3-channel pad), the 8-channel heads' data gradients (zero and
# reflect pad, the reflect fold) and a stride-2 data gradient whose parity
# classes gather 8 channels; forward and data gradient against f64 torch on
# the same quantised operands
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('case', [(8, 32, 7, 2, 'zero', 4, 64, 96), (32, 8, 3, 1, 'reflect', 2, 32, 64),
                                  (128, 8, 3, 1, 'reflect', 2, 16, 24), (16, 8, 3, 2, 'zero', 2, 24, 40),
                                  (24, 8, 5, 1, 'zero', 2, 20, 36)])
@pytest.mark.parametrize('pack', [0, 3])
def test_tappack(dtype, case, pack):
    from umamd import functional as U
    from umamd._lib import PAD_REFLECT, PAD_ZERO, lib
    C, K, R, stride, mode, N, H, W = case
    pad = (R - 1) // 2
    g = torch.Generator().manual_seed(21)
    w = (torch.rand(K, C, R, R, generator=g) - 0.5) * 0.3
    x = torch.randn(N, C, H, W, generator=g)
    wq, xq = w.to(dtype).double(), x.to(dtype).double()
    xr = xq.clone().requires_grad_(True)
    xp = F.pad(xr, (pad,) * 4, mode='reflect' if mode == 'reflect' else 'constant')
    ref_y = F.conv2d(xp, wq, stride=stride)
    dy = torch.randn(ref_y.shape, generator=g)
    dyq = dy.to(dtype).double()
    (ref_y * dyq).sum().backward()
    wf, wT = U._pack(w.to(DEV), C, dtype)
    pm = PAD_REFLECT if mode == 'reflect' else PAD_ZERO
    old = lib().um_set_tuning(b'tappack', pack)
    try:
        y = U._conv_fwd(_nhwc(x).to(dtype), wf, None, K, R, stride, pad, pm,
                        out_dtype=torch.float32)
        dx = U._conv_dgrad(_nhwc(dy).to(dtype), wT, (N, H, W, C), K, R, stride, pad, pm)
        torch.cuda.synchronize()
    finally:
        lib().um_set_tuning(b'tappack', old)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(_nchw(y), ref_y) < 1e-5
    assert _rel(_nchw(dx), xr.grad) < tol


# stride-2 data gradient: the four parity classes in one launch (knob cls4,
# default: LDS-DMA tiles -- 64x64 when C is a multiple of 64, 64x32 when C is
# 32 (cls_glds 3; 1: the 64-multiples only) -- with per-class split-K when K
# is a multiple of 64; else 256-row register tiles), the register form forced
# (cls_glds 0), and as four launches; odd and even image sizes (classes of
# different sizes), both pad parities, 8-channel dy (tap packing), against f64
# torch
@pytest.mark.parametrize('case', [(32, 64, 5, 2, 32, 64), (64, 128, 3, 2, 16, 32),
                                  (16, 32, 3, 2, 15, 21), (48, 8, 3, 2, 18, 26),
                                  (24, 16, 7, 1, 9, 13), (128, 256, 3, 2, 8, 16),
                                  (64, 64, 3, 2, 15, 21), (64, 64, 5, 2, 12, 20),
                                  (256, 512, 3, 8, 16, 32)])
@pytest.mark.parametrize('mode', [(0, 3), (1, 3), (1, 1), (1, 0)])
def test_dgrad_stride2_classes(case, mode):
    from umamd import functional as U
    from umamd._lib import PAD_ZERO, lib
    C, K, R, N, H, W = case
    cls4, glds = mode
    pad = (R - 1) // 2
    dtype = torch.bfloat16
    g = torch.Generator().manual_seed(17)
    w = (torch.rand(K, C, R, R, generator=g) - 0.5) * 0.2
    P = (H + 2 * pad - R) // 2 + 1
    Q = (W + 2 * pad - R) // 2 + 1
    dy = torch.randn(N, K, P, Q, generator=g)
    wq, dyq = w.to(dtype).double(), dy.to(dtype).double()
    ref = torch.nn.grad.conv2d_input((N, C, H, W), wq, dyq, stride=2, padding=pad)
    _, wT = U._pack(w.to(DEV), C, dtype, wf=False)
    old = lib().um_set_tuning(b'cls4', cls4)
    old_g = lib().um_set_tuning(b'cls_glds', glds)
    try:
        dx = U._conv_dgrad(_nhwc(dy).to(dtype), wT, (N, H, W, C), K, R, 2, pad, PAD_ZERO)
        torch.cuda.synchronize()
    finally:
        lib().um_set_tuning(b'cls4', old)
        lib().um_set_tuning(b'cls_glds', old_g)
    assert _rel(_nchw(dx), ref) < 1e-2


@pytest.mark.parametrize('C,H,W', [(32, 16, 32), (64, 8, 16), (256, 4, 8), (96, 3, 5)])
def test_disp_head_split(C, H, W, monkeypatch):
    """The bf16 disparity/uncertainty head as the GEMM with split-bf16
    weights (um_pack_weight_split: hi + lo rows in the padding columns of the
    4-output GEMM), against an f64 reference with the UNROUNDED f32 weights:
    the forward is f32-accurate (the plain bf16 GEMM head is off by the
    weight rounding), and the backward sees the f32 weight."""
    import umamd.functional as U
    N, K, scale = 2, 4, 0.3
    x = F.elu(torch.randn(N, C, H, W)).to(torch.bfloat16).float()
    conv = nn.Conv2d(C, K, 3)
    nn.init.xavier_uniform_(conv.weight)
    conv.bias.data.uniform_(-0.5, 0.5)
    conv = conv.to(DEV)
    dd = torch.randn(N, K, H, W)

    def ref():
        xr = x.double().requires_grad_(True)
        wr = conv.weight.detach().double().cpu().requires_grad_(True)
        z = F.conv2d(F.pad(xr, (1, 1, 1, 1), mode='reflect'), wr,
                     conv.bias.detach().double().cpu())
        d = scale * torch.sigmoid(z)
        d.backward(dd.double())
        return d.detach(), xr.grad, wr.grad

    def run(split):
        monkeypatch.setattr(U, '_SPLIT_HEAD', split)
        xd = _nhwc(x).to(torch.bfloat16)
        Cp = (C + 7) // 8 * 8
        if Cp != C:
            xd = F.pad(xd, (0, Cp - C))
        xd.requires_grad_(True)
        conv.weight.grad = None
        d = U.disp_head(xd, conv, scale)
        d.backward(_nhwc(dd))
        return _nchw(d), _nchw(xd.grad)[:, :C], conv.weight.grad.cpu()

    d_ref, dx_ref, dw_ref = ref()
    d_s, dx_s, dw_s = run(True)
    d_p, dx_p, dw_p = run(False)
    e_s, e_p = _rel(d_s, d_ref), _rel(d_p, d_ref)
    assert e_s <= 2e-5, (e_s, e_p)
    assert e_s < e_p, (e_s, e_p)
    # backward: dlogit is bf16 in both, the split one sees the f32 weight
    assert _rel(dx_s, dx_ref) <= 1e-2, _rel(dx_s, dx_ref)
    assert _rel(dw_s, dw_ref) <= 1e-2, _rel(dw_s, dw_ref)
    assert _rel(dx_s, dx_ref) <= _rel(dx_p, dx_ref) * 1.5 + 1e-4


@pytest.mark.parametrize('C,H,W', [(32, 16, 32), (64, 8, 16), (128, 4, 48), (256, 6, 16),
                                   (32, 32, 64), (32, 12, 16), (64, 6, 32), (64, 4, 16)])
def test_disp_head_onepass(C, H, W, monkeypatch):
    """The one-pass head kernels (csrc/disphead.hip: strip MFMA with direct
    operand loads, the reflect adjoint folded into the dlogit load) against
    the f64 reference with the unrounded weights, and against the
    implicit-GEMM head path (UMAMD_ONEPASS_HEAD=0) on the same inputs; the
    data gradient's accumulate mode through the C entry.  Shapes cover
    W = 16 (the border columns 1 and W-2 in one strip) and H = 4 (mirror
    rows 1 and H-2 adjacent)."""
    import umamd.functional as U
    from umamd._lib import call, ptr, query
    N, K, scale = 2, 4, 0.3
    assert query('um_disp_head_ok', N, H, W, C, C) == 1
    torch.manual_seed(C + H + W)
    x = F.elu(torch.randn(N, C, H, W)).to(torch.bfloat16).float()
    conv = nn.Conv2d(C, K, 3)
    nn.init.xavier_uniform_(conv.weight)
    conv.bias.data.uniform_(-0.5, 0.5)
    conv = conv.to(DEV)
    dd = torch.randn(N, K, H, W)

    xr = x.double().requires_grad_(True)
    z = F.conv2d(F.pad(xr, (1, 1, 1, 1), mode='reflect'), conv.weight.detach().double().cpu(),
                 conv.bias.detach().double().cpu())
    d_ref = scale * torch.sigmoid(z)
    d_ref.backward(dd.double())

    def run(onepass):
        monkeypatch.setattr(U, '_ONEPASS_HEAD', onepass)
        xd = _nhwc(x).to(torch.bfloat16).requires_grad_(True)
        conv.weight.grad = None
        d = U.disp_head(xd, conv, scale)
        d.backward(_nhwc(dd))
        return _nchw(d), _nchw(xd.grad), conv.weight.grad.cpu()

    d_o, dx_o, dw_o = run(True)
    d_g, dx_g, dw_g = run(False)
    assert _rel(d_o, d_ref.detach()) <= 2e-5, _rel(d_o, d_ref.detach())
    assert _rel(d_o, d_g) <= 2e-5
    assert _rel(dx_o, xr.grad) <= 1e-2, _rel(dx_o, xr.grad)
    # the GEMM path rounds the same bf16 dlogit; the two differ by the bf16
    # rounding of dx (1-2 ulp at the max: <= 8e-3) and the border-pixel
    # mirror sums (f32 sum -> bf16 operand): no worse against the reference
    assert _rel(dx_o, dx_g) <= 8e-3, _rel(dx_o, dx_g)
    assert _rel(dx_o, xr.grad) <= 1.25 * _rel(dx_g, xr.grad) + 1e-3
    assert _rel(dw_o, dw_g) <= 1e-6

    # accumulate: dx += adjoint(dlogit), straight through the C entry
    wf, wT = U._pack(conv.weight, C, torch.bfloat16, ldT=8, split=True)
    dl = torch.randn(N, H, W, 8, device=DEV).to(torch.bfloat16)
    base = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
    d0 = torch.empty_like(base)
    call('um_disp_head_dgrad', N, H, W, C, ptr(dl), 8, ptr(wT), ptr(d0), C, 0)
    d1 = base.clone()
    call('um_disp_head_dgrad', N, H, W, C, ptr(dl), 8, ptr(wT), ptr(d1), C, 1)
    torch.cuda.synchronize()
    assert _rel(d1.float(), base.float() + d0.float()) <= 5e-3


@pytest.mark.parametrize('case', [CONV_CASES[1], CONV_CASES[3], CONV_CASES[7], CONV_CASES[4]])
def test_conv_bn_elu_ybf16(case, monkeypatch):
    """bf16 activations with the pre-BN y stored in bf16 (UM_Y_ACT, the
    UMAMD_Y_ACT=1 build): two training steps on the same input, outputs,
    gradients and the running statistics after both updates against the
    fp32 CPU reference."""
    from umamd import functional as U
    from umamd._lib import PAD_REFLECT, PAD_ZERO
    monkeypatch.setattr(U, '_Y_ACT', True)
    Cin, Cout, k, stride, mode, H, W = case
    N, pad = 2, (k - 1) // 2
    conv, bn = nn.Conv2d(Cin, Cout, k, stride), nn.BatchNorm2d(Cout)
    with torch.no_grad():
        conv.bias.uniform_(2.0, 4.0)  # a large mean: the bf16 y's worst case
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    x = torch.randn(N, Cin, H, W) + 1.0
    cr, br = nn.Conv2d(Cin, Cout, k, stride), nn.BatchNorm2d(Cout)
    cr.load_state_dict(conv.state_dict())
    br.load_state_dict(bn.state_dict())
    cd, bd = conv.to(DEV), bn.to(DEV)
    xq = _nhwc(x).to(torch.bfloat16)
    xs = _nchw(xq)  # the reference sees the same bf16-rounded input
    for step in range(2):
        xr = xs.clone().requires_grad_(True)
        xp = F.pad(xr, (pad,) * 4, mode='reflect' if mode == 'reflect' else 'constant')
        yr = F.elu(br(cr(xp)))
        g = torch.randn_like(yr)
        cr.zero_grad()
        br.zero_grad()
        (yr * g).sum().backward()
        xd = xq.clone().requires_grad_(True)
        cd.zero_grad()
        bd.zero_grad()
        with U.stat_scope(U.StatArena(), DEV):
            yd = U.conv_bn_elu(xd, cd, bd, pad, PAD_REFLECT if mode == 'reflect' else PAD_ZERO)
        (yd.float() * _nhwc(g)).sum().backward()
        assert _rel(_nchw(yd), yr) < 5e-2, step
        assert _rel(_nchw(xd.grad), xr.grad) < 2.5e-1, step
        assert _rel(cd.weight.grad, cr.weight.grad) < 2.5e-1, step
        assert _rel(bd.weight.grad, br.weight.grad) < 2.5e-1, step
    assert _rel(bd.running_mean, br.running_mean) < 1e-3
    assert _rel(bd.running_var, br.running_var) < 2e-2


# the streaming 1x1 kernel (stream1x1.hip, tuning key s1x1) against the
# 256-row GEMM tiles it replaces (s1x1 = 0) and f64 torch on the same bf16
# operands: bias / residual (the attention's 1x1 convs), f32 output (the skip
# conv's z map), accumulate onto up2(z) with the BN statistics slots of the
# sum (the skip conv's feature-map half) and the data gradient with
# accumulate; ragged pixel counts and reduction widths padded to 32/64/128
@pytest.mark.parametrize('case', [(2, 64, 128, 32, 96, 'bias'), (2, 64, 128, 32, 32, 'residual'),
                                  (1, 129, 131, 64, 32, 'f32'), (2, 64, 128, 32, 64, 'up2stats'),
                                  (1, 129, 131, 96, 32, 'dgrad'), (2, 64, 128, 64, 192, 'bias'),
                                  (1, 128, 130, 192, 64, 'dgrad'), (2, 64, 128, 128, 128, 'up2stats')])
def test_stream1x1(case):
    _check_1x1(case, b's1x1')


# the small-M 1x1 kernel (stream1x1.hip s1x1_small_kernel, tuning key
# s1x1_small, M in [256, 16384) pixels) against the GEMM tiles it replaces and
# f64 torch: the deep layers' shapes (attention K/Q/V and reprojection at
# 8x16 .. 32x64, C up to 512 = 16 k-steps held in registers), ragged pixel
# counts, reduction widths padded to the next power-of-two k-step count, the
# same epilogues; M < 256 stays on the GEMM (both arms)
@pytest.mark.parametrize('case', [(2, 16, 32, 256, 512, 'bias'), (2, 16, 32, 512, 256, 'residual'),
                                  (1, 33, 35, 64, 32, 'f32'), (2, 32, 64, 128, 64, 'up2stats'),
                                  (1, 31, 33, 96, 32, 'dgrad'), (2, 8, 16, 512, 512, 'dgrad'),
                                  (2, 16, 32, 320, 64, 'bias'), (1, 8, 16, 64, 32, 'bias'),
                                  (1, 62, 64, 256, 512, 'up2stats'), (2, 8, 32, 512, 48, 'residual')])
def test_s1x1_small(case):
    _check_1x1(case, b's1x1_small')


def _check_1x1(case, key):
    from umamd import functional as U
    from umamd import _lib as L
    from umamd._lib import PAD_ZERO, call, lib, ptr
    N, H, W, C, K, mode = case
    g = torch.Generator().manual_seed(11)
    x = (torch.rand(N, H, W, C, generator=g) - 0.3).to(torch.bfloat16).to(DEV)
    wt = (torch.randn(K, C, 1, 1, generator=g) / C ** 0.5).to(DEV)
    bias = torch.randn(K, generator=g).to(DEV)
    res = torch.randn(N, H, W, K, generator=g).to(torch.bfloat16).to(DEV)
    prev = torch.randn(N, H, W, C, generator=g).to(torch.bfloat16).to(DEV)
    h, w = H // 2, W // 2
    z = torch.randn(N, h, w, K, generator=g).to(DEV)
    wq = wt.to(torch.bfloat16).double()[:, :, 0, 0]

    def run():
        wf, _ = U._pack(wt, C, torch.bfloat16)
        if mode == 'up2stats':
            y = torch.empty(N, H, W, K, dtype=torch.float32, device=DEV)
            slots = torch.zeros(L.STAT_SLOTS * K * 2 + 1, dtype=torch.float64, device=DEV)
            call('um_conv2d_fwd_up2', L.UM_BF16, N, H, W, C, C, ptr(x), ptr(wf), ptr(bias), K, H,
                 W, ptr(y), K, L.EPI_STAT_SLOTS, ptr(slots), ptr(z), h, w, K)
            return y, slots
        if mode == 'residual':
            return U._conv_fwd(x, wf, bias, K, 1, 1, 0, PAD_ZERO, epi=L.EPI_RESIDUAL,
                               residual=res), None
        if mode == 'f32':
            return U._conv_fwd(x, wf, None, K, 1, 1, 0, PAD_ZERO, out_dtype=torch.float32), None
        return U._conv_fwd(x, wf, bias, K, 1, 1, 0, PAD_ZERO), None

    if mode == 'dgrad':
        # dx (C' = K channels) += dy (C channels) . W^T with W [C][K]: a K -> C conv's
        # input gradient; dgrad of (dy: C ch) through wT packed from a [C, K] weight
        wfw = (torch.randn(C, K, 1, 1, generator=g) / K ** 0.5).to(DEV)
        _, wTd = U._pack(wfw, K, torch.bfloat16)
        outs = []
        for flag in (1, 0):
            old = lib().um_set_tuning(key, flag)
            try:
                dx = prev[..., :K].contiguous().clone()
                U._conv_dgrad(x, wTd, (N, H, W, K), C, 1, 1, 0, PAD_ZERO, dx=dx, accumulate=True)
                torch.cuda.synchronize()
            finally:
                lib().um_set_tuning(key, old)
            outs.append(dx.double())
        ref = prev[..., :K].double() + torch.einsum('nhwc,ck->nhwk', x.double(),
                                                    wfw.to(torch.bfloat16).double()[:, :, 0, 0])
        assert _rel(outs[0], ref) < 1e-2 and _rel(outs[0], outs[1]) < 1e-2
        return
    outs = []
    for flag in (1, 0):
        old = lib().um_set_tuning(key, flag)
        try:
            outs.append(run())
            torch.cuda.synchronize()
        finally:
            lib().um_set_tuning(key, old)
    ref = torch.einsum('nhwc,kc->nhwk', x.double(), wq)
    if mode != 'f32':
        ref = ref + bias.double()
    if mode == 'residual':
        ref = ref + res.double()
    if mode == 'up2stats':
        ref = ref + F.interpolate(z.double().permute(0, 3, 1, 2), scale_factor=2,
                                  mode='bilinear', align_corners=True).permute(0, 2, 3, 1)
    (y1, s1), (y0, s0) = outs
    tol = 1e-2 if y1.dtype == torch.bfloat16 else 1e-5
    assert _rel(y1.double(), ref) < tol and _rel(y1.double(), y0.double()) < tol
    if mode == 'up2stats':
        st1 = s1[:L.STAT_SLOTS * K * 2].view(L.STAT_SLOTS, K, 2).sum(0)
        st0 = s0[:L.STAT_SLOTS * K * 2].view(L.STAT_SLOTS, K, 2).sum(0)
        e1, e2 = ref.sum(dim=(0, 1, 2)), (ref * ref).sum(dim=(0, 1, 2))
        assert float(((st1[:, 0] - e1).abs() / ref.abs().sum(dim=(0, 1, 2))).max()) < 1e-4
        assert float(((st1[:, 1] - e2).abs() / e2).max()) < 1e-4
        assert torch.allclose(st1, st0, rtol=1e-5, atol=1e-3)
        assert float(s1[-1]) == N * H * W
