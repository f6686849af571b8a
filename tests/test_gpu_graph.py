"""Whole-step HIP graph capture (train/graph.py) against the eager step.

Same initial weights, same inputs: W eager warm-up steps + K graph replays
must track W + K eager steps (losses per step and final parameters, l1 loss
so later steps stay well conditioned).  The runs differ only by float-atomic
summation order in the loss backward; Adam turns that into sign noise on
near-zero gradients, so two EAGER runs already drift apart: measured on
MI355X, 5e-5 rel on the loss at step 3 and 1e-3..4e-3 by steps 5-8.
So the check is per step from a shared state: the eager step starts from an
exact copy of the captured run's weights, BN stats and Adam moments/step."""
import pytest
import torch

from test_gpu_model import DEV, _cfg, _model, _uniform_pair

pytestmark = pytest.mark.gpu


def _adam_clone(opt_src, m_src, m_dst):
    """Adam for m_dst holding a copy of opt_src's state (moments + step)."""
    from umamd.optim import Adam
    opt = Adam(m_dst.parameters(), opt_src.param_groups[0]['lr'])
    for ps, pd in zip(m_src.parameters(), m_dst.parameters()):
        st = opt_src.state[ps]
        opt.state[pd] = {'exp_avg': st['exp_avg'].clone(), 'exp_avg_sq': st['exp_avg_sq'].clone()}
    ds = opt._device_state(0, opt.param_groups[0], next(m_dst.parameters()).device)
    ds['step'].copy_(opt_src._dev[0]['step'])
    return opt


@pytest.mark.parametrize('dtype', ['fp32', 'bf16'])
def test_captured_step_matches_eager(dtype):
    from train.graph import CapturedTrainStep
    from train.loss import TukraUncertaintyLoss
    from train.train import train_step
    cfg = _cfg()
    cfg['loss']['error_loss_config']['loss_type'] = 'l1'
    left, right = _uniform_pair(2, 64, 128)
    left, right = left.to(DEV), right.to(DEV)
    lf = TukraUncertaintyLoss(**cfg['loss'])
    from umamd.optim import Adam

    m_g = _model(cfg, dtype).train()
    opt_g = Adam(m_g.parameters(), 1e-4)
    cap = CapturedTrainStep(m_g, lf, opt_g, left, right, 0.3, warmup=2)
    for _ in range(2):
        cap()
    torch.cuda.synchronize()
    # eager step from an exact copy of the graph's current state
    m_e = _model(cfg, dtype).train()
    m_e.load_state_dict(m_g.state_dict())
    opt_e = _adam_clone(opt_g, m_g, m_e)
    dl_e, el_e, _ = train_step(m_e, left, right, lf, opt_e, 0.3)
    dl_g, el_g = cap()
    torch.cuda.synchronize()
    # same parameters in: the losses agree to summation order
    for a, b in ((float(dl_e), float(dl_g)), (float(el_e), float(el_g))):
        assert abs(a - b) <= 1e-5 * abs(a) + 1e-7, (a, b)
    # warm-up updates are undone at capture (restore_state): 3 replays
    assert int(opt_g._dev[0]['step']) == int(opt_e._dev[0]['step']) == 3
    se, sg = m_e.state_dict(), m_g.state_dict()
    pnames = {k for k, _ in m_e.named_parameters()}
    for k in se:
        if k in pnames:
            # one Adam step from equal state: |update| <~ 3 lr, and gradient
            # sign noise on near-zero gradients can flip it
            d = float((se[k] - sg[k]).abs().max())
            assert d <= 6e-4, (k, d)
        elif se[k].is_floating_point():  # running stats: same forward
            d = float((se[k] - sg[k]).abs().max())
            assert d <= 1e-4 * (float(se[k].abs().max()) + 1.0), (k, d)
        else:
            assert torch.equal(se[k], sg[k]), k


def test_capture_restores_pre_warmup_state():
    """CapturedTrainStep's eager warm-up steps are undone after capture: the
    weights, BN buffers and Adam state equal the initial ones, and the first
    replay matches one eager step from that initial state."""
    from train.graph import CapturedTrainStep
    from train.loss import TukraUncertaintyLoss
    from train.train import train_step
    from umamd.optim import Adam
    cfg = _cfg()
    cfg['loss']['error_loss_config']['loss_type'] = 'l1'
    left, right = _uniform_pair(2, 64, 128)
    left, right = left.to(DEV), right.to(DEV)
    lf = TukraUncertaintyLoss(**cfg['loss'])
    m_g = _model(cfg).train()
    init = {k: v.clone() for k, v in m_g.state_dict().items()}
    opt_g = Adam(m_g.parameters(), 1e-4)
    cap = CapturedTrainStep(m_g, lf, opt_g, left, right, 0.3, warmup=2)
    for k, v in m_g.state_dict().items():
        assert torch.equal(v, init[k]), k
    assert int(opt_g._dev[0]['step']) == 0
    assert all(float(st['exp_avg'].abs().max()) == 0 for st in opt_g.state.values())
    dl_g, el_g = cap()
    m_e = _model(cfg).train()
    opt_e = Adam(m_e.parameters(), 1e-4)
    dl_e, el_e, _ = train_step(m_e, left, right, lf, opt_e, 0.3)
    torch.cuda.synchronize()
    for a, b in ((float(dl_e), float(dl_g)), (float(el_e), float(el_g))):
        assert abs(a - b) <= 1e-5 * abs(a) + 1e-7, (a, b)


def test_set_lr_reaches_graph():
    from train.graph import CapturedTrainStep
    from train.loss import TukraUncertaintyLoss
    from umamd.optim import Adam
    cfg = _cfg()
    cfg['loss']['error_loss_config']['loss_type'] = 'l1'
    left, right = _uniform_pair(2, 64, 128)
    m = _model(cfg).train()
    opt = Adam(m.parameters(), 1e-4)
    cap = CapturedTrainStep(m, TukraUncertaintyLoss(**cfg['loss']), opt, left.to(DEV),
                            right.to(DEV), 0.3, warmup=1)
    opt.set_lr(0.0)
    before = {k: v.clone() for k, v in m.state_dict().items() if k.endswith('weight')}
    cap()
    torch.cuda.synchronize()
    after = m.state_dict()
    for k, v in before.items():
        assert torch.equal(v, after[k]), k  # lr 0: Adam leaves weights unchanged


@pytest.mark.parametrize('dtype', ['fp32', 'bf16'])
def test_wgrad_side_stream_matches_single_stream(dtype):
    """umamd.overlap.WgradStream (weight gradients on a side stream, joined
    at the end of backward) gives the same gradients as the one-stream
    backward from the same state; only the loss backward's float-atomic
    summation order differs between two runs."""
    from train.loss import TukraUncertaintyLoss
    import train.utils as u
    from umamd.overlap import WgradStream
    cfg = _cfg()
    left, right = _uniform_pair(2, 64, 128)
    left, right = left.to(DEV), right.to(DEV)
    lf = TukraUncertaintyLoss(**cfg['loss'])
    m = _model(cfg, dtype).train()
    named = [(k, p) for k, p in m.named_parameters() if p.requires_grad]
    params = [p for _, p in named]
    ov = WgradStream(params)
    grads = []
    for use in (False, True):
        for p in params:
            p.grad = None
        pyr = u.scale_pyramid(torch.cat([left, right], 1), 4)
        d = m(left, 0.3)
        dl, el = lf(pyr, d, u.reconstruct_pyramid(d, pyr), 0, None)
        if use:
            with ov:
                (dl + el).backward()
        else:
            (dl + el).backward()
        torch.cuda.synchronize()
        grads.append([p.grad.detach().clone() for p in params])
    for (k, _), a, b in zip(named, grads[0], grads[1]):
        d = float((a - b).norm())
        assert d <= 1e-3 * float(a.norm()) + 1e-5, (k, d, float(a.norm()))
    for p in params:
        p.grad = torch.zeros_like(p)
    with pytest.raises(RuntimeError):
        with ov:
            pass


def _ddp_one_rank(monkeypatch, bucket_mb=None, captures=1):
    """The data-parallel captured step (DDP wrapper, SyncBN statistics and
    the packed gradient all-reduce recorded in the graph as RCCL nodes) on a
    one-rank 'nccl' group -- the only RCCL group a 1-GPU box can form: it
    captures (``captures`` times in a row, each new capture closing the last,
    as train_model does on a scale change; no wait for the process group's
    watchdog in between), replays, leaves .grad as views of the reduced
    buffer and tracks the single-process eager step (at world 1 the average
    is the identity)."""
    import socket
    import torch.distributed as dist
    from train.graph import CapturedTrainStep
    from train.loss import TukraUncertaintyLoss
    from train.parallel import data_parallel, unwrap
    from train.train import train_step
    from umamd.functional import BNSync
    from umamd.optim import Adam
    if bucket_mb is not None:
        monkeypatch.setenv('UMAMD_GRAD_BUCKET_MB', str(bucket_mb))
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0,
                            world_size=1)
    BNSync.force = True
    try:
        cfg = _cfg()
        cfg['loss']['error_loss_config']['loss_type'] = 'l1'
        left, right = _uniform_pair(2, 64, 128)
        left, right = left.to(DEV), right.to(DEV)
        lf = TukraUncertaintyLoss(**cfg['loss'])
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):  # DDP under the capture stream
            m_g = data_parallel(_model(cfg).train(), 0)
        torch.cuda.current_stream().wait_stream(st)
        opt_g = Adam(m_g.parameters(), 1e-4)
        cap = None
        for _ in range(captures):
            if cap is not None:
                cap.close()
            cap = CapturedTrainStep(m_g, lf, opt_g, left, right, 0.3, warmup=1, stream=st)
        assert cap.group is not None and cap.world == 1
        if bucket_mb is not None:
            # every parameter its own bucket: the attention's K/V gradients
            # (views into the fused QKV weight gradient) sit in buckets apart
            assert len(cap._buckets.buckets) == sum(cap._buckets.layout)
        for _ in range(2):
            cap()
        torch.cuda.synchronize()
        lo = cap._flat.data_ptr()
        hi = lo + cap._flat.numel() * 4
        for p in unwrap(m_g).parameters():
            assert lo <= p.grad.data_ptr() < hi
        m_e = _model(cfg).train()
        m_e.load_state_dict(unwrap(m_g).state_dict())
        opt_e = _adam_clone(opt_g, unwrap(m_g), m_e)
        dl_e, el_e, _ = train_step(m_e, left, right, lf, opt_e, 0.3)
        dl_g, el_g = cap()
        torch.cuda.synchronize()
        for a, b in ((float(dl_e), float(dl_g)), (float(el_e), float(el_g))):
            assert abs(a - b) <= 1e-5 * abs(a) + 1e-7, (a, b)
        ge = {k: p.grad for k, p in m_e.named_parameters()}
        bad = []
        for k, p in unwrap(m_g).named_parameters():
            d = float((p.grad - ge[k]).norm())
            if not d <= 1e-3 * float(ge[k].norm()) + 1e-5:
                bad.append((k, d, float(ge[k].norm()), float(p.grad.norm())))
        assert not bad, (len(bad), bad[:12])
    finally:
        BNSync.force = False
        dist.destroy_process_group()


def test_captured_ddp_step_one_rank(monkeypatch):
    _ddp_one_rank(monkeypatch)


def test_captured_ddp_tiny_buckets(monkeypatch):
    """Buckets of one parameter each (a bucket boundary between the
    attention's query/key/value gradients, which are views into one deferred
    weight-gradient output: umamd.overlap.WgradStream.is_pending must see
    them by address range)."""
    _ddp_one_rank(monkeypatch, bucket_mb=1e-6)


def test_captured_ddp_recapture(monkeypatch):
    """Three captures back to back, each closing the last (train_model's
    recapture on a disparity-scale change), with no wait in between."""
    _ddp_one_rank(monkeypatch, captures=3)


@pytest.mark.parametrize('cfgname', ['config.yml', 'config_nodes10.yml'])
@pytest.mark.parametrize('dtype', ['fp32', 'bf16'])
def test_stage_fn_matches_per_node_autograd(cfgname, dtype):
    """GraphBlockFn (each GraphBlock one autograd node; node input gradients
    accumulated straight into the predecessors' buffers) against the
    per-node autograd path (MergeFn + ConvBNELUFn, autograd summing the
    fan-out gradients): same forward, gradients equal up to summation order.
    nodes=10 graphs cover several input and output nodes per stage."""
    import train.utils as u
    from train.loss import TukraUncertaintyLoss
    from umamd import functional as U
    cfg = _cfg(cfgname)
    cfg['loss']['error_loss_config']['loss_type'] = 'bayesian'
    left, right = _uniform_pair(2, 64, 128, seed=3)
    left, right = left.to(DEV), right.to(DEV)
    pyr = u.scale_pyramid(torch.cat([left, right], 1), 4)
    res = []
    old = U._STAGE_FN
    try:
        for flag in (True, False):
            U._STAGE_FN = flag
            m = _model(cfg, dtype).train()
            lf = TukraUncertaintyLoss(**cfg['loss'])
            d = m(left, 0.3)
            dl, el = lf(pyr, d, u.reconstruct_pyramid(d, pyr), 0, None)
            (dl + el).backward()
            torch.cuda.synchronize()
            res.append((float(dl), float(el), {k: p.grad.detach().clone()
                                               for k, p in m.named_parameters()},
                        {k: v.detach().clone() for k, v in m.state_dict().items()
                         if 'running' in k}))
    finally:
        U._STAGE_FN = old
    (dl1, el1, g1, b1), (dl0, el0, g0, b0) = res
    assert abs(dl1 - dl0) <= 1e-6 * abs(dl0) and abs(el1 - el0) <= 1e-6 * abs(el0)
    from _parity import atol_of, pre_bn_bias
    # bf16: the node gradients are bf16 buffers summed in another order (GEMM
    # epilogue / merge accumulate vs autograd adds), each sum rounded: node 0
    # of a K5 stage takes 4 contributions (measured up to 2.6e-2 on its BN bias)
    tol = 1e-4 if dtype == 'fp32' else 5e-2
    for k in g0:
        if pre_bn_bias(k):  # true gradient 0: summation noise only
            continue
        if dtype == 'bf16' and not ('node_blocks' in k and k.endswith('.weight')):
            # bf16: sums over whole maps whose true value is small next to
            # their terms (merge weights: a ~1e-3 dot of 2M terms of size ~1,
            # measured |g| 0.2 either way; biases) are noise-dominated in
            # both paths; the GraphBlock's conv and BN weights are compared
            continue
        d = float((g1[k] - g0[k]).norm())
        # merge-weight gradients: whole-map sums with heavy cancellation (the
        # per-element floor of the parity tests)
        assert d <= tol * float(g0[k].norm()) + g0[k].numel() ** 0.5 * atol_of(k), \
            (k, d, float(g0[k].norm()))
    for k in b0:
        assert torch.allclose(b1[k], b0[k], rtol=1e-6, atol=1e-7), k


@pytest.mark.parametrize('dtype', ['fp32', 'bf16'])
def test_fused_merge_matches_separate_merge(dtype):
    """A node's merge computed inside its last predecessor's BN apply pass
    (um_bn_elu_fwd_slots_merge) against the separate um_merge_fwd launch:
    same coefficients, same source order, the stored (rounded) activation of
    the fusing layer -> bit-identical disparities and gradients."""
    from umamd import functional as U
    cfg = _cfg('config.yml')
    left, _ = _uniform_pair(2, 64, 128, seed=5)
    left = left.to(DEV)
    res = []
    old = U._FUSED_MERGE
    try:
        for flag in (True, False):
            U._FUSED_MERGE = flag
            m = _model(cfg, dtype).train()
            d = m(left, 0.3)
            (sum((t.float() ** 2).mean() for t in d)).backward()
            torch.cuda.synchronize()
            res.append(([t.detach().clone() for t in d],
                        {k: p.grad.detach().clone() for k, p in m.named_parameters()}))
    finally:
        U._FUSED_MERGE = old
    (d1, g1), (d0, g0) = res
    for a, b in zip(d1, d0):
        assert torch.equal(a, b)
    for k in g0:
        assert torch.equal(g1[k], g0[k]), k


@pytest.mark.parametrize('dtype', ['fp32', 'bf16'])
def test_merge_bn_reduce_matches_separate_reduce(dtype):
    """A GraphBlock node's BN-backward sums taken by the merge backward that
    completes its gradient (um_merge_bwd_bn) against the separate
    um_bn_elu_bwd_reduce_slots launch: the same sums over the same stored
    gradient, in another partial-sum order -> equal disparities, gradients
    within f32 summation noise."""
    from umamd import functional as U
    cfg = _cfg('config.yml')
    left, _ = _uniform_pair(2, 64, 128, seed=7)
    left = left.to(DEV)
    res = []
    old = U._MERGE_BN_REDUCE
    calls = []
    orig = U._merge_bn_target

    def spy(*args):
        r = orig(*args)
        calls.append(r is not None)
        return r
    U._merge_bn_target = spy
    try:
        for flag in (True, False):
            U._MERGE_BN_REDUCE = flag
            m = _model(cfg, dtype).train()
            d = m(left, 0.3)
            (sum((t.float() ** 2).mean() for t in d)).backward()
            torch.cuda.synchronize()
            res.append(([t.detach().clone() for t in d],
                        {k: p.grad.detach().clone() for k, p in m.named_parameters()}))
    finally:
        U._MERGE_BN_REDUCE = old
        U._merge_bn_target = orig
    assert sum(calls) >= 10, calls  # nodes 1-3 of each of the 5 stages
    (d1, g1), (d0, g0) = res
    for a, b in zip(d1, d0):
        assert torch.equal(a, b)
    # the conv weights, as test_grad_slots_match_autograd_sums: the biases in
    # front of a training-mode BN have a gradient that is zero up to summation
    # noise (closed form, sum of x-hat = 0), and the merge weights' gradients
    # are stage-wide dot products of near-cancelling terms (fp32 1.2e-4; in
    # bf16 one rounding flip of dy moves them by O(1) of their size)
    tol = 1e-4 if dtype == 'fp32' else 5e-2
    keys = [k for k in g0 if k.endswith('.weight') and g0[k].dim() == 4]
    worst = max((float((g1[k] - g0[k]).norm() / g0[k].norm()), k) for k in keys)
    print('merge-BN reduce worst rel', worst)
    assert worst[0] < tol, worst


@pytest.mark.parametrize('dtype', ['fp32', 'bf16'])
def test_grad_slots_match_autograd_sums(dtype):
    """Fan-out input gradients accumulated into one shared buffer by the
    registered consumers (umamd.functional.GradSlots) against autograd
    summing each consumer's own gradient: same losses; gradients equal up to
    the summation order of the fan-out sums (fp32 1e-5, bf16 5e-2 rel-norm on
    the conv weights, as test_stage_fn_matches_per_node_autograd)."""
    import train.utils as u
    from train.loss import TukraUncertaintyLoss
    from umamd import functional as U
    from _parity import atol_of, pre_bn_bias
    cfg = _cfg('config.yml')
    cfg['loss']['error_loss_config']['loss_type'] = 'bayesian'
    left, right = _uniform_pair(2, 64, 128, seed=9)
    left, right = left.to(DEV), right.to(DEV)
    pyr = u.scale_pyramid(torch.cat([left, right], 1), 4)
    res = []
    old = U._GRAD_SLOTS
    try:
        for flag in (True, False):
            U._GRAD_SLOTS = flag
            m = _model(cfg, dtype).train()
            lf = TukraUncertaintyLoss(**cfg['loss'])
            d = m(left, 0.3)
            dl, el = lf(pyr, d, u.reconstruct_pyramid(d, pyr), 0, None)
            (dl + el).backward()
            torch.cuda.synchronize()
            res.append((float(dl), float(el),
                        {k: p.grad.detach().clone() for k, p in m.named_parameters()}))
    finally:
        U._GRAD_SLOTS = old
    (dl1, el1, g1), (dl0, el0, g0) = res
    assert dl1 == dl0 and el1 == el0
    tol = 1e-5 if dtype == 'fp32' else 5e-2
    for k in g0:
        if pre_bn_bias(k) or (dtype == 'bf16' and not k.endswith('.weight')):
            continue
        d = float((g1[k] - g0[k]).norm())
        # + the per-element floor of whole-map sums with heavy cancellation
        # (merge weights: ~1e-5 true value, summation-order noise of the same size)
        assert d <= tol * float(g0[k].norm()) + g0[k].numel() ** 0.5 * atol_of(k), \
            (k, d, float(g0[k].norm()))


def test_grad_slots_guard_unregistered_consumer(monkeypatch):
    """GradSlots' guard: an activation with two registered (umamd) consumers
    AND a consumer outside them (here a plain torch sum) would lose gradient
    terms silently; the pooled tensor's gradient hook raises instead and
    turns pooling off, and the next step (autograd's own sums) gives the
    gradient of the reference composition."""
    import torch.nn as nn
    from umamd import functional as U
    from umamd._lib import PAD_ZERO
    monkeypatch.setattr(U.GradSlots, 'broken', False)
    torch.manual_seed(0)
    c1, b1 = nn.Conv2d(16, 16, 3).to(DEV), nn.BatchNorm2d(16).to(DEV)
    c2, b2 = nn.Conv2d(16, 16, 3).to(DEV), nn.BatchNorm2d(16).to(DEV)
    x0 = torch.randn(2, 8, 16, 16, device=DEV)

    def step():
        x = x0.clone().requires_grad_(True)
        with U.stat_scope(U.StatArena(), DEV), U.grad_slots():
            y1 = U.conv_bn_elu(x, c1, b1, 1, PAD_ZERO)
            y2 = U.conv_bn_elu(x, c2, b2, 1, PAD_ZERO)  # x: two registered uses
        loss = y1.sum() + 2 * y2.sum() + 3 * (x * x).sum()  # + an unregistered use
        loss.backward()
        torch.cuda.synchronize()
        return x.grad

    with pytest.raises(RuntimeError, match='GradSlots'):
        step()
    assert U.GradSlots.broken
    got = step()  # pooling off: autograd sums every consumer
    monkeypatch.setattr(U, '_GRAD_SLOTS', False)
    ref = step()
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-6)
    # and without the outside consumer the pooled path is silent and exact
    monkeypatch.setattr(U.GradSlots, 'broken', False)
    monkeypatch.setattr(U, '_GRAD_SLOTS', True)
    x = x0.clone().requires_grad_(True)
    with U.stat_scope(U.StatArena(), DEV), U.grad_slots():
        y1 = U.conv_bn_elu(x, c1, b1, 1, PAD_ZERO)
        y2 = U.conv_bn_elu(x, c2, b2, 1, PAD_ZERO)
    (y1.sum() + 2 * y2.sum()).backward()
    torch.cuda.synchronize()
    assert not U.GradSlots.broken
    assert x.grad is not None and torch.isfinite(x.grad).all()


@pytest.mark.parametrize('k,fs,acc', [(2, 0, (0, 1)), (3, 2, (1, 0, 1)), (4, 1, (0, 0, 1, 1)),
                                      (5, 3, (1, 1, 0, 0, 1))])
@pytest.mark.parametrize('dt,ydt', [(torch.bfloat16, torch.float32), (torch.bfloat16, torch.bfloat16),
                                    (torch.float32, torch.float32)])
def test_merge_bwd_bn_kernel(k, fs, acc, dt, ydt):
    """um_merge_bwd_bn against torch: dsrc_s (+)= sigmoid(w_s) * dm (stored
    in the activation dtype), the per-block dots sum(dm * src_s) and the
    BN-ELU backward sums of source fs over its stored gradient.  k = 2..4
    take the loads-first instances, k = 5 the runtime source loop."""
    from umamd import _lib as L
    from umamd._lib import call, ptr, query
    M, C = 3000, 32
    g = torch.Generator().manual_seed(11 + k)
    rnd = lambda *s: torch.randn(*s, generator=g)  # noqa: E731
    srcs = [rnd(M, C).to(dt).to(DEV) for _ in range(k)]
    d0 = [rnd(M, C).to(dt) for _ in range(k)]
    dsrcs = [t.clone().to(DEV) for t in d0]
    dm = rnd(M, C).to(dt).to(DEV)
    w = rnd(k).to(DEV)
    widx = list(range(k))
    y = rnd(M, C).to(ydt).to(DEV)
    mean, invstd = rnd(C).to(DEV), (rnd(C).abs() + 0.5).to(DEV)
    scale, shift = rnd(C).to(DEV), rnd(C).to(DEV)
    slots = torch.zeros(L.STAT_SLOTS * C * 2 + 1, dtype=torch.float64, device=DEV)
    nparts = query('um_merge_bn_parts', M * C)
    parts = torch.zeros((nparts, k), dtype=torch.float32, device=DEV)
    ci, cp = L.ctypes.c_int, L.ctypes.c_void_p
    code = L.dtype_code(dt) | (L.Y_ACT if ydt != torch.float32 else 0)
    call('um_merge_bwd_bn', code, k, (cp * k)(*[t.data_ptr() for t in srcs]),
         (cp * k)(*[t.data_ptr() for t in dsrcs]), (ci * k)(*acc), (ci * k)(*widx), ptr(w), None,
         M * C, ptr(dm), ptr(parts), fs, ptr(y), C, ptr(mean), ptr(invstd), ptr(scale), ptr(shift),
         1, ptr(slots))
    torch.cuda.synchronize()
    coef = torch.sigmoid(w).cpu()
    dmf = dm.float().cpu()
    for s in range(k):
        want = ((d0[s].float() if acc[s] else 0) + coef[s] * dmf).to(dt).float()
        # one rounding of the activation dtype apart at most (fma vs mul + add)
        tol = 1e-6 if dt == torch.float32 else 2 ** -7
        torch.testing.assert_close(dsrcs[s].float().cpu(), want, rtol=tol, atol=1e-6)
        dot = (dmf.double() * srcs[s].double().cpu()).sum()
        assert abs(parts[:, s].double().sum().cpu() - dot) <= 1e-4 * (dmf.abs().sum() + 1), s
    r = dsrcs[fs].double().cpu()
    yc = y.double().cpu()
    z = yc * scale.double().cpu() + shift.double().cpu()
    dz = torch.where(z > 0, r, r * torch.exp(z))
    xhat = (yc - mean.double().cpu()) * invstd.double().cpu()
    got = slots[:L.STAT_SLOTS * C * 2].view(L.STAT_SLOTS, C, 2).sum(0).cpu()
    torch.testing.assert_close(got[:, 0], dz.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(got[:, 1], (dz * xhat).sum(0), rtol=1e-4, atol=1e-3)
    assert slots[-1].item() == M
