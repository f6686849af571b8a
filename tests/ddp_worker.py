"""Worker for the data-parallel tests (launched as a subprocess per rank by
tests/test_ddp_cpu.py and tests/test_gpu_ddp.py; not collected by pytest).

mode 'cpu'    : gloo, CPU only -- host logic of the DP wrapper: SyncBN
                conversion, BNSync world detection, f64 stats all-reduce, DDP
                construction and gradient averaging hooks on plain tensors.
mode 'order'  : gloo, CPU -- the captured step's collective order (SyncBN +
                gradient buckets through one ordered communicator) recorded
                on every rank (umamd.rccl).
mode 'single' : one process, full batch on cuda:0, one train step.
mode 'ddp'    : gloo ranks sharing cuda:0, each on its batch shard, one
                DDP+SyncBN train step (SURVEY 8c golden (v): SyncBN identity).
mode 'ddp_uneven': the same with shards of 1 and 3 images (per-rank counts).
Writes results to <out>/<mode>_<rank>.pt (torch.save of tensors only).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (os.path.join(REPO, 'uncertainty-model_amd'), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import yaml  # noqa: E402


def cfg():
    with open(os.path.join(REPO, 'config.yml')) as f:
        c = yaml.safe_load(f)
    c['model']['encoder']['load_graph'] = os.path.join(REPO, c['model']['encoder']['load_graph'])
    c['loss']['error_loss_config']['loss_type'] = 'bayesian'
    return c


def model_with_formula_weights(c, dtype='fp32'):
    import model as M
    from oracle import model as OM, step as OS
    m = M.RandomlyConnectedModel(**c['model'], dtype=dtype)
    specs = OS.param_specs(c['model'], OM.load_stage_graphs(c['model']['encoder']))
    m.load_state_dict(OS.formula_state_dict(specs))
    return m


def batch(total=4, h=64, w=128):
    g = torch.Generator().manual_seed(1234)
    return torch.rand(total, 3, h, w, generator=g), torch.rand(total, 3, h, w, generator=g)


def run_cpu(rank, world, out):
    from train.parallel import count_sync_bn, data_parallel
    from umamd.functional import BNSync
    c = cfg()
    sm = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model_with_formula_weights(c))
    bns = [mod for mod in sm.modules() if isinstance(mod, torch.nn.SyncBatchNorm)]
    st = torch.arange(6, dtype=torch.float64) * (rank + 1)
    BNSync(bns[0]).all_reduce(st)
    # torch's DDP refuses SyncBatchNorm on CPU modules and the model's
    # forward is HIP-only: gradient averaging is checked on a small module
    # through the same wrapper (gradient_as_bucket_view, buckets, hooks)
    torch.manual_seed(0)
    dp = data_parallel(torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4)),
                       sync_bn=False)
    x = torch.ones(3, 8) * (rank + 1)
    dp(x).sum().backward()
    nparams = sum(p.numel() for p in model_with_formula_weights(c).parameters())
    # the captured step's own gradient exchange (train/graph.py _reduce_grads:
    # pack -> one all-reduce -> .grad views), host logic on the same module;
    # the third Linear is unused and keeps .grad None
    from train.graph import CapturedTrainStep
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4),
                              torch.nn.Linear(4, 4))
    net[1](net[0](x)).sum().backward()
    cs = CapturedTrainStep.__new__(CapturedTrainStep)
    cs.model, cs.group, cs.world = net, dist.group.WORLD, world
    cs._buckets = None
    cs._reduce_grads()
    # bucketed exchange from the backward's hooks (umamd.gradsync): 3 buckets
    # of this net, launched in backward order as each one's gradients land
    from umamd.gradsync import GradBuckets
    torch.manual_seed(0)
    net2 = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4),
                               torch.nn.Linear(4, 4))
    gb = GradBuckets(net2.parameters(), dist.group.WORLD, world, cap_mb=80 / 2 ** 20)
    order = []
    orig_launch = gb._launch
    gb._launch = lambda bi: (order.append(bi), orig_launch(bi))
    for it in range(2):  # step 1 learns the layout (reduced in finish); step 2 from hooks
        for p in net2.parameters():
            p.grad = None
        order.clear()
        gb.arm()
        net2[2](net2[1](net2[0](x))).sum().backward()
        launched_in_backward = list(order)
        gb.finish()
    bucket_grads = [p.grad.clone() for p in net2.parameters()]
    assert launched_in_backward == list(range(len(gb.buckets))) and len(gb.buckets) >= 3, \
        (launched_in_backward, [len(b) for b in gb.buckets])
    flat_grads = [p.grad.clone() for p in list(net.parameters())[:4]]
    assert all(p.grad is None for p in net[2].parameters())
    assert all(p.grad.data_ptr() >= cs._flat.data_ptr() for p in list(net.parameters())[:4])
    torch.save({'flat_grads': flat_grads, 'bucket_grads': bucket_grads, 'x': x,
                'n_sync_bn': torch.tensor(count_sync_bn(sm)),
                'world_seen': torch.tensor(BNSync(bns[0]).world),
                'stats': st,
                'grads': [p.grad.clone() for p in dp.parameters()],
                'nparams': torch.tensor(nparams)},
               os.path.join(out, f'cpu_{rank}.pt'))


class _RecordingComm:
    """Stand-in for umamd.rccl.Comm on gloo/CPU: the same collective-chain
    bookkeeping (umamd.rccl._Order, with fake streams) and a log of every
    collective; the values go through the gloo group."""

    def __init__(self, group):
        from umamd import rccl
        self.group = group
        self.ranks = dist.get_process_group_ranks(group)
        self.stream = 'launch'  # the issuing stream of the next collective
        self.order = rccl._Order(record=lambda s: ('event', s), wait=lambda s, ev: None)
        self.seq = []

    @property
    def world(self):
        return dist.get_world_size(self.group)

    def all_reduce(self, t, average=False):
        self.order.before(self.stream)
        self.order.sig.append((int(t.numel()), str(t.dtype)))
        self.seq.append((self.stream, tuple(t.shape), str(t.dtype), bool(average)))
        dist.all_reduce(t, group=self.group)
        if average:
            t.mul_(1.0 / dist.get_world_size(self.group))


def run_order(rank, world, out):
    """The captured step's collective sequence (SyncBN statistics on the
    launch stream, gradient buckets on the communication stream, tiny
    buckets) recorded on both ranks: the same order everywhere, and a wait
    on the previous collective's stream at every switch (umamd.rccl)."""
    from umamd import rccl
    from umamd.functional import BNSync
    from umamd.gradsync import GradBuckets
    rec = _RecordingComm(dist.group.WORLD)
    bn = torch.nn.SyncBatchNorm(4)
    sync = BNSync(bn)
    assert sync.collective

    class SyncLayer(torch.autograd.Function):
        """a SyncBN-like layer: all-reduce in forward and in backward"""
        @staticmethod
        def forward(ctx, x, i):
            st = torch.full((4 + i,), float(rank + 1), dtype=torch.float64)
            sync.all_reduce(st)
            assert torch.all(st == 3.0)
            ctx.i = i
            return x * 1.0

        @staticmethod
        def backward(ctx, g):
            st = torch.full((8 + ctx.i,), float(rank + 1), dtype=torch.float64)
            sync.all_reduce(st)
            assert torch.all(st == 3.0)
            return g, None

    torch.manual_seed(0)
    layers = torch.nn.ModuleList([torch.nn.Linear(8, 8) for _ in range(6)])
    gb = GradBuckets(layers.parameters(), dist.group.WORLD, world, cap_mb=300 / 2 ** 20)
    orig = gb._reduce

    def on_comm_stream(dst):
        prev, rec.stream = rec.stream, 'comm'
        try:
            orig(dst)
        finally:
            rec.stream = prev
    gb._reduce = on_comm_stream
    x = torch.ones(2, 8) * (rank + 1)
    seqs = []
    with rccl.use(rec):
        for it in range(2):  # step 1 learns the layout, step 2 launches from hooks
            rec.seq = []
            rec.order.reset()
            for p in layers.parameters():
                p.grad = None
            gb.arm()
            h = x
            for i, lin in enumerate(layers):
                h = SyncLayer.apply(lin(h), i)
            h.sum().backward()
            gb.finish()
            seqs.append(list(rec.seq))
            log = list(rec.order.log)
    # every switch of issuing stream waits on the previous one
    prev = None
    for i, e in enumerate(log):
        if e[0] == 'coll':
            if prev is not None and prev != e[1]:
                assert log[i - 1] == ('wait', e[1], prev), (i, log[i - 1], e)
            prev = e[1]
    kinds = [s for s, *_ in seqs[1]]
    assert 'comm' in kinds and kinds.count('launch') == 12, kinds
    # the buckets launch during the backward: comm collectives between the
    # launch-stream (SyncBN backward) ones
    first_comm = kinds.index('comm')
    assert 'launch' in kinds[first_comm:], kinds
    allseq = [None] * world
    dist.all_gather_object(allseq, seqs)
    assert all(s == allseq[0] for s in allseq), 'collective order differs between ranks'
    # umamd.rccl.check_order: passes on the recorded sequence; a rank that
    # issued one collective more (or in another order) fails on every rank
    rccl.check_order(rec)
    rec.order.sig.append((rank + 1, 'torch.float64'))
    try:
        rccl.check_order(rec)
        raise AssertionError('check_order missed a rank-dependent collective sequence')
    except RuntimeError as e:
        assert 'different order' in str(e), e
    torch.save({'seq': [[list(map(str, e)) for e in s] for s in seqs],
                'grads': [p.grad.clone() for p in layers.parameters()]},
               os.path.join(out, f'order_{rank}.pt'))


def run_bnx(rank, world, out):
    """umamd.bnx on two processes sharing cuda:0: statistics-slot tensors of
    several widths exchanged over the IPC arenas, three steps of 5 slots;
    every rank must end with the rank-ordered sum of the ranks' slot sums
    (computed here from the same seeded draws), bit for bit."""
    from umamd import bnx
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    x = bnx.BNExchange(dist.group.WORLD)
    widths = [16, 64, 512, 1024, 40]
    results = []
    for step in range(3):
        x.begin_forward()
        outs = []
        for i, C in enumerate(widths):
            def draw(r):
                g = torch.Generator().manual_seed(1000 * step + 10 * i + r)
                t = torch.randn(16 * C * 2 + 1, generator=g, dtype=torch.float64)
                t[-1] = 100 + r
                return t
            mine = draw(rank).to(dev)
            x.all_reduce_slots(mine, C)
            # expected: per rank the 16 slots summed in slot order, then the
            # ranks in rank order (the kernel's order)
            exp = torch.zeros(2 * C + 1, dtype=torch.float64)
            for r in range(world):
                d = draw(r)
                v = torch.zeros(2 * C, dtype=torch.float64)
                for sl in range(16):
                    v = v + d[sl * 2 * C:(sl + 1) * 2 * C]
                exp[:2 * C] = exp[:2 * C] + v
                exp[2 * C] = exp[2 * C] + d[-1]
            outs.append((mine.cpu(), exp))
        torch.cuda.synchronize()
        for got, exp in outs:
            C2 = exp.numel() - 1
            assert torch.equal(got[:C2], exp[:C2]), (step, float((got[:C2] - exp[:C2]).abs().max()))
            assert torch.equal(got[C2:16 * C2], torch.zeros(15 * C2, dtype=torch.float64))
            assert float(got[-1]) == float(exp[-1])
        results.append(len(outs))
    # time: 40 exchanges (one step's forward) of C = 256, both ranks in lockstep
    t = torch.zeros(16 * 256 * 2 + 1, dtype=torch.float64, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for rep in range(3):
        x.begin_forward()
        dist.barrier()
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(40):
            x.all_reduce_slots(t, 256)
        ev[1].record()
        ev[1].synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1e3 / 40
    print(f'bnx rank {rank}: {us:.2f} us per exchange (C=256, 2 processes on one GPU)', flush=True)
    x.check()
    x.close()
    torch.save({'steps': torch.tensor(len(results)), 'us_per_exchange': torch.tensor(us)},
               os.path.join(out, f'bnx_{rank}.pt'))


def run_step(mode, rank, world, out):
    from train.loss import TukraUncertaintyLoss
    from train.parallel import data_parallel, unwrap
    from train.train import train_step
    from umamd.optim import Adam
    c = cfg()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    m = model_with_formula_weights(c).to(dev).train()
    if mode in ('ddp', 'ddp_uneven'):
        m = data_parallel(m, 0)
    left, right = batch()
    if mode == 'ddp_uneven':  # rank 0: image 0, rank 1: images 1-3
        sl = slice(0, 1) if rank == 0 else slice(1, 4)
    else:
        per = left.shape[0] // world
        sl = slice(rank * per, (rank + 1) * per)
    left, right = left[sl].to(dev), right[sl].to(dev)
    lf = TukraUncertaintyLoss(**c['loss'])
    opt = Adam(m.parameters(), 1e-4)
    dl, el, _ = train_step(m, left, right, lf, opt, 0.3)
    torch.cuda.synchronize()
    # Adam reads .grad but does not modify it; under DDP these are the
    # all-reduced (averaged) bucket views
    grads = {n: p.grad.detach().clone().cpu() for n, p in unwrap(m).named_parameters()}
    sd = {k: v.detach().clone().cpu() for k, v in unwrap(m).state_dict().items()}
    from umamd import bnx
    nx = 0
    for x in bnx._exchanges.values():  # UMAMD_SYNCBN_IPC=1: the exchanges this step used
        x.check()
        nx += x.slot
    bnx.close_all()
    torch.save({'disp': torch.tensor(float(dl)), 'err': torch.tensor(float(el)),
                'grads': grads, 'state': sd, 'bnx_exchanges': torch.tensor(nx)},
               os.path.join(out, f'{mode}_{rank}.pt'))


def main():
    mode, out = sys.argv[1], sys.argv[2]
    rank = int(os.environ.get('RANK', '0'))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if mode in ('cpu', 'order', 'ddp', 'ddp_uneven', 'bnx'):
        dist.init_process_group('gloo', init_method='env://', rank=rank, world_size=world)
    if mode == 'cpu':
        run_cpu(rank, world, out)
    elif mode == 'order':
        run_order(rank, world, out)
    elif mode == 'bnx':
        run_bnx(rank, world, out)
    else:
        run_step(mode, rank, world, out)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
