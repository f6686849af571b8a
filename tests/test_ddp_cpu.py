"""Data-parallel host logic on CPU, world_size 2 over gloo (no GPU): the
wrapper of reference parallel_main.py:156-158 (train/parallel.py) converts
all 40 BN layers to SyncBatchNorm, the umamd BN path sees world=2 and sums
its f64 statistics across ranks, and DDP averages gradients."""
import os
import socket
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch(mode, world, out, timeout=300, **extra_env):
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(free_port()),
               WORLD_SIZE=str(world), **extra_env)
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, 'ddp_worker.py'),
                                       mode, out], env=e))
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=timeout))
        except subprocess.TimeoutExpired:
            p.kill()
            codes.append('timeout')
    assert codes == [0] * world, codes


def test_dp_wrapper_gloo_world2(tmp_path):
    launch('cpu', 2, str(tmp_path))
    r = [torch.load(tmp_path / f'cpu_{i}.pt', weights_only=True) for i in range(2)]
    for x in r:
        assert int(x['n_sync_bn']) == 40
        assert int(x['world_seen']) == 2
        # sum over ranks of arange(6) * (rank + 1)
        assert torch.equal(x['stats'], torch.arange(6, dtype=torch.float64) * 3)
        assert int(x['nparams']) == 22_493_949
    # rank r feeds x = (r+1): the averaged gradient equals the gradient at
    # the mean input (linear in x for the first layer's weight)
    torch.manual_seed(0)
    ref = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4))
    g = [torch.zeros_like(p) for p in ref.parameters()]
    for k in (1, 2):
        ref.zero_grad()
        ref(torch.ones(3, 8) * k).sum().backward()
        g = [a + p.grad / 2 for a, p in zip(g, ref.parameters())]
    for x in r:
        for a, b in zip(x['grads'], g):
            assert torch.allclose(a, b, rtol=1e-6, atol=1e-6)
        # CapturedTrainStep's packed all-reduce gives DDP's average
        for a, b in zip(x['flat_grads'], g):
            assert torch.allclose(a, b, rtol=1e-6, atol=1e-6)
    # the bucketed, hook-launched exchange (umamd.gradsync) on a 3-layer net
    torch.manual_seed(0)
    ref3 = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4),
                               torch.nn.Linear(4, 4))
    g3 = [torch.zeros_like(p) for p in ref3.parameters()]
    for k in (1, 2):
        ref3.zero_grad()
        ref3(torch.ones(3, 8) * k).sum().backward()
        g3 = [a + p.grad / 2 for a, p in zip(g3, ref3.parameters())]
    for x in r:
        for a, b in zip(x['bucket_grads'], g3):
            assert torch.allclose(a, b, rtol=1e-6, atol=1e-6)


def test_collective_order_same_on_ranks_world2(tmp_path):
    """umamd.rccl: SyncBN all-reduces (launch stream) and gradient-bucket
    all-reduces (communication stream, one-parameter-sized buckets) go
    through ONE communicator in one chain: identical sequence on both ranks
    (asserted inside the workers), a wait at every stream switch, and the
    averaged gradients of the plain backward."""
    launch('order', 2, str(tmp_path))
    r = [torch.load(tmp_path / f'order_{i}.pt', weights_only=True) for i in range(2)]
    assert r[0]['seq'] == r[1]['seq']
    for a, b in zip(r[0]['grads'], r[1]['grads']):
        assert torch.equal(a, b)
