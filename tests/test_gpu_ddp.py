"""SyncBN + DDP identity on the HIP path (SURVEY 8c golden (v), 8e): two
gloo ranks sharing cuda:0, each training on half of a B=4 batch through
train.parallel.data_parallel (reference parallel_main.py:156-158), must
reproduce one process training on the whole batch: same loss (mean over
ranks), same averaged gradients, same BN running statistics.  RCCL needs
one GPU per rank, so the exchange runs over gloo here; the umamd BN path
issues the same all_reduce calls either way."""
import pytest
import torch

from test_ddp_cpu import launch
from test_gpu_model import _pre_bn_bias

pytestmark = pytest.mark.gpu


def test_syncbn_ddp_matches_single_process(tmp_path, ipc=False):
    launch('single', 1, str(tmp_path))
    launch('ddp', 2, str(tmp_path), **({'UMAMD_SYNCBN_IPC': '1'} if ipc else {}))
    s = torch.load(tmp_path / 'single_0.pt', weights_only=True)
    r = [torch.load(tmp_path / f'ddp_{i}.pt', weights_only=True) for i in range(2)]
    # every BN statistics exchange on the IPC path (40 forward + 40
    # backward) or none of them
    assert [int(x['bnx_exchanges']) for x in r] == ([80, 80] if ipc else [0, 0])
    for key in ('disp', 'err'):
        mean = (float(r[0][key]) + float(r[1][key])) / 2
        assert abs(mean - float(s[key])) <= 1e-4 * abs(float(s[key])), (key, mean, float(s[key]))
    bad = []
    for k, g in s['grads'].items():
        assert torch.equal(r[0]['grads'][k], r[1]['grads'][k]), k  # all-reduced: identical
        if _pre_bn_bias(k):
            continue
        d = float((r[0]['grads'][k].double() - g.double()).norm())
        n = float(g.double().norm())
        atol = 3e-5 if k.endswith('mean_weight') else 1e-6
        if d > 2e-2 * n + atol:
            bad.append((k, d, n))
    assert not bad, bad[:8]
    for k, v in s['state'].items():
        a, b = r[0]['state'][k], r[1]['state'][k]
        if 'running' in k or 'num_batches' in k:
            assert torch.equal(a, b), k
            if v.is_floating_point():
                assert float((a - v).abs().max()) <= 1e-3 * (float(v.abs().max()) + 1e-3), k
            else:
                assert torch.equal(a, v), k
        elif v.is_floating_point() and not _pre_bn_bias(k):
            # first Adam step moves each weight by ~lr * sign(grad)
            assert torch.equal(a, b), k
            assert float((a - v).abs().max()) <= 2.5e-4, k


def test_syncbn_uneven_rank_batches(tmp_path):
    """Shards of 1 and 3 images: SyncBN must weight each rank by its own
    element count (torch SyncBatchNorm all-gathers the counts), so the BN
    running statistics equal those of one process on all 4 images.  (The
    gradients differ by design: DDP averages per-rank means equally.)"""
    launch('single', 1, str(tmp_path))
    launch('ddp_uneven', 2, str(tmp_path))
    s = torch.load(tmp_path / 'single_0.pt', weights_only=True)
    r = [torch.load(tmp_path / f'ddp_uneven_{i}.pt', weights_only=True) for i in range(2)]
    n = 0
    for k, v in s['state'].items():
        if 'running' in k:
            a, b = r[0]['state'][k], r[1]['state'][k]
            assert torch.equal(a, b), k
            assert float((a - v).abs().max()) <= 1e-3 * (float(v.abs().max()) + 1e-3), k
            n += 1
    assert n == 80
