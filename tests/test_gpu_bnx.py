"""SyncBN statistics over the IPC exchange (umamd.bnx, csrc/bnx.hip;
UMAMD_SYNCBN_IPC=1) instead of one collective per BN layer and direction
(reference parallel_main.py:156-158).  Two processes share cuda:0 (the
box has one GPU; the arenas are mapped by HIP IPC either way), gloo carries
only the one-time handle exchange and DDP's gradients."""
import pytest
import torch

from test_ddp_cpu import launch
from test_gpu_ddp import test_syncbn_ddp_matches_single_process as _ddp_check

pytestmark = pytest.mark.gpu


def test_bnx_exchange_two_processes(tmp_path):
    """three steps x five widths (16..1024 channels): every rank ends with
    the rank-ordered sum, bit for bit, zeros in slots 1..15, the summed
    count; no exchange timed out (um_bnx_status)"""
    launch('bnx', 2, str(tmp_path), timeout=240)
    for r in range(2):
        z = torch.load(tmp_path / f'bnx_{r}.pt', weights_only=True)
        assert int(z['steps']) == 3
        print(f'rank {r}: {float(z["us_per_exchange"]):.2f} us per exchange')


def test_syncbn_ddp_ipc_matches_single_process(tmp_path):
    """the full model's SyncBN + DDP step with every BN statistics exchange
    (40 forward + 40 backward) on the IPC path: the same identity as the
    gloo collective path (test_gpu_ddp) against one process on the whole
    batch"""
    _ddp_check(tmp_path, ipc=True)
