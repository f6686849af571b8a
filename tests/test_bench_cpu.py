"""bench.py's host-side logic on CPU: ``--gpus N`` spawns N rank processes
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one rendezvous port), the
worst exit status propagates and a failing rank stops the others."""
import json
import os
import subprocess
import sys

from conftest import REPO

CHILD = r'''
import json, os, sys, time
keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')
with open(os.path.join(sys.argv[1], 'rank%s.json' % os.environ['RANK']), 'w') as f:
    json.dump({k: os.environ.get(k) for k in keys}, f)
if sys.argv[2] == 'fail' and os.environ['RANK'] == '1':
    sys.exit(3)
if sys.argv[2] == 'fail':
    time.sleep(60)  # must be stopped by the launcher
'''


def _spawn(tmp_path, n, mode):
    code = ('import sys; sys.path.insert(0, %r); import bench; '
            'sys.exit(bench.spawn_ranks(%d, [sys.executable, "-c", %r, %r, %r]))'
            % (REPO, n, CHILD, str(tmp_path), mode))
    return subprocess.run([sys.executable, '-c', code], timeout=120, capture_output=True,
                          text=True)


def test_spawn_sets_rank_env(tmp_path):
    r = _spawn(tmp_path, 4, 'ok')
    assert r.returncode == 0, r.stderr
    envs = [json.load(open(tmp_path / f'rank{i}.json')) for i in range(4)]
    assert [e['RANK'] for e in envs] == ['0', '1', '2', '3']
    assert [e['LOCAL_RANK'] for e in envs] == ['0', '1', '2', '3']
    assert {e['WORLD_SIZE'] for e in envs} == {'4'}
    assert {e['MASTER_ADDR'] for e in envs} == {'127.0.0.1'}
    assert len({e['MASTER_PORT'] for e in envs}) == 1


def test_spawn_propagates_failure(tmp_path):
    r = _spawn(tmp_path, 3, 'fail')
    assert r.returncode == 3, (r.returncode, r.stderr)


def test_bench_parses_gpus_flag():
    sys.path.insert(0, REPO)
    import bench
    old = sys.argv
    try:
        sys.argv = ['bench.py', '--gpus', '8', '--steps', '3']
        a = bench.parse()
    finally:
        sys.argv = old
    assert a.gpus == 8 and a.steps == 3
    assert os.path.exists(os.path.join(REPO, 'tests', 'golden', 'traj_c2.npz'))


def test_post_timing_leg_failure_keeps_the_line(monkeypatch):
    """A leg after the timed region that raises (here the CPU baseline and
    the eager comparison) is recorded in ``leg_errors``; the other legs and
    the measured value still go out (bench.main prints the line after
    post_timing_legs returns)."""
    import argparse
    import bench

    def boom(*a, **k):
        raise RuntimeError('leg exploded')
    monkeypatch.setattr(bench, 'cpu_baseline', boom)
    monkeypatch.setattr(bench, 'time_eager', boom)
    monkeypatch.setattr(bench, 'time_fp32', lambda *a, **k: {'value': 1.0})
    a = argparse.Namespace(loader_steps=0, eager_steps=3, no_roofline=True, dtype='bf16',
                           fp32_steps=5, no_cpu_baseline=False, no_loss_delta=True, height=256,
                           width=512, batch=8, loss_type='bayesian', config='config.yml',
                           cpu_steps=5)

    class _Stream:  # torch.cuda.stream(...) stand-in on a CPU-only host
        pass
    monkeypatch.setattr(bench.torch.cuda, 'stream', lambda s: __import__('contextlib').nullcontext())
    monkeypatch.setattr(bench.torch.cuda, 'synchronize', lambda: None)
    errors = {}
    res = bench.post_timing_legs(a, None, True, None, None, None, None, None, 0.3, None, None,
                                 _Stream(), errors)
    assert res['fp32_line'] == {'value': 1.0}
    assert res['cpu_baseline'] is None and res['eager_launch'] is None
    assert set(errors) == {'cpu_baseline', 'eager_launch'}
    assert 'leg exploded' in errors['cpu_baseline']
