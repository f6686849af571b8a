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
