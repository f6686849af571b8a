#!/usr/bin/env python3
"""bf16 precision arms at BASELINE config 2 (B=8 256x512 bayesian, formula
weights, the bench's synthetic pair, scale 0.3): for each arm (a set of
environment knobs) run the captured bf16 trajectory in a child process and
print its loss deltas against the reference's fp32 trajectory
(tests/golden/traj_c2.npz) and beside the reference's OWN bf16-autocast
deviation on the same workload (tests/golden/traj_c2_bf16.npz).

    python tools/bf16_arms.py                      # default arms
    python tools/bf16_arms.py 'UMAMD_F32_DEC=4' ''  # given arms ('' = defaults)
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(steps):
    sys.path.insert(0, REPO)
    import torch
    import bench
    cfg = bench.load_cfg(os.path.join(REPO, 'config.yml'), 'bayesian')
    tr = bench.loss_trajectory(cfg, os.environ.get('ARM_DTYPE', 'bf16'), torch.device('cuda', 0),
                               steps)
    print('TRAJ ' + json.dumps(tr), flush=True)


def deltas(tr, gold):
    dd = [abs(a[0] / b[0] - 1) for a, b in zip(tr, gold)]
    de = [abs(a[1] / b[1] - 1) for a, b in zip(tr, gold)]
    return {'step0_disp': dd[0], 'step0_error': de[0], 'max_disp': max(dd), 'max_error': max(de)}


def main():
    import numpy as np
    if len(sys.argv) > 1 and sys.argv[1] == '--child':
        child(int(sys.argv[2]))
        return
    g = np.load(os.path.join(REPO, 'tests/golden/traj_c2.npz'))
    n = sum(1 for k in g.files if k.startswith('disp_loss_'))
    gold = [(float(g[f'disp_loss_{i}']), float(g[f'error_loss_{i}'])) for i in range(n)]
    ab = os.path.join(REPO, 'tests/golden/traj_c2_bf16.npz')
    if os.path.exists(ab):
        a = np.load(ab)
        ac = [(float(a[f'disp_loss_{i}']), float(a[f'error_loss_{i}'])) for i in range(n)]
        print('reference bf16 autocast: ' + json.dumps(deltas(ac, gold)), flush=True)
    arms = sys.argv[1:] or ['', 'UMAMD_F32_DEC=4', 'UMAMD_F32_DEC=3', 'UMAMD_F32_DEC=1']
    for arm in arms:
        env = dict(os.environ)
        for kv in arm.split():
            k, v = kv.split('=', 1)
            env[k] = v
        r = subprocess.run([sys.executable, __file__, '--child', str(n)], env=env,
                           capture_output=True, text=True, timeout=600)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith('TRAJ ')]
        if r.returncode != 0 or not line:
            print(f'arm [{arm}] FAILED rc={r.returncode}\n{r.stderr[-2000:]}', flush=True)
            break
        tr = json.loads(line[0][5:])
        print(f'arm [{arm}]: ' + json.dumps(deltas(tr, gold)) +
              f' step0 {tr[0]}', flush=True)


if __name__ == '__main__':
    main()
