import sys, os
sys.path.insert(0, os.path.join(os.environ.get('GRAFT_REPO_ROOT', '/root/repo'), 'tests'))
import conftest  # noqa
import torch
from test_gpu_model import DEV, _cfg, _model, _uniform_pair
from train.graph import CapturedTrainStep
from train.loss import TukraUncertaintyLoss
from train.train import train_step
from umamd.optim import Adam
cfg = _cfg(); cfg['loss']['error_loss_config']['loss_type'] = 'l1'
left, right = _uniform_pair(2, 64, 128); left, right = left.to(DEV), right.to(DEV)
lf = TukraUncertaintyLoss(**cfg['loss'])
def eager(n):
    m = _model(cfg).train(); o = Adam(m.parameters(), 1e-4); out = []
    for _ in range(n):
        dl, el, _ = train_step(m, left, right, lf, o, 0.3); out.append((float(dl), float(el)))
    return m, out
m1, e1 = eager(8); m2, e2 = eager(8)
print('eager1', e1); print('eager2', e2)
m3 = _model(cfg).train(); o3 = Adam(m3.parameters(), 1e-4)
cap = CapturedTrainStep(m3, lf, o3, left, right, 0.3, warmup=2)
g = []
for _ in range(6):
    dl, el = cap(); g.append((float(dl), float(el)))
print('graph ', g)
print('step', [int(v['step']) for v in o3._dev.values()])
