"""Drop-in boundary: the reference's own main.py (unchanged, from
/root/reference) starts on this repository's ``model`` / ``train`` packages
through tools/ref_entry.py, builds our model, loss and transforms, runs the
reference's DaVinciDataset loader through our transforms, and reaches
``train_model`` (captured here instead of training: no GPU on this host).
torchvision is absent from the image, so ``torchvision.transforms.Compose``
is provided by ``train.transforms.Compose``.  Skipped where the reference
is not mounted (the GPU box)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

REF = '/root/reference'

DRIVER = r'''
import json, os, runpy, sys, types
sys.dont_write_bytecode = True
repo, ref, home = sys.argv[1:4]
extra = sys.argv[4:]
pkg = os.path.join(repo, 'uncertainty-model_amd')
sys.path[:0] = [pkg, ref]
import train, train.transforms as T
tv = types.ModuleType('torchvision'); tv.transforms = types.ModuleType('torchvision.transforms')
tv.transforms.Compose = T.Compose
sys.modules['torchvision'] = tv; sys.modules['torchvision.transforms'] = tv.transforms
seen = {}
def fake_train_model(model, loader, loss_function, epochs, lr, disc, disc_loss, **kw):
    batch = next(iter(loader))
    seen.update(model=type(model).__module__ + '.' + type(model).__name__,
                loss=type(loss_function).__module__ + '.' + type(loss_function).__name__,
                nparams=sum(p.numel() for p in model.parameters()),
                nstate=len(model.state_dict()), epochs=epochs, lr=lr,
                batch_shape=list(batch['left'].shape), batch_min=float(batch['left'].min()),
                batch_max=float(batch['left'].max()), evaluate_every=kw.get('evaluate_every'),
                val_batches=len(kw['val_loader']), disc=disc is not None,
                disc_class=(type(disc).__module__ + '.' + type(disc).__name__) if disc else None,
                disc_params=sum(p.numel() for p in disc.parameters()) if disc else 0,
                disc_loss=type(disc_loss).__name__ if disc_loss is not None else None)
    return [], []
train.train_model = fake_train_model
os.chdir(ref)
sys.argv = [os.path.join(ref, 'main.py'), 'config.yml', 'da-vinci', '--home', home,
            '--epochs', '1', '--batch-size', '2', '--workers', '0', '--no-cuda',
            '--training-size', '4', '--validation-size', '2', '--no-pbar'] + extra
runpy.run_path(sys.argv[0], run_name='__main__')
print('SEEN ' + json.dumps(seen))
'''


@pytest.mark.skipif(not os.path.isdir(REF), reason='reference not mounted')
@pytest.mark.parametrize('adversarial', [False, True])
def test_reference_main_reaches_train_model(tmp_path, adversarial):
    from PIL import Image
    rng = np.random.default_rng(0)
    for split, n in (('train', 4), ('test', 2)):
        for view in ('image_0', 'image_1'):
            d = tmp_path / 'datasets' / 'da-vinci' / split / view
            d.mkdir(parents=True)
            for i in range(n):
                arr = rng.integers(0, 256, (288, 384, 3), dtype=np.uint8)
                Image.fromarray(arr).save(d / f'{i:06d}.png')
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE='1')
    extra = ['--adversarial'] if adversarial else []
    r = subprocess.run([sys.executable, '-c', DRIVER, REPO, REF, str(tmp_path)] + extra, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    seen = json.loads(r.stdout.split('SEEN ', 1)[1])
    assert seen['model'] == 'model.model.RandomlyConnectedModel'
    assert seen['loss'] == 'train.loss.TukraUncertaintyLoss'
    assert seen['nparams'] == 22493949 and seen['nstate'] == 353
    assert seen['batch_shape'] == [2, 3, 256, 512]
    assert 0.0 <= seen['batch_min'] and seen['batch_max'] <= 1.0
    assert seen['evaluate_every'] == 10 and seen['val_batches'] == 1
    assert seen['disc'] == adversarial
    if adversarial:  # config.yml discriminator: 7,625,230 parameters
        assert seen['disc_class'] == 'model.discriminator.RandomDiscriminator'
        assert seen['disc_params'] == 7625230 and seen['disc_loss'] == 'BCELoss'
    assert not any(p.endswith('__pycache__') for p, _, _ in os.walk(REF))


PAR_DRIVER = r'''
import json, os, runpy, socket, sys, types
sys.dont_write_bytecode = True
repo, ref, home = sys.argv[1:4]
pkg = os.path.join(repo, 'uncertainty-model_amd')
sys.path[:0] = [pkg, ref]
import torch, torch.distributed as dist, torch.multiprocessing as mp
import torch.nn.parallel as tnp
import train, train.transforms as T
tv = types.ModuleType('torchvision'); tv.transforms = types.ModuleType('torchvision.transforms')
tv.transforms.Compose = T.Compose
sys.modules['torchvision'] = tv; sys.modules['torchvision.transforms'] = tv.transforms
# one process, gloo world 1 (no GPU here): the spawn runs main(0) inline
mp.spawn = lambda fn, args=(), nprocs=1, **kw: fn(0, *args)
_init = dist.init_process_group
def init_gloo(backend, init_method=None, world_size=-1, rank=-1, **kw):
    seen['backend_asked'] = backend
    return _init('gloo', init_method=init_method, world_size=world_size, rank=rank)
dist.init_process_group = init_gloo
class DDP(tnp.DistributedDataParallel):  # torch refuses device_ids and SyncBN on CPU modules
    def __init__(self, module, device_ids=None, **kw):
        seen['ddp_device_ids'] = device_ids
        super().__init__(module, **kw)
    def _passing_sync_batchnorm_handle(self, module):
        seen['sync_bn_check'] = True
tnp.DistributedDataParallel = DDP
seen = {}
def fake_train_model(model, loader, loss_function, epochs, lr, disc, disc_loss, **kw):
    from torch.nn import SyncBatchNorm
    inner = model.module
    seen.update(wrapper=isinstance(model, tnp.DistributedDataParallel),
                model=type(inner).__module__ + '.' + type(inner).__name__,
                loss=type(loss_function).__module__ + '.' + type(loss_function).__name__,
                nparams=sum(p.numel() for p in model.parameters()),
                nstate=len(inner.state_dict()),
                sync_bn=sum(isinstance(m, SyncBatchNorm) for m in inner.modules()),
                world=dist.get_world_size(), rank=kw.get('rank'),
                sampler=type(loader.sampler).__name__,
                batch_shape=list(next(iter(loader))['left'].shape), disc=disc is not None)
    return [], []
train.train_model = fake_train_model
with socket.socket() as s:
    s.bind(('127.0.0.1', 0)); port = s.getsockname()[1]
os.chdir(ref)
sys.argv = [os.path.join(ref, 'parallel_main.py'), 'config.yml', 'da-vinci', '--home', home,
            '--epochs', '1', '--batch-size', '2', '--workers', '0', '--no-cuda',
            '--training-size', '4', '--validation-size', '2', '--no-pbar',
            '--number-of-gpus', '1', '--master-address', '127.0.0.1', '--master-port', str(port)]
try:
    runpy.run_path(sys.argv[0], run_name='__main__')
except SystemExit:
    pass
print('SEEN ' + json.dumps(seen))
'''


@pytest.mark.skipif(not os.path.isdir(REF), reason='reference not mounted')
def test_reference_parallel_main_builds_ddp_on_our_packages(tmp_path):
    """The reference's DDP entry point (parallel_main.py:84-218, unchanged)
    on our packages: init_process_group (gloo, world 1: no GPU here),
    SyncBatchNorm conversion of our model (40 BN layers, :157), the DDP
    wrapper (:158), DistributedSampler loaders, our loss, up to train_model."""
    from PIL import Image
    rng = np.random.default_rng(1)
    for split, n in (('train', 4), ('test', 2)):
        for view in ('image_0', 'image_1'):
            d = tmp_path / 'datasets' / 'da-vinci' / split / view
            d.mkdir(parents=True)
            for i in range(n):
                arr = rng.integers(0, 256, (288, 384, 3), dtype=np.uint8)
                Image.fromarray(arr).save(d / f'{i:06d}.png')
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE='1')
    r = subprocess.run([sys.executable, '-c', PAR_DRIVER, REPO, REF, str(tmp_path)], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    seen = json.loads(r.stdout.split('SEEN ', 1)[1])
    assert seen['backend_asked'] == 'nccl' and seen['world'] == 1 and seen['rank'] == 0
    assert seen['wrapper'] and seen['ddp_device_ids'] == [0] and seen['sync_bn_check']
    assert seen['model'] == 'model.model.RandomlyConnectedModel'
    assert seen['loss'] == 'train.loss.TukraUncertaintyLoss'
    assert seen['nparams'] == 22493949 and seen['nstate'] == 353
    assert seen['sync_bn'] == 40
    assert seen['sampler'] == 'DistributedSampler'
    assert seen['batch_shape'] == [2, 3, 256, 512] and not seen['disc']
    assert not any(p.endswith('__pycache__') for p, _, _ in os.walk(REF))
