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
