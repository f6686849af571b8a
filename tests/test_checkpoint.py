"""Checkpoint I/O (reference train/train.py:18-48,
main.py:126-137, train/utils.py:328-330): save_model writes the reference's
state_dict schema (NCHW f32 parameters, 353 model entries; {'model', 'disc'}
with a discriminator), the finetune path loads it back -- with the DDP
``module.`` prefix stripped by prepare_state_dict -- and the weights round
trip bit-exactly.  CPU only (no kernel runs)."""
import os

import torch
import yaml

from conftest import REPO


def _cfg():
    with open(os.path.join(REPO, 'config.yml')) as f:
        c = yaml.safe_load(f)
    c['model']['encoder']['load_graph'] = os.path.join(REPO, c['model']['encoder']['load_graph'])
    c['discriminator']['load_graph'] = os.path.join(REPO, c['discriminator']['load_graph'])
    return c


def test_save_and_finetune_load_roundtrip(tmp_path):
    import model as M
    import train.utils as u
    from train.train import save_model
    c = _cfg()
    torch.manual_seed(0)
    m = M.RandomlyConnectedModel(**c['model'])
    save_model(m, str(tmp_path), epoch_number=3)
    save_model(m, str(tmp_path), is_final=True)
    sd = torch.load(tmp_path / 'epoch_003.pt', weights_only=True)
    assert len(sd) == 353
    assert all(v.dtype in (torch.float32, torch.int64) for v in sd.values())
    m2 = M.RandomlyConnectedModel(**c['model'])
    m2.load_state_dict(u.prepare_state_dict(sd))  # main.py:135-137
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k]), k
    # a DistributedDataParallel checkpoint carries 'module.' prefixes
    ddp_sd = {'module.' + k: v for k, v in torch.load(tmp_path / 'final.pt',
                                                       weights_only=True).items()}
    m3 = M.RandomlyConnectedModel(**c['model'])
    m3.load_state_dict(u.prepare_state_dict(ddp_sd))
    assert torch.equal(m3.state_dict()['decoder.layers.4.disp.layers.0.weight'],
                       m.state_dict()['decoder.layers.4.disp.layers.0.weight'])


def test_adversarial_checkpoint_schema(tmp_path):
    import model as M
    import train.utils as u
    from train.train import save_model
    c = _cfg()
    m = M.RandomlyConnectedModel(**c['model'])
    d = M.RandomDiscriminator(**c['discriminator'])
    save_model(m, str(tmp_path), d, epoch_number=1)
    sd = torch.load(tmp_path / 'epoch_001.pt', weights_only=True)
    assert set(sd) == {'model', 'disc'}
    d2 = M.RandomDiscriminator(**c['discriminator'])
    d2.load_state_dict(u.prepare_state_dict(sd['disc']))  # main.py:129-133
    assert sum(v.numel() for k, v in sd['disc'].items()
               if not ('running' in k or 'num_batches' in k)) == 7625230
    for k, v in d.state_dict().items():
        assert torch.equal(v, d2.state_dict()[k]), k
