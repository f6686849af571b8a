"""Input pipeline on the GPU (csrc/imageprep.hip, umamd/imageprep.py) against
the reference's transforms on the host: Pillow's bilinear resize (oracle
restatement pinned bit-for-bit to PIL by tests/test_imageprep_cpu.py, and PIL
itself), RandomFlip, ToTensor and RandomAugment with the same numpy draws.
Tolerance: bit-exact without augmentation (integer resampling, IEEE /255);
1e-6 absolute with augmentation (powf on the device vs torch's CPU pow, both
within ~1 ulp of the exact power)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _imgs(n, h, w, seed):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for _ in range(2 * n)]


@pytest.mark.parametrize('src', [(288, 384), (256, 512), (600, 900)])
def test_stereo_prep_matches_oracle(src):
    from oracle import transforms as OT
    from umamd import imageprep as IP
    n = 4
    imgs = _imgs(n, *src, seed=src[0])
    prep = np.zeros((n, 8), np.float32)
    prep[:, 2:7] = 1
    prep[1, 0] = 1                                     # flip only
    prep[2, 1:7] = (1, 0.83, 1.7, 0.9, 1.1, 1.05)      # augment only
    prep[3] = (1, 1, 1.15, 0.6, 1.2, 0.8, 0.95, 0)     # both
    batch = {'left': torch.from_numpy(np.stack(imgs[:n])),
             'right': torch.from_numpy(np.stack(imgs[n:])),
             'prep': torch.from_numpy(prep)}
    out = IP.stereo_prep(batch, (256, 512), torch.device(DEV))
    torch.cuda.synchronize()
    for i in range(n):
        rl, rr = OT.prep_pair(imgs[i], imgs[n + i], prep[i], 256, 512)
        for got, ref in ((out['left'][i].cpu(), rl), (out['right'][i].cpu(), rr)):
            if prep[i, 1]:
                assert float((got - ref).abs().max()) <= 1e-6, i
            else:
                assert torch.equal(got, ref), i


def test_device_augment_loader_matches_reference_pipeline():
    """DeviceAugment through a DataLoader (workers draw, GPU computes) vs the
    reference's CPU pipeline (train.transforms Compose with PIL resize) under
    the same numpy seed."""
    from PIL import Image
    from torch.utils.data import DataLoader
    import train.transforms as T
    from umamd.imageprep import to_device
    imgs = _imgs(3, 288, 384, seed=7)
    pairs = [{'left': Image.fromarray(imgs[i]), 'right': Image.fromarray(imgs[3 + i])}
             for i in range(3)]

    class DS(torch.utils.data.Dataset):
        def __init__(self, tf):
            self.tf = tf

        def __len__(self):
            return 3

        def __getitem__(self, i):
            return self.tf(dict(pairs[i]))

    ref_tf = T.Compose([T.ResizeImage((256, 512)), T.RandomFlip(0.5), T.ToTensor(),
                        T.RandomAugment(0.5, gamma=(0.8, 1.2), brightness=(0.5, 2.0),
                                        colour=(0.8, 1.2))])
    for seed in (3, 11):
        np.random.seed(seed)
        ref = next(iter(DataLoader(DS(ref_tf), batch_size=3, num_workers=0)))
        np.random.seed(seed)
        b = next(iter(DataLoader(DS(T.DeviceAugment((256, 512))), batch_size=3,
                                 num_workers=0)))
        assert b['left'].dtype == torch.uint8 and b['prep'].shape == (3, 8)
        left, right = to_device(b, torch.device(DEV))
        torch.cuda.synchronize()
        assert left.shape == (3, 3, 256, 512) and left.dtype == torch.float32
        assert float((left.cpu() - ref['left']).abs().max()) <= 1e-6
        assert float((right.cpu() - ref['right']).abs().max()) <= 1e-6
