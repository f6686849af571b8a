"""train.transforms (reference train/transforms.py:15-129), host-side, CPU.

RandomFlip / RandomAugment are checked against outputs of the reference's
own classes on the same seeded numpy RNG draws (tests/golden/transforms.npz,
make_goldens.py); Resize / ToTensor against their torchvision semantics
(torchvision is absent from the image: parity for those two is pinned by the
definitions restated in train/transforms.py, not by torchvision itself)."""
import os

import numpy as np
import torch

from conftest import GOLDEN


def test_flip_augment_match_reference_draws():
    import train.transforms as T
    z = np.load(os.path.join(GOLDEN, 'transforms.npz'))
    left, right = torch.from_numpy(z['left']), torch.from_numpy(z['right'])
    flip = T.RandomFlip(0.5)
    aug = T.RandomAugment(0.5, gamma=(0.8, 1.2), brightness=(0.5, 2.0), colour=(0.8, 1.2))
    np.random.seed(2024)
    for i in range(12):
        out = aug(flip({'left': left.clone(), 'right': right.clone()}))
        assert torch.equal(out['left'], torch.from_numpy(z[f'left{i}'])), i
        assert torch.equal(out['right'], torch.from_numpy(z[f'right{i}'])), i


def test_resize_to_tensor_pil_and_tensor():
    from PIL import Image
    import train.transforms as T
    rng = np.random.default_rng(0)
    arr = rng.integers(0, 256, (60, 100, 3), dtype=np.uint8)
    pil = Image.fromarray(arr)
    pipe = T.Compose([T.ResizeImage((32, 64)), T.ToTensor()])
    out = pipe({'left': pil, 'right': pil.transpose(Image.FLIP_LEFT_RIGHT)})
    ref = torch.from_numpy(np.array(pil.resize((64, 32), Image.BILINEAR))).permute(2, 0, 1)
    assert out['left'].shape == (3, 32, 64) and out['left'].dtype == torch.float32
    assert torch.equal(out['left'], ref.float() / 255)
    assert torch.equal(out['right'], out['left'].flip(-1)) or \
        float((out['right'] - out['left'].flip(-1)).abs().max()) < 2 / 255
    # tensor input: antialiased bilinear, same size is the identity
    t = torch.rand(3, 32, 64)
    assert torch.allclose(T.resize(t, (32, 64)), t, atol=1e-6)
    assert T.resize(t, (16, 32)).shape == (3, 16, 32)


def test_to_tensor_modes():
    from PIL import Image
    import train.transforms as T
    g = Image.fromarray(np.arange(12, dtype=np.uint8).reshape(3, 4), mode='L')
    t = T.to_tensor(g)
    assert t.shape == (1, 3, 4) and abs(float(t[0, 2, 3]) - 11 / 255) < 1e-7
