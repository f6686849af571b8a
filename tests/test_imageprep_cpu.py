"""Input pipeline, host side (CPU): Pillow's bilinear resize restated by the
oracle (oracle/transforms.py) and the product's coefficient tables
(umamd/imageprep.py) against PIL itself, bit for bit; the worker-side draws
against the reference's RandomFlip / RandomAugment draw order."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

SIZES = [((288, 384), (256, 512)), ((256, 512), (256, 512)), ((1024, 1280), (256, 512)),
         ((100, 60), (37, 151)), ((7, 9), (64, 3))]


@pytest.mark.parametrize('src,dst', SIZES)
def test_oracle_resize_matches_pil(src, dst):
    from PIL import Image
    from oracle import transforms as OT
    rng = np.random.default_rng(hash(src + dst) % 2 ** 32)
    arr = rng.integers(0, 256, src + (3,), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(arr).resize((dst[1], dst[0]), Image.BILINEAR))
    assert np.array_equal(OT.pil_resize(arr, *dst), ref)


@pytest.mark.parametrize('n_in,n_out', [(384, 512), (288, 256), (1280, 512), (60, 151), (9, 3),
                                        (512, 512)])
def test_product_coeffs_match_oracle(n_in, n_out):
    from oracle import transforms as OT
    from umamd import imageprep as IP
    bounds, kk, ks = IP.resize_coeffs(n_in, n_out)
    for x, (lo, q) in enumerate(OT.pil_coeffs(n_in, n_out)):
        assert tuple(bounds[x]) == (lo, len(q))
        assert list(kk[x, :len(q)]) == q and not kk[x, len(q):].any()


def test_draws_follow_reference_order():
    """StereoDraws consumes numpy's global RNG exactly like the reference's
    RandomFlip(0.5) then RandomAugment(0.5, ...) (tests/golden/transforms.npz
    holds the reference's outputs for seed 2024: flip and augment decisions
    and values reproduce them through the oracle's arithmetic)."""
    from oracle import transforms as OT
    from umamd import imageprep as IP
    z = np.load(os.path.join(GOLDEN, 'transforms.npz'))
    left = torch.from_numpy(z['left'])
    right = torch.from_numpy(z['right'])
    # the golden's inputs are f32 [3, 24, 40] in [0, 1): only the draws matter
    u8 = np.zeros((24, 40, 3), np.uint8)
    d = IP.StereoDraws(0.5, 0.5, gamma=(0.8, 1.2), brightness=(0.5, 2.0), colour=(0.8, 1.2))
    np.random.seed(2024)
    for i in range(12):
        prep = d({'left': u8, 'right': u8})['prep'].numpy()
        # apply the drawn transform to the golden's float inputs
        out = []
        for t in (left, right):
            x = t.flip(-1) if prep[0] else t
            if prep[1]:
                x = torch.clamp(x ** float(prep[2]) * float(prep[3]) *
                                torch.from_numpy(prep[4:7]).view(3, 1, 1), 0, 1)
            out.append(x)
        assert torch.allclose(out[0], torch.from_numpy(z[f'left{i}']), atol=1e-6), i
        assert torch.allclose(out[1], torch.from_numpy(z[f'right{i}']), atol=1e-6), i
