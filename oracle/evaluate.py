"""CPU restatement of the evaluation metrics (test infrastructure only).

* ``ssim_gauss``: torchmetrics.functional.structural_similarity_index_measure
  as reference train/evaluate.py:142-146 calls it (gaussian_kernel=True,
  sigma=1.5, data_range=1.0, k1=0.01, k2=0.03, reduction 'sum').  torchmetrics
  is NOT in this image and the reference pins no version (requirements.txt:13):
  this restates the published torchmetrics >= 0.11 `_ssim_update` algorithm --
  window size int(3.5*sigma+0.5)*2+1 = 11, reflect padding by 5, depthwise
  conv with the outer product of the normalised 1-D gaussian, then the crop
  of the 5-pixel border, per-image mean over channels and pixels.  PARITY
  UNPINNED for this metric (no reference output exists to check it against).
* ``curve`` / ``ause`` / ``aurg``: reference train/sparsification.py:8-61,
  pinned by tests/golden/sparsification.npz (generated from the reference).
"""
import torch
import torch.nn.functional as F


def _gaussian(ks, sigma, dtype):
    dist = torch.arange((1 - ks) / 2, (1 + ks) / 2, 1, dtype=dtype)
    g = torch.exp(-torch.pow(dist / sigma, 2) / 2)
    return (g / g.sum()).unsqueeze(0)


def ssim_gauss(preds, target, sigma=1.5, data_range=1.0, k1=0.01, k2=0.03, reduction='sum'):
    c = preds.shape[1]
    ks = int(3.5 * sigma + 0.5) * 2 + 1
    pad = (ks - 1) // 2
    dtype = preds.dtype
    gx = _gaussian(ks, sigma, dtype)
    kernel = torch.matmul(gx.t(), gx).expand(c, 1, ks, ks)
    p = F.pad(preds, (pad, pad, pad, pad), mode='reflect')
    t = F.pad(target, (pad, pad, pad, pad), mode='reflect')
    inp = torch.cat((p, t, p * p, t * t, p * t))
    out = F.conv2d(inp, kernel, groups=c).split(preds.shape[0])
    mu_p2, mu_t2, mu_pt = out[0].pow(2), out[1].pow(2), out[0] * out[1]
    s_p, s_t, s_pt = out[2] - mu_p2, out[3] - mu_t2, out[4] - mu_pt
    c1, c2 = (k1 * data_range) ** 2, (k2 * data_range) ** 2
    idx = ((2 * mu_pt + c1) * (2 * s_pt + c2)) / ((mu_p2 + mu_t2 + c1) * (s_p + s_t + c2))
    idx = idx[..., pad:-pad, pad:-pad]
    per = idx.reshape(idx.shape[0], -1).mean(-1)
    return per.sum() if reduction == 'sum' else per.mean() if reduction != 'none' else per


def curve(oracle_error, predicted_error, kernel_size=11, steps=100):
    """reference sparsification.curve (:8-36)"""
    b = predicted_error.size(0)
    pool = torch.nn.AvgPool2d(kernel_size, stride=1)
    o = pool(oracle_error).view(b, 2, -1)
    p = pool(predicted_error).view(b, 2, -1)
    srt = o.gather(2, p.argsort(2, True))
    mean = o.mean(dim=2)
    out = []
    for step in range(steps):
        removed = int(step / steps * o.size(2))
        out.append((srt[:, :, removed:].mean(dim=2) / mean).mean())
    return torch.stack(out)


def ause(oracle_curve, predicted_curve):
    return (predicted_curve - oracle_curve).sum() / len(oracle_curve)


def aurg(predicted_curve, random_curve):
    return ause(predicted_curve, random_curve)
