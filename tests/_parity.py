"""Shared parity helpers of the test suite (test infrastructure).

Gradient checks are by DIRECTION, not only by norm:
  * ``rel_norm(g, g_ref)`` = ||g - g_ref|| / ||g_ref|| when both full tensors
    are in memory (the oracle on the same inputs);
  * ``sketch_worst`` compares 8 Rademacher projections of the gradient with
    the reference's own (stored in the step goldens by make_goldens.py via
    oracle.step.grad_sketch): ||S(g) - S(g_ref)|| estimates sqrt(8) *
    ||g - g_ref||, so a gradient of the right norm and the wrong direction
    fails where a norm comparison would pass.
"""
from __future__ import annotations

import torch

from oracle import step as OS


def pre_bn_bias(k: str) -> bool:
    """Parameters whose true gradient is 0, so their value is fp noise
    (SURVEY 8c): conv biases followed by a training-mode BatchNorm, the
    attention key bias (softmax over pixels is invariant to a per-channel
    shift, reference model/layers/attention.py:63) and the last stage's
    value/reprojection biases (a per-channel constant on x4, which the decoder
    only consumes through BN'd convs, model/decoder.py:51)."""
    if k in ('encoder.layers.4.layers.1.values.bias',
             'encoder.layers.4.layers.1.reprojection.bias'):
        return True
    return k.endswith('.bias') and ('convolution.layers.0.' in k or 'keys.bias' in k or any(
        t in k for t in ('upsample.0.layers.0.layers.0.', 'squeeze_excite.0.layers.0.layers.0.',
                         'iconv.layers.0.layers.0.')))


def atol_of(k: str) -> float:
    """per-element absolute floor: the merge weights' ~1e-5 gradients are sums
    over whole feature maps with heavy cancellation (fp32 vs fp64 of the
    reference itself differ by ~3e-5)"""
    return 3e-5 if k.endswith('mean_weight') else 1e-6


def rel_norm(g: torch.Tensor, ref: torch.Tensor) -> float:
    g = g.detach().to('cpu', torch.float64)
    ref = ref.detach().to('cpu', torch.float64)
    return float((g - ref).norm() / ref.norm().clamp_min(1e-30))


def grad_worst(grads, ref_grads, tol, tol_of=None):
    """Full-tensor check: ||g - g_ref|| <= tol * ||g_ref|| + sqrt(n) * atol
    per parameter with a non-zero true gradient -> (worst ratio, name, rel)"""
    worst = (0.0, None, 0.0)
    for k, g in grads.items():
        if pre_bn_bias(k) or ref_grads.get(k) is None:
            continue
        r = ref_grads[k].detach().to('cpu', torch.float64)
        d = float((g.detach().to('cpu', torch.float64) - r).norm())
        t = tol_of(k) if tol_of is not None else tol
        bound = t * float(r.norm()) + (r.numel() ** 0.5) * atol_of(k)
        worst = max(worst, (d / bound, k, d / max(float(r.norm()), 1e-30)))
    return worst


def sketch_worst(grads, z, tol, tol_of=None):
    """Sketch check against a golden: ||S(g) - S(g_ref)|| <= tol *
    ||S(g_ref)|| + sqrt(8) * atol per parameter -> (worst ratio, name, rel)"""
    worst = (0.0, None, 0.0)
    for k, g in grads.items():
        if pre_bn_bias(k) or f'sketch/{k}' not in z.files:
            continue
        ref = torch.from_numpy(z[f'sketch/{k}'])
        d = float((OS.grad_sketch(k, g) - ref).norm())
        t = tol_of(k) if tol_of is not None else tol
        bound = t * float(ref.norm()) + (OS.SKETCHES ** 0.5) * atol_of(k)
        worst = max(worst, (d / bound, k, d / max(float(ref.norm()), 1e-30)))
    return worst
