"""One training step on the CPU oracle + deterministic weights -- TEST ORACLE.

  * ``param_specs(model_cfg, graphs)``: the reference state_dict schema
    (names, shapes, kind) derived from the config, restating the module tree of
    model/model.py:15-19, model/encoder.py:26-40, model/layers/encoder.py:
    21-52,55-127,130-176,228-259, model/layers/attention.py:22-40 and
    model/layers/decoder.py:11-208.
  * ``formula_state_dict``: weights as a deterministic function of
    (parameter name, element index), so goldens need no weight file.
  * ``train_step``: train/train.py:116-129 (pyramid -> model -> reconstruct ->
    loss -> backward -> Adam) with torch.optim.Adam semantics
    (train/train.py:228: Adam(params, lr), default betas/eps).
"""
from __future__ import annotations

import math
import zlib
from collections import OrderedDict
from typing import Dict, List, Tuple

import torch

from . import graph as og
from . import loss as L
from . import model as M


def _conv(specs, pre, cin, cout, k, bias=True):
    specs.append((pre + 'weight', (cout, cin, k, k), 'conv'))
    if bias:
        specs.append((pre + 'bias', (cout,), 'conv_bias'))


def _bn(specs, pre, c):
    specs += [(pre + 'weight', (c,), 'bn_weight'), (pre + 'bias', (c,), 'bn_bias'),
              (pre + 'running_mean', (c,), 'running_mean'),
              (pre + 'running_var', (c,), 'running_var'),
              (pre + 'num_batches_tracked', (), 'nbt')]


def param_specs(model_cfg, graphs) -> List[Tuple[str, tuple, str]]:
    specs: List[Tuple[str, tuple, str]] = []
    for s, lay in enumerate(model_cfg['encoder']['layers']):
        nodes, _, _ = og.graph_info(graphs[s])
        cin, cout, k = lay['in_channels'], lay['out_channels'], lay['kernel_size']
        for node in nodes:
            pre = f'encoder.layers.{s}.layers.0.node_blocks.{node.id}.'
            if len(node.inputs) > 1:
                specs.append((pre + 'mean_weight', (len(node.inputs),), 'mean_weight'))
            ci = cin if node.node_type == 'input' else cout
            _conv(specs, pre + 'convolution.layers.0.', ci, cout, k)
            _bn(specs, pre + 'convolution.layers.1.', cout)
        for nm in ('keys', 'queries', 'values', 'reprojection'):
            _conv(specs, f'encoder.layers.{s}.layers.1.{nm}.', cout, cout, 1)
    for s, lay in enumerate(model_cfg['decoder']['layers']):
        pre = f'decoder.layers.{s}.'
        up = lay['upsample_channels'] * 4
        _conv(specs, pre + 'upsample.0.layers.0.layers.0.', lay['in_channels'], up, 3)
        if lay.get('batch_norm', True):
            _bn(specs, pre + 'upsample.0.layers.1.', up)
        cse = lay['feature_in_channels'] + lay['skip_in_channels']
        so = lay['skip_out_channels']
        _conv(specs, pre + 'squeeze_excite.0.layers.0.layers.0.', cse, so, 1)
        _bn(specs, pre + 'squeeze_excite.0.layers.1.', so)
        red = so // 16
        specs.append((pre + 'squeeze_excite.1.excite.0.weight', (red, so), 'fc'))
        specs.append((pre + 'squeeze_excite.1.excite.2.weight', (so, red), 'fc'))
        dch = lay.get('disp_channels', 2)
        ci = lay['upsample_channels'] + so + (dch if lay.get('concat_disp', True) else 0)
        _conv(specs, pre + 'iconv.layers.0.layers.0.', ci, lay['out_channels'], 3)
        if lay.get('batch_norm', True):
            _bn(specs, pre + 'iconv.layers.1.', lay['out_channels'])
        if lay.get('calculate_disp', True):
            _conv(specs, pre + 'disp.layers.0.', lay['out_channels'], dch, 3)
    return specs


def disc_param_specs(disc_cfg, graphs) -> List[Tuple[str, tuple, str]]:
    """state_dict schema of reference model/discriminator.py:33-51 (the
    encoder-stage layout of param_specs under ``layers.{s}`` and ``conv``,
    then ``linear``).  ``graphs`` holds one graph per stage incl. the final
    one (stage len(layers) + 1)."""
    specs: List[Tuple[str, tuple, str]] = []
    stages = list(disc_cfg['layers']) + [disc_cfg['final_conv']]
    for s, lay in enumerate(stages):
        base = f'layers.{s}.' if s < len(disc_cfg['layers']) else 'conv.'
        nodes, _, _ = og.graph_info(graphs[s])
        cin, cout, k = lay['in_channels'], lay['out_channels'], lay['kernel_size']
        for node in nodes:
            pre = f'{base}layers.0.node_blocks.{node.id}.'
            if len(node.inputs) > 1:
                specs.append((pre + 'mean_weight', (len(node.inputs),), 'mean_weight'))
            ci = cin if node.node_type == 'input' else cout
            _conv(specs, pre + 'convolution.layers.0.', ci, cout, k)
            _bn(specs, pre + 'convolution.layers.1.', cout)
        for nm in ('keys', 'queries', 'values', 'reprojection'):
            _conv(specs, f'{base}layers.1.{nm}.', cout, cout, 1)
    specs.append(('linear.weight', (1, disc_cfg['linear_in_features']), 'fc'))
    specs.append(('linear.bias', (1,), 'conv_bias'))
    return specs


def _formula(name: str, n: int, lo: float, hi: float) -> torch.Tensor:
    """Deterministic values in [lo, hi] from (name, index): a low-discrepancy
    sine sequence keyed by crc32(name)."""
    h = zlib.crc32(name.encode())
    a = 0.6180339887 + (h % 997) / 997.0 * 0.3
    b = (h >> 10) % 1000 / 1000.0 * 6.28318
    i = torch.arange(n, dtype=torch.float64)
    u = 0.5 + 0.5 * torch.sin(i * a * 12.9898 + b + i * i * 1e-4)
    return (lo + (hi - lo) * u).to(torch.float32)


def formula_state_dict(specs) -> "OrderedDict[str, torch.Tensor]":
    sd = OrderedDict()
    for name, shape, kind in specs:
        n = int(math.prod(shape)) if shape else 1
        if kind == 'conv':
            fan_in = shape[1] * shape[2] * shape[3]
            fan_out = shape[0] * shape[2] * shape[3]
            bnd = math.sqrt(6.0 / (fan_in + fan_out))
            v = _formula(name, n, -bnd, bnd)
        elif kind == 'fc':
            bnd = 1.0 / math.sqrt(shape[1])
            v = _formula(name, n, -bnd, bnd)
        elif kind == 'conv_bias':
            v = _formula(name, n, -0.05, 0.05)
        elif kind == 'bn_weight':
            v = _formula(name, n, 0.8, 1.2)
        elif kind == 'bn_bias':
            v = _formula(name, n, -0.1, 0.1)
        elif kind == 'running_mean':
            v = torch.zeros(n)
        elif kind == 'running_var':
            v = torch.ones(n)
        elif kind == 'mean_weight':
            v = _formula(name, n, 0.0, 2.0)
        elif kind == 'nbt':
            sd[name] = torch.tensor(0, dtype=torch.long)
            continue
        else:
            raise ValueError(kind)
        sd[name] = v.reshape(shape).clone()
    return sd


def adam_update(params: Dict[str, torch.Tensor], grads: Dict[str, torch.Tensor],
                state: Dict, lr: float, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam single-tensor semantics (no weight decay, no amsgrad)."""
    b1, b2 = betas
    step = state.setdefault('step', 0) + 1
    state['step'] = step
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    with torch.no_grad():
        for k, p in params.items():
            g = grads.get(k)
            if g is None:
                continue
            m = state.setdefault('m.' + k, torch.zeros_like(p))
            v = state.setdefault('v.' + k, torch.zeros_like(p))
            m.mul_(b1).add_(g, alpha=1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
            p.addcdiv_(m, denom, value=-lr / bc1)


def train_step(P: Dict[str, torch.Tensor], left, right, scale, model_cfg, loss_cfg,
               graphs, adam_state: Dict, lr: float = 1e-4, scales: int = 4):
    """train/train.py:116-129.  ``P`` holds trainable params (float tensors)
    and BN buffers; params are updated in place.  Returns a dict with the loss
    scalars, per-term values and the gradients."""
    trainable = {k: v for k, v in P.items()
                 if v.is_floating_point() and 'running_' not in k}
    for v in trainable.values():
        v.requires_grad_(True)
        v.grad = None
    images = torch.cat([left, right], 1)
    pyr = L.scale_pyramid(images, scales)
    disps = M.model_forward(left, P, model_cfg, graphs, scale, training=True)
    recon = L.reconstruct_pyramid(disps, pyr)
    dl, el, terms = L.total_loss(pyr, disps, recon, loss_cfg)
    (dl + el).backward()
    grads = {k: v.grad.detach().clone() for k, v in trainable.items() if v.grad is not None}
    for v in trainable.values():
        v.requires_grad_(False)
    adam_update(trainable, grads, adam_state, lr)
    return {'disp_loss': float(dl.detach()), 'error_loss': float(el.detach()),
            'terms': {k: float(v.detach()) if torch.is_tensor(v) else float(v) for k, v in terms.items()},
            'grads': grads, 'disps': [d.detach() for d in disps]}


SKETCHES = 8


def grad_sketch(name: str, g: torch.Tensor, k: int = SKETCHES) -> torch.Tensor:
    """k Rademacher projections <g, r_j> of one gradient tensor, r_j in
    {-1,+1}^numel drawn from a CPU generator seeded by (crc32(name), j): a
    direction-sensitive fingerprint (a wrong direction with the right norm
    changes it) that goldens can store in 8 doubles per parameter.
    ||sketch(g) - sketch(g_ref)|| / ||sketch(g_ref)|| estimates the rel-norm
    ||g - g_ref|| / ||g_ref||."""
    x = g.detach().to('cpu', torch.float64).reshape(-1)
    base = zlib.crc32(name.encode())
    out = torch.empty(k, dtype=torch.float64)
    for j in range(k):
        gen = torch.Generator().manual_seed(base * 16 + j)
        r = torch.randint(0, 2, (x.numel(),), generator=gen, dtype=torch.int8)
        out[j] = (x * (r.to(torch.float64) * 2 - 1)).sum()
    return out


def bench_inputs(batch: int, height: int, width: int, seed: int = 1234):
    """the bench's synthetic pair (bench.py: U[0,1) from a CPU generator)"""
    g = torch.Generator(device='cpu').manual_seed(seed)
    left = torch.rand(batch, 3, height, width, generator=g)
    right = torch.rand(batch, 3, height, width, generator=g)
    return left, right
