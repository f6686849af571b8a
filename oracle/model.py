"""Functional CPU restatement of the reference model forward -- TEST ORACLE.

Parameters are passed as a flat ``{state_dict name: tensor}`` mapping whose
names are the reference's ``RandomlyConnectedModel.state_dict()`` keys, so the
same formula-generated weights can be loaded into the reference (golden
generation), into this oracle, and into the HIP build.

Reference anchors:
  encoder stage      model/layers/encoder.py:201-262, model/encoder.py:42-53
  node block         model/layers/encoder.py:115-127 (F3 weight mapping)
  conv block         model/layers/encoder.py:21-52 (zero pad, conv, BN, ELU)
  graph block        model/layers/encoder.py:178-198
  attention          model/layers/attention.py:42-76
  decoder            model/decoder.py:34-62, model/layers/decoder.py:11-249
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import torch
import torch.nn.functional as F

from . import graph as og

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


BN_EPS = 1e-5
BN_MOMENTUM = 0.1


def batch_norm_train(x: torch.Tensor, P: Dict[str, torch.Tensor], pre: str,
                     update: bool = True) -> torch.Tensor:
    """nn.BatchNorm2d in training mode (torch semantics, eps 1e-5, momentum
    0.1): normalise with the biased batch variance, update running stats with
    the unbiased one."""
    n = x.numel() / x.shape[1]
    mean = x.mean(dim=(0, 2, 3))
    var_b = x.var(dim=(0, 2, 3), unbiased=False)
    if update and (pre + 'running_mean') in P:
        with torch.no_grad():
            var_u = var_b * (n / max(n - 1, 1))
            P[pre + 'running_mean'].mul_(1 - BN_MOMENTUM).add_(BN_MOMENTUM * mean)
            P[pre + 'running_var'].mul_(1 - BN_MOMENTUM).add_(BN_MOMENTUM * var_u)
            P[pre + 'num_batches_tracked'].add_(1)
    xh = (x - mean[None, :, None, None]) / torch.sqrt(var_b[None, :, None, None] + BN_EPS)
    return xh * P[pre + 'weight'][None, :, None, None] + P[pre + 'bias'][None, :, None, None]


def batch_norm_eval(x, P, pre):
    rm, rv = P[pre + 'running_mean'], P[pre + 'running_var']
    xh = (x - rm[None, :, None, None]) / torch.sqrt(rv[None, :, None, None] + BN_EPS)
    return xh * P[pre + 'weight'][None, :, None, None] + P[pre + 'bias'][None, :, None, None]


def bn(x, P, pre, training):
    return batch_norm_train(x, P, pre) if training else batch_norm_eval(x, P, pre)


# ----------------------------------------------------------------- encoder --
def enc_conv_block(x, P, pre, k, stride, training):
    """Zero pad (k-1)/2 -> Conv2d(k, stride, bias) -> BN -> ELU
    (model/layers/encoder.py:21-52)."""
    p = (k - 1) // 2
    y = F.conv2d(F.pad(x, (p, p, p, p)), P[pre + 'layers.0.weight'],
                 P[pre + 'layers.0.bias'], stride=stride)
    return F.elu(bn(y, P, pre + 'layers.1.', training))


def node_merge(inputs: Sequence[torch.Tensor], w: Optional[torch.Tensor]):
    """Sigmoid-weighted predecessor merge (model/layers/encoder.py:115-124).

    F3: the first input is weighted by sigmoid(w[0]) and input i+1 by
    sigmoid(w[i]) -- input 1 reuses w[0], the last weight is never used."""
    if len(inputs) <= 1:
        return inputs[0]
    out = torch.sigmoid(w[0]) * inputs[0]
    for i, x in enumerate(inputs[1:]):
        out = out + torch.sigmoid(w[i]) * x
    return out


def graph_block(x, P, pre, graph, kernel, training):
    """Evaluate the DAG in id order; average the output nodes
    (model/layers/encoder.py:178-198; out-of-place sum)."""
    nodes, in_nodes, out_nodes = og.graph_info(graph)
    res = {}
    for idx in in_nodes:
        res[idx] = enc_conv_block(x, P, f'{pre}node_blocks.{idx}.convolution.',
                                  kernel, 2, training)
    for node in nodes:
        if node.id in in_nodes:
            continue
        ins = [res[i] for i in node.inputs]
        w = P.get(f'{pre}node_blocks.{node.id}.mean_weight')
        m = node_merge(ins, w)
        res[node.id] = enc_conv_block(m, P, f'{pre}node_blocks.{node.id}.convolution.',
                                      kernel, 1, training)
    out = res[out_nodes[0]]
    for idx in out_nodes[1:]:
        out = out + res[idx]
    return out / len(out_nodes)


def efficient_attention(x, P, pre, heads):
    """Linear attention (model/layers/attention.py:42-76): softmax(K) over
    pixels, softmax(Q) over the head's channels, ctx = K V^T, out = ctx^T Q,
    1x1 reprojection + residual."""
    b, c, h, w = x.shape
    s = h * w
    K = F.conv2d(x, P[pre + 'keys.weight'], P[pre + 'keys.bias']).reshape(b, c, s)
    Q = F.conv2d(x, P[pre + 'queries.weight'], P[pre + 'queries.bias']).reshape(b, c, s)
    V = F.conv2d(x, P[pre + 'values.weight'], P[pre + 'values.bias']).reshape(b, c, s)
    d = c // heads
    outs = []
    for i in range(heads):
        sl = slice(i * d, (i + 1) * d)
        k = torch.softmax(K[:, sl], dim=2)
        q = torch.softmax(Q[:, sl], dim=1)
        ctx = torch.bmm(k, V[:, sl].transpose(1, 2))
        outs.append(torch.bmm(ctx.transpose(1, 2), q).reshape(b, d, h, w))
    att = torch.cat(outs, dim=1)
    return F.conv2d(att, P[pre + 'reprojection.weight'], P[pre + 'reprojection.bias']) + x


def encoder_forward(x, P, enc_cfg, graphs, training=True):
    """RandomEncoder.forward (model/encoder.py:42-53)."""
    feats = []
    for s, layer in enumerate(enc_cfg['layers']):
        pre = f'encoder.layers.{s}.layers.'
        x = graph_block(x, P, pre + '0.', graphs[s], layer['kernel_size'], training)
        x = efficient_attention(x, P, pre + '1.', layer.get('heads', 8))
        feats.append(x)
    return feats


def load_stage_graphs(enc_cfg, root: Optional[str] = None):
    """Graphs per stage (model/layers/encoder.py:237-242), read from the repo's
    JSON adjacency files; ``load_graph: None`` maps to the committed
    ``graphs/nodes_{n}_seed_{seed}`` files (generated by networkx 3.4.2's
    connected_watts_strogatz_graph(n, 4, 0.75, seed=stage*seed))."""
    d = enc_cfg.get('load_graph') or \
        f"graphs/nodes_{enc_cfg.get('nodes', 5)}_seed_{enc_cfg.get('seed', 42)}"
    if not os.path.isabs(d):
        d = os.path.join(root or REPO, d)
    return [og.load_json(os.path.join(d, f'stage_{s + 1}.json'))
            for s in range(len(enc_cfg['layers']))]


# ----------------------------------------------------------------- decoder --
def up2(x):
    """F.interpolate(scale_factor=2, bilinear, align_corners=True)."""
    return F.interpolate(x, scale_factor=2, mode='bilinear', align_corners=True)


def dec_conv(x, P, pre, reflect_pad: bool, sigmoid=False):
    """ConvLayer: optional reflect pad 1, conv, optional sigmoid
    (model/layers/decoder.py:11-52)."""
    if reflect_pad:
        x = F.pad(x, (1, 1, 1, 1), mode='reflect')
    y = F.conv2d(x, P[pre + 'layers.0.weight'], P[pre + 'layers.0.bias'])
    return torch.sigmoid(y) if sigmoid else y


def dec_conv_elu(x, P, pre, pad, use_bn, training):
    """ConvELUBlock: ConvLayer -> BN? -> ELU (model/layers/decoder.py:55-87)."""
    y = dec_conv(x, P, pre + 'layers.0.', pad)
    if use_bn:
        y = bn(y, P, pre + 'layers.1.', training)
    return F.elu(y)


def squeeze_excite(x, P, pre):
    """SELayer, fc=True (model/layers/decoder.py:90-136)."""
    b, c = x.shape[:2]
    z = x.mean(dim=(2, 3))
    z = torch.relu(z @ P[pre + 'excite.0.weight'].t())
    z = torch.sigmoid(z @ P[pre + 'excite.2.weight'].t())
    return x * z.view(b, c, 1, 1)


def decoder_stage(x, feat, skip, disp, scale, P, pre, cfg, training):
    """DecoderStage.forward (model/layers/decoder.py:210-249)."""
    use_bn = cfg.get('batch_norm', True)
    skip = up2(skip)
    skip = dec_conv_elu(torch.cat((feat, skip), 1), P, pre + 'squeeze_excite.0.',
                        False, True, training)
    skip = squeeze_excite(skip, P, pre + 'squeeze_excite.1.')
    xu = F.pixel_shuffle(dec_conv_elu(x, P, pre + 'upsample.0.', True, use_bn, training), 2)
    xc = torch.cat((xu, skip), 1)
    if cfg.get('concat_disp', True):
        xc = torch.cat((xc, up2(disp)), 1)
    out = dec_conv_elu(xc, P, pre + 'iconv.', True, use_bn, training)
    d = scale * dec_conv(out, P, pre + 'disp.', True, sigmoid=True) \
        if cfg.get('calculate_disp', True) else None
    return out, skip, d


def decoder_forward(left, feats, P, dec_cfg, scale, training=True):
    """DepthDecoder.forward wiring (model/decoder.py:34-62)."""
    f1, f2, f3, f4, x4 = feats
    L = dec_cfg['layers']
    o5, s5, _ = decoder_stage(x4, f4, x4, None, scale, P, 'decoder.layers.0.', L[0], training)
    o4, s4, d4 = decoder_stage(o5, f3, s5, None, scale, P, 'decoder.layers.1.', L[1], training)
    o3, s3, d3 = decoder_stage(o4, f2, s4, d4, scale, P, 'decoder.layers.2.', L[2], training)
    o2, s2, d2 = decoder_stage(o3, f1, s3, d3, scale, P, 'decoder.layers.3.', L[3], training)
    _, _, d1 = decoder_stage(o2, left, s2, d2, scale, P, 'decoder.layers.4.', L[4], training)
    return (d1, d2, d3, d4) if training else d1


def model_forward(image, P, model_cfg, graphs, scale=1.0, training=True):
    """RandomlyConnectedModel.forward (model/model.py:21-23)."""
    feats = encoder_forward(image, P, model_cfg['encoder'], graphs, training)
    return decoder_forward(image, feats, P, model_cfg['decoder'], scale, training)
