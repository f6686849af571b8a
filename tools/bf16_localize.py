#!/usr/bin/env python3
"""Where the bf16 build's step-0 loss deviation comes from (GPU).

Inputs: tests/test_gpu_model.py's U[0,1) pair (B=2, 64x128, seed 99) and the
config-2 shape pair (B=8, 256x512, seed 99), formula weights, bayesian loss.
Arms, each against the fp32 build:
  bf16            the bench build
  fp32+w16[sel]   the fp32 build with the conv weights of ``sel`` rounded to
                  bf16 (weight rounding alone, no activation rounding)
Prints the relative loss deltas and, per disparity scale, the relative
deviation of the mean uncertainty sigma (channels 2-3) and disparity (0-1).

    python tools/bf16_localize.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, 'uncertainty-model_amd'), REPO, os.path.join(REPO, 'tests')):
    sys.path.insert(0, p)

import torch  # noqa: E402

DEV = 'cuda'


def run(cfg, dtype, left, right, sd_mod=None):
    import train.utils as u
    from test_gpu_model import _model
    from train.loss import TukraUncertaintyLoss
    m = _model(cfg, dtype).train()
    if sd_mod is not None:
        sd = m.state_dict()
        with torch.no_grad():
            for k, v in sd.items():
                if sd_mod(k, v):
                    v.copy_(v.to(torch.bfloat16).float())
    lf = TukraUncertaintyLoss(**cfg['loss'])
    pyr = u.scale_pyramid(torch.cat([left, right], 1), 4)
    with torch.no_grad():
        d = m(left, 0.3)
        dl, el = lf(pyr, d, u.reconstruct_pyramid(d, pyr), 0, None)
    torch.cuda.synchronize()
    stats = [(float(x[:, 0:2].double().mean()), float(x[:, 2:4].double().mean())) for x in d]
    return float(dl), float(el), stats


def f32_tail_patch(on):
    """bf16 model arm: each decoder stage's iconv (on its bf16-rounded
    concat input) and disparity head run in f32, the stage output rounded to
    bf16 for the next stage -- isolates the head-input activation rounding"""
    from model.layers import decoder as D
    from umamd import functional as U
    from umamd._lib import CAT_COPY, CAT_PSHUF, CAT_UP2
    if not hasattr(D.DecoderStage, '_orig_fwd'):
        D.DecoderStage._orig_fwd = D.DecoderStage._fwd
    if not on:
        D.DecoderStage._fwd = D.DecoderStage._orig_fwd
        return

    def _fwd(self, x, feature_map, skip, disparity=None, scale=1.0):
        N, H, W, _ = feature_map.shape
        dtype = x.dtype
        skip_t, skip_g = skip if isinstance(skip, tuple) else (skip, None)
        se_block = self.squeeze_excite[0]
        u1, gate = U.skip_conv_bn_elu(feature_map, skip_t, skip_g, se_block.layers[0].layers[0],
                                      se_block.layers[1], self.squeeze_excite[1],
                                      self.feature_in_channels, self.skip_in_channels)
        xu = self.upsample[0]._fwd(x)
        srcs = [U.CatSource(xu, CAT_PSHUF, self.upsample_channels),
                U.CatSource(u1, CAT_COPY, self.skip_out_channels, gate)]
        if self.concat_disp:
            srcs.append(U.CatSource(disparity, CAT_UP2, self.disp_channels))
        cat2, segs2 = U.concat(srcs, N, H, W, dtype)
        out = self.iconv._fwd(cat2.float(), segs=segs2)
        disp = U.disp_head(out, self.disp.layers[0], scale) if self.calculate_disp else None
        return out.to(dtype), (u1, gate), disp
    D.DecoderStage._fwd = _fwd


def split_patch(mode):
    """bf16 model arm: 'enc32' runs the encoder in f32 (features rounded to
    bf16 for the decoder), 'dec32' the decoder in f32 on the bf16 encoder's
    features; None restores the model"""
    from model import model as MM
    from umamd import functional as U
    from umamd import packer as P
    if not hasattr(MM.RandomlyConnectedModel, '_orig_forward'):
        MM.RandomlyConnectedModel._orig_forward = MM.RandomlyConnectedModel.forward
    if mode is None:
        MM.RandomlyConnectedModel.forward = MM.RandomlyConnectedModel._orig_forward
        return

    def forward(self, image, scale=1):
        x16 = U.image_to_nhwc(image, torch.bfloat16)
        x32 = U.image_to_nhwc(image, torch.float32)
        with P.scope(self._packer), U.stat_scope(self._stats, x16.device), U.grad_slots():
            if mode == 'enc32':
                feats = [f.to(torch.bfloat16) for f in self.encoder._fwd(x32)]
                disps = self.decoder._fwd(x16, *feats, scale=float(scale))
            else:
                feats = [f.float() for f in self.encoder._fwd(x16)]
                disps = self.decoder._fwd(x32, *feats, scale=float(scale))
        disps = tuple(d.permute(0, 3, 1, 2) for d in disps)
        return disps
    MM.RandomlyConnectedModel.forward = forward


def stage_patch(k):
    """bf16 model arm: encoder stage k (0..4) runs in f32 on its
    bf16-rounded input, its output rounded back to bf16; None restores"""
    from model import encoder as E
    if not hasattr(E.RandomEncoder, '_orig_fwd'):
        E.RandomEncoder._orig_fwd = E.RandomEncoder._fwd
    if k is None:
        E.RandomEncoder._fwd = E.RandomEncoder._orig_fwd
        return

    def _fwd(self, x):
        enc = []
        for i, layer in enumerate(self.layers):
            x = layer._fwd(x.float()).to(x.dtype) if i == k else layer._fwd(x)
            enc.append(x)
        return tuple(enc)
    E.RandomEncoder._fwd = _fwd


def main():
    from test_gpu_model import _cfg, _uniform_pair
    cfg = _cfg()
    cfg['loss']['error_loss_config']['loss_type'] = 'bayesian'
    conv_w = lambda k, v: v.dim() == 4  # noqa: E731
    sels = {
        'all conv weights': conv_w,
        'encoder convs': lambda k, v: v.dim() == 4 and k.startswith('encoder'),
        'decoder convs': lambda k, v: v.dim() == 4 and k.startswith('decoder'),
        'decoder non-head convs': lambda k, v: v.dim() == 4 and k.startswith('decoder')
        and '.disp.' not in k,
        'all params': lambda k, v: v.is_floating_point() and 'running' not in k,
    }
    for (b, h, w) in ((2, 64, 128), (8, 256, 512)):
        left, right = [t.to(DEV) for t in _uniform_pair(b, h, w, seed=99)]
        base = run(cfg, 'fp32', left, right)
        print(f'== B={b} {h}x{w}: fp32 losses {base[0]:.6f} {base[1]:.6f}', flush=True)

        def report(name, r):
            dd, de = r[0] / base[0] - 1, r[1] / base[1] - 1
            sc = ' '.join(f's{i}: d{a[0] / bb[0] - 1:+.2e} sig{a[1] / bb[1] - 1:+.2e}'
                          for i, (a, bb) in enumerate(zip(r[2], base[2])))
            print(f'{name:28s} disp {dd:+.3e} err {de:+.3e} | {sc}', flush=True)
        report('bf16', run(cfg, 'bf16', left, right))
        f32_tail_patch(True)
        report('bf16, iconv+head f32', run(cfg, 'bf16', left, right))
        f32_tail_patch(False)
        for mode in ('enc32', 'dec32'):
            split_patch(mode)
            report('bf16, ' + mode, run(cfg, 'bf16', left, right))
            split_patch(None)
        for k in range(5):
            stage_patch(k)
            report(f'bf16, enc stage {k} f32', run(cfg, 'bf16', left, right))
            stage_patch(None)
        if os.environ.get('LOC_WEIGHTS'):
            for name, sel in sels.items():
                report('fp32+w16 ' + name, run(cfg, 'fp32', left, right, sel))


if __name__ == '__main__':
    main()
