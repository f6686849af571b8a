"""Loss-stack micro-benchmark at BASELINE config 2 (B=8, 256x512, 4 scales):
forward and backward launch times (HIP events) for each value of a tuning
knob, smooth (increasing-tap) and per-pixel-noise disparities.
Usage: python tools/loss_scatter_micro.py [knob] [values...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'uncertainty-model_amd'))
from tests.test_gpu_loss_stack import _cfg, _smooth_preds  # noqa: E402
import train.utils as u  # noqa: E402
from train.loss import TukraUncertaintyLoss  # noqa: E402
from umamd import lossfn as LF  # noqa: E402
from umamd._lib import lib  # noqa: E402


def run(preds, imgs, iters=20):
    lf = TukraUncertaintyLoss(**_cfg())
    pyr = u.scale_pyramid(imgs, 4)
    pd = [p.requires_grad_(True) for p in preds]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for it in range(iters + 3):
        with LF.deferred_recon():
            rec = u.reconstruct_pyramid(pd, pyr)
        torch.cuda.synchronize()
        ev[0].record()
        dl, el = lf(pyr, pd, rec, 0, None)
        ev[1].record()
        torch.autograd.grad(dl + el, pd)
        ev[2].record()
        torch.cuda.synchronize()
        if it >= 3:
            tf += ev[0].elapsed_time(ev[1])
            tb += ev[1].elapsed_time(ev[2])
    return tf / iters * 1e3, tb / iters * 1e3


def main():
    knob = sys.argv[1] if len(sys.argv) > 1 else 'loss_scatter'
    vals = [int(v) for v in sys.argv[2:]] or [0, 1]
    g = torch.Generator().manual_seed(1)
    imgs = torch.rand(8, 6, 256, 512, generator=g).cuda()
    cases = {'smooth': [p.cuda() for p in _smooth_preds(8, 256, 512, 2)],
             'noise': [(0.02 + 0.2 * torch.rand(8, 4, 256 >> i, 512 >> i, generator=g)).cuda()
                       for i in range(4)]}
    only = os.environ.get('LOSS_MICRO_CASE')
    if only:
        cases = {only: cases[only]}
    for rep in range(2):
        for v in vals:
            old = lib().um_set_tuning(knob.encode(), v)
            for name, pr in cases.items():
                f, b = run([p.detach().clone() for p in pr], imgs)
                print(f'{knob}={v} {name:6s} fwd {f:7.1f} us  bwd {b:7.1f} us', flush=True)
            lib().um_set_tuning(knob.encode(), old)


if __name__ == '__main__':
    main()
