"""Probe: for every GraphBlock node whose BN-backward sums the merge backward
took (um_merge_bwd_bn), recompute them with um_bn_elu_bwd_reduce_slots into
a zeroed buffer and compare.  python tools/merge_bn_probe.py [fp32|bf16]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (os.path.join(REPO, 'uncertainty-model_amd'), REPO, os.path.join(REPO, 'tests')):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    dtype = sys.argv[1] if len(sys.argv) > 1 else 'fp32'
    from test_gpu_model import _cfg, _model, _uniform_pair
    from umamd import functional as U
    from umamd import _lib as L
    from umamd._lib import call, ptr
    orig = U._cbe_bwd

    def probe(ctx, da, *args, **kw):
        if ctx.prereduced and ctx.slots_b is not None:
            x, wT, y, mean, invstd, scale, shift = ctx.saved[:7]
            N, H, W, Cp, K, Creal, R, P, Q = ctx.geom
            M = N * P * Q
            ref = torch.zeros_like(ctx.slots_b)
            dd = da.contiguous()
            call('um_bn_elu_bwd_reduce_slots', U._ydt(dd, y), M, K, P * Q, ptr(dd), K, ptr(y), K,
                 ptr(mean), ptr(invstd), ptr(scale), ptr(shift), None, int(ctx.spec.elu), ptr(ref))
            torch.cuda.synchronize()
            n = L.STAT_SLOTS * K * 2
            got = ctx.slots_b[:n].view(L.STAT_SLOTS, K, 2).sum(0)
            want = ref[:n].view(L.STAT_SLOTS, K, 2).sum(0)
            rel = float((got - want).abs().max() / (want.abs().max() + 1e-30))
            print(f'node K={K} M={M}: slots rel {rel:.3e}  got[0]={got[0].tolist()} want[0]={want[0].tolist()} '
                  f'count got {float(ctx.slots_b[n]):.0f} want {float(ref[n]):.0f}', flush=True)
        return orig(ctx, da, *args, **kw)
    U._cbe_bwd = probe
    cfg = _cfg('config.yml')
    left, _ = _uniform_pair(2, 64, 128, seed=7)
    m = _model(cfg, dtype).train()
    d = m(left.cuda(), 0.3)
    (sum((t.float() ** 2).mean() for t in d)).backward()
    torch.cuda.synchronize()


if __name__ == '__main__':
    main()
