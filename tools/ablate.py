#!/usr/bin/env python3
"""Ablation timing of the captured bench step (measurement aid, not a
product path): the C-ABI entries of the named groups are skipped (their
outputs stay uninitialised, so the numbers are meaningless; only the step
time is read), showing how much of the step each group holds on the
critical path.  Usage:  python tools/ablate.py GROUP[,GROUP...] [bench args]
Groups: see GROUPS."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, 'uncertainty-model_amd'), REPO):
    sys.path.insert(0, p)

GROUPS = {
    'none': (),
    'wgrad': ('um_conv2d_wgrad', 'um_conv_wgrad_reduce_seg', 'um_colsum', 'um_colsum_batch',
              'um_reduce_rows', 'um_merge_wgrad_batch', 'um_merge_wgrad'),
    'wred': ('um_conv_wgrad_reduce_seg',),
    'bnfwd': ('um_bn_elu_fwd_slots', 'um_bn_elu_fwd_slots_merge'),
    'bnbwd': ('um_bn_elu_bwd_reduce_slots', 'um_bn_elu_bwd_apply_slots', 'um_merge_bwd_bn'),
    'loss': ('um_loss_fwd', 'um_loss_bwd'),
    'cat': ('um_concat_build', 'um_concat_bwd_src'),
    'attn': ('um_attn_fwd', 'um_attn_bwd'),
    'adam': ('um_adam_step_dev', 'um_adam_step'),
}


def main():
    groups = sys.argv[1].split(',')
    skip = set()
    for g in groups:
        skip |= set(GROUPS[g])
    sys.argv = [sys.argv[0]] + sys.argv[2:]
    from umamd import _lib as L
    from umamd import functional as F
    orig = L.call

    def call(name, *args, work=None):
        if name in skip:
            return None
        return orig(name, *args, work=work)
    L.call = call
    F.call = call
    import umamd.lossfn as LF
    LF.call = call
    import bench
    bench.main()


if __name__ == '__main__':
    main()
