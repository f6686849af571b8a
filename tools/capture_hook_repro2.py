"""Repro 2: as capture_hook_repro.py, but each parameter gradient's final
value is written by a libumamd kernel (um_axpy) inside a custom autograd
Function, as the model's HIP ops do.
  python tools/capture_hook_repro2.py NLAYERS USE_UMAMD(0/1)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'uncertainty-model_amd'))

import torch  # noqa: E402


class MatFn(torch.autograd.Function):
    use_umamd = True

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        g = x.t() @ dy
        if MatFn.use_umamd:
            from umamd._lib import call, ptr
            gw = torch.zeros_like(w)
            call('um_axpy', 0, gw.numel(), 1.0, ptr(g), ptr(gw))
        else:
            gw = torch.zeros_like(w)
            gw.add_(g)
        return dy @ w.t(), gw


def main():
    n = int(sys.argv[1])
    MatFn.use_umamd = sys.argv[2] == '1'
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s1.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s1):
        ws = [torch.nn.Parameter(torch.randn(64, 64, device=dev) * 0.1) for _ in range(n)]
    flat = torch.zeros(n * 4096, device=dev)
    keep, raw = [], []
    armed = [False]

    def mk(i):
        def hook(p):
            if not armed[0]:
                return
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            s2.wait_event(ev)
            keep.append(ev)
            raw.append(p.grad)
            with torch.cuda.stream(s2):
                flat[i * 4096:(i + 1) * 4096].copy_(p.grad.reshape(-1))
        return hook
    for i, w in enumerate(ws):
        w.register_post_accumulate_grad_hook(mk(i))
    x = torch.randn(32, 64, device=dev)

    def fwd_bwd():
        h = x
        for w in ws:
            h = torch.tanh(MatFn.apply(h, w))
        h.square().mean().backward()
    with torch.cuda.stream(s1):
        fwd_bwd()
    torch.cuda.synchronize()
    ref = torch.cat([w.grad.reshape(-1) for w in ws])
    with torch.cuda.stream(s1):
        for w in ws:
            w.grad = None
    armed[0] = True
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s1, capture_error_mode='thread_local'):
        fwd_bwd()
        s1.wait_stream(s2)
    flat.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    bad = sum(1 for i in range(n) if not torch.allclose(flat[i * 4096:(i + 1) * 4096],
                                                        ref[i * 4096:(i + 1) * 4096],
                                                        rtol=1e-4, atol=1e-6))
    print(f'layers={n} umamd={MatFn.use_umamd}: bad params {bad} of {n}', flush=True)


if __name__ == '__main__':
    main()
