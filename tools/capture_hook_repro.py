"""Repro: post-accumulate-grad hooks that fork a copy of each parameter's
gradient onto a second stream, inside a captured forward+backward.
  python tools/capture_hook_repro.py NLAYERS MODE(global|thread_local)"""
import sys

import torch


def main():
    n, mode = int(sys.argv[1]), sys.argv[2]
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s1.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s1):
        layers = [torch.nn.Linear(64, 64).to(dev) for _ in range(n)]
    params = [p for l in layers for p in l.parameters()]
    flat = torch.zeros(sum(p.numel() for p in params), device=dev)
    offs, o = {}, 0
    for p in params:
        offs[id(p)] = (o, p.numel())
        o += p.numel()
    keep, raw = [], []
    armed = [False]

    def hook(p):
        if not armed[0]:
            return
        cur = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(cur)
        s2.wait_event(ev)
        keep.append(ev)
        raw.append(p.grad)
        off, k = offs[id(p)]
        with torch.cuda.stream(s2):
            flat[off:off + k].copy_(p.grad.reshape(-1))
    for p in params:
        p.register_post_accumulate_grad_hook(hook)
    x = torch.randn(32, 64, device=dev)

    def fwd_bwd():
        h = x
        for l in layers:
            h = torch.tanh(l(h))
        h.square().mean().backward()
    with torch.cuda.stream(s1):
        for p in params:
            p.grad = None
        fwd_bwd()
    torch.cuda.synchronize()
    ref = torch.cat([p.grad.reshape(-1) for p in params])
    with torch.cuda.stream(s1):
        for p in params:
            p.grad = None
    armed[0] = True
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s1, capture_error_mode=mode):
        fwd_bwd()
        s1.wait_stream(s2)
    flat.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    bad = sum(1 for p in params
              if not torch.allclose(flat[offs[id(p)][0]:offs[id(p)][0] + p.numel()],
                                    ref[offs[id(p)][0]:offs[id(p)][0] + p.numel()],
                                    rtol=1e-4, atol=1e-6))
    print(f'layers={n} mode={mode}: bad params {bad} of {len(params)}', flush=True)


if __name__ == '__main__':
    main()
