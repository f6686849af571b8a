"""Probe: capture an RCCL all-reduce of a one-rank 'nccl' group in a HIP
graph (torch.cuda.graph) and replay it.  Usage:
  python tools/rccl_capture_probe.py MODE OP [ASYNC]
MODE: global | thread_local | relaxed; OP: sum | avg; ASYNC: 1 = async_op + wait.
VARIANT (4th arg): plain | f64pool (f64 tensor allocated inside the capture)
| fork (work forked to a second stream around the collective) | many (100
small collectives)."""
import os
import socket
import sys
import time

import torch
import torch.distributed as dist


def main():
    mode, op = sys.argv[1], sys.argv[2]
    use_async = len(sys.argv) > 3 and sys.argv[3] == '1'
    variant = sys.argv[4] if len(sys.argv) > 4 else 'plain'
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1)
    rop = dist.ReduceOp.AVG if op == 'avg' else dist.ReduceOp.SUM
    t = torch.ones(1 << 20, device='cuda')
    dist.all_reduce(t, op=rop)  # communicator init, eager
    torch.cuda.synchronize()
    print('eager ok', float(t[0]), torch.cuda.nccl.version(), flush=True)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        t.mul_(2)
        dist.all_reduce(t, op=rop)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    print('side-stream eager ok', flush=True)
    # let the process group's watchdog retire the eager work: it polls the
    # end events of outstanding work, and HIP refuses that query while the
    # stream they were recorded on is capturing
    time.sleep(float(os.environ.get('PROBE_SLEEP', '0')))
    with torch.cuda.graph(g, stream=side, capture_error_mode=mode):
        t.mul_(2)
        if variant == 'f64pool':
            u = torch.ones(3, 64, dtype=torch.float64, device='cuda') * t[0]
            dist.all_reduce(u)
            t.add_(u.sum().float() - u.sum().float())
        elif variant == 'fork':
            s2 = torch.cuda.Stream()
            s2.wait_stream(side)
            with torch.cuda.stream(s2):
                v = t * 3
            dist.all_reduce(t, op=rop)
            side.wait_stream(s2)
            t.add_(v - v)
        elif variant == 'many':
            for _ in range(100):
                u = torch.ones(2, 32, dtype=torch.float64, device='cuda')
                dist.all_reduce(u)
            dist.all_reduce(t, op=rop)
        elif variant == 'autograd':
            # collective inside a backward: runs on autograd's device thread
            class AR(torch.autograd.Function):
                @staticmethod
                def forward(ctx, x):
                    return x * 1.0

                @staticmethod
                def backward(ctx, gy):
                    gy = gy.clone()
                    dist.all_reduce(gy)
                    return gy
            w = t.detach().clone().requires_grad_(True)
            AR.apply(w).sum().backward()
            t.add_(w.grad - w.grad)
            dist.all_reduce(t, op=rop)
        elif use_async:
            dist.all_reduce(t, op=rop, async_op=True).wait()
        else:
            dist.all_reduce(t, op=rop)
    print('captured', flush=True)
    g.replay()
    torch.cuda.synchronize()
    print('replayed', float(t[0]), flush=True)
    time.sleep(1.0)  # the watchdog polls again after the capture
    g.replay()
    torch.cuda.synchronize()
    print('replayed again', float(t[0]), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
