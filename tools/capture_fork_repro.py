"""Repro: many fork/join pairs between two streams inside one HIP graph
capture, from the capturing thread or from a worker thread (as autograd's
device thread does for post-accumulate-grad hooks).
  python tools/capture_fork_repro.py N THREAD(0/1) MODE(global|thread_local)"""
import sys
import threading

import torch


def main():
    n, from_thread, mode = int(sys.argv[1]), sys.argv[2] == '1', sys.argv[3]
    dev = torch.device('cuda', 0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    src = [torch.zeros(4096, device=dev) for _ in range(n)]
    dst = torch.zeros(n, 4096, device=dev)
    keep = []
    torch.cuda.synchronize()

    def body():
        for i in range(n):
            with torch.cuda.stream(s1):
                src[i].fill_(float(i + 1))      # the "gradient" producer
                src[i].mul_(2.0)
                ev = torch.cuda.Event()
                ev.record(s1)
            s2.wait_event(ev)
            keep.append(ev)
            with torch.cuda.stream(s2):
                dst[i].copy_(src[i])            # the "bucket pack"
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s1, capture_error_mode=mode):
        if from_thread:
            t = threading.Thread(target=body)
            t.start()
            t.join()
        else:
            body()
        s1.wait_stream(s2)
    for s in src:
        s.zero_()
    dst.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    want = torch.arange(1, n + 1, device=dev, dtype=torch.float32)[:, None] * 2.0
    bad = int((dst != want).any(1).sum())
    print(f'n={n} thread={from_thread} mode={mode}: bad rows {bad} of {n}', flush=True)


if __name__ == '__main__':
    main()
