"""Probe: umamd.gradsync.GradBuckets with one-parameter buckets on a one-rank
'nccl' group, eager and captured, against a plain backward.
  python tools/ddp_tiny_probe.py OVERLAP(0/1) CAPTURE(0/1) [MODE]
MODE: noar (skip the all-reduce), nohook (launch every bucket in finish),
big (16 MB buckets)."""
import os
import socket
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (os.path.join(REPO, 'uncertainty-model_amd'), REPO, os.path.join(REPO, 'tests')):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ov_on, cap_on = sys.argv[1] == '1', sys.argv[2] == '1'
    from test_gpu_model import _cfg, _model, _uniform_pair
    from train.loss import TukraUncertaintyLoss
    import train.utils as u
    from umamd import lossfn as LF, rccl
    from umamd.gradsync import GradBuckets
    from umamd.overlap import WgradStream
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1)
    cfg = _cfg()
    cfg['loss']['error_loss_config']['loss_type'] = 'l1'
    left, right = _uniform_pair(2, 64, 128)
    left, right = left.cuda(), right.cuda()
    lf = TukraUncertaintyLoss(**cfg['loss'])
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        m = _model(cfg).train()
    torch.cuda.synchronize()
    named = [(k, p) for k, p in m.named_parameters()]
    params = [p for _, p in named]
    mode = sys.argv[3] if len(sys.argv) > 3 else ''
    gb = GradBuckets(params, dist.group.WORLD, 1, cap_mb=16 if mode == 'big' else 1e-6)
    if mode == 'noar':
        rccl.Comm.all_reduce = lambda self, t, average=False: None
    if mode == 'nohook':
        GradBuckets._hook = lambda self, p: None
    if mode == 'same':  # pack on the launch stream itself: no fork
        def same(self, bi):
            self.launched.add(bi)
            b = self.buckets[bi]
            off, n = self.slices[bi]
            grads = [p.grad for p in b]
            self.raw += grads
            torch.cat([g.reshape(-1) for g in grads], out=self.flat[off:off + n])
        GradBuckets._launch = same
    if mode == 'clone':  # fork, but the comm stream copies a clone made on the launch stream
        def clone(self, bi):
            self.launched.add(bi)
            b = self.buckets[bi]
            off, n = self.slices[bi]
            grads = [p.grad.clone() for p in b]
            self.raw += grads
            from umamd import overlap as O
            O.stream_wait(self.stream, torch.cuda.current_stream(), self._events)
            with torch.cuda.stream(self.stream):
                torch.cat([g.reshape(-1) for g in grads], out=self.flat[off:off + n])
        GradBuckets._launch = clone
    if mode in ('evlate', 'fin'):
        PEND = []

        def late(self, bi):
            self.launched.add(bi)
            b = self.buckets[bi]
            off, n = self.slices[bi]
            grads = [p.grad for p in b]
            self.raw += grads
            ev = None
            if mode == 'evlate':  # event at hook time, fork at finish
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream())
            PEND.append((ev, grads, off, n))
        GradBuckets._launch = late
        of = GradBuckets.finish

        def fin2(self):
            cur = torch.cuda.current_stream()
            for ev, grads, off, n in PEND:
                if ev is None:
                    ev = torch.cuda.Event()
                    ev.record(cur)
                self.stream.wait_event(ev)
                self._events.append(ev)
                with torch.cuda.stream(self.stream):
                    torch.cat([g_.reshape(-1) for g_ in grads], out=self.flat[off:off + n])
            PEND.clear()
            return of(self)
        GradBuckets.finish = fin2
    if mode in ('evmid', 'midclone2', 'midcopy'):
        Q = []

        def mid(self, bi):
            self.launched.add(bi)
            b = self.buckets[bi]
            off, n = self.slices[bi]
            grads = [p.grad for p in b]
            self.raw += grads
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            self._events.append(ev)
            Q.append((ev, grads, off, n))
            take = Q[:-1] if mode == 'evmid' else Q[:]
            for e_, gs, o_, n_ in take:
                self.stream.wait_event(e_)
                with torch.cuda.stream(self.stream):
                    if mode == 'midclone2':
                        gs = [g_.clone() for g_ in gs]
                        self.raw += gs
                    if mode == 'midcopy':
                        self.flat[o_:o_ + n_].copy_(gs[0].reshape(-1))
                    else:
                        torch.cat([g_.reshape(-1) for g_ in gs], out=self.flat[o_:o_ + n_])
            del Q[:len(take)]
        GradBuckets._launch = mid
        of2 = GradBuckets.finish

        def fin3(self):
            for e_, gs, o_, n_ in Q:
                self.stream.wait_event(e_)
                with torch.cuda.stream(self.stream):
                    torch.cat([g_.reshape(-1) for g_ in gs], out=self.flat[o_:o_ + n_])
            Q.clear()
            return of2(self)
        GradBuckets.finish = fin3
    if mode in ('rec', 'hold'):
        HOLD = []

        def rec(self, bi):
            self.launched.add(bi)
            b = self.buckets[bi]
            off, n = self.slices[bi]
            grads = [p.grad for p in b]
            self.raw += grads
            HOLD.extend(grads)
            from umamd import overlap as O
            O.stream_wait(self.stream, torch.cuda.current_stream(), self._events)
            if mode == 'rec':
                for g_ in grads:
                    g_.record_stream(self.stream)
            with torch.cuda.stream(self.stream):
                torch.cat([g_.reshape(-1) for g_ in grads], out=self.flat[off:off + n])
        GradBuckets._launch = rec
    import threading
    orig_launch = GradBuckets._launch
    log = []

    order = {}

    def spy(self, bi):
        if gb_capturing[0]:
            order[bi] = (len(order), torch.cuda.current_stream().cuda_stream == st.cuda_stream,
                         torch.cuda.is_current_stream_capturing())
        cap = torch.cuda.is_current_stream_capturing()
        if cap and len(log) < 6:
            cur = torch.cuda.current_stream()
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                joined = torch.cuda.is_current_stream_capturing()
            log.append((bi, threading.current_thread().name, cur.cuda_stream == st.cuda_stream,
                        joined))
        elif not cap and torch.cuda.is_available() and len(log) < 12 and gb_capturing[0]:
            log.append((bi, threading.current_thread().name, 'NOT CAPTURING',
                        torch.cuda.current_stream().cuda_stream == st.cuda_stream))
        return orig_launch(self, bi)
    gb_capturing = [False]
    in_finish = [False]
    if mode not in ('same', 'clone', 'rec', 'hold', 'evlate', 'fin', 'evmid', 'midclone2', 'midcopy'):
        GradBuckets._launch = spy
    orig_finish = GradBuckets.finish

    def fin(self):
        in_finish[0] = True
        try:
            return orig_finish(self)
        finally:
            in_finish[0] = False
    GradBuckets.finish = fin
    comms = rccl.comms_for(dist.group.WORLD)
    ov = WgradStream(params) if ov_on else None

    def fwd_bwd(use_buckets):
        pyr = u.scale_pyramid(torch.cat([left, right], 1), 4)
        d = m(left, 0.3)
        with LF.deferred_recon():
            rec = u.reconstruct_pyramid(d, pyr)
        dl, el = lf(pyr, d, rec, 0, None)
        if ov is not None:
            with ov:
                if use_buckets:
                    gb.arm()
                (dl + el).backward()
        else:
            if use_buckets:
                gb.arm()
            (dl + el).backward()
        if use_buckets:
            gb.finish()

    with torch.cuda.stream(st), rccl.use(comms):
        # reference gradients: plain backward (BN batch stats: same every step,
        # no optimiser step is taken)
        for p in params:
            p.grad = None
        fwd_bwd(False)
        torch.cuda.synchronize()
        ref = [p.grad.detach().clone() for p in params]
        for i in range(2):  # first: layout; second: hook-launched buckets
            for p in params:
                p.grad = None
            fwd_bwd(True)
        torch.cuda.synchronize()
        eager = [p.grad.detach().clone() for p in params]
        print('buckets', len(gb.buckets), 'launched in backward', len(gb.launched), flush=True)
        if cap_on:
            for p in params:
                p.grad = None
            g = torch.cuda.CUDAGraph()
            gb_capturing[0] = True
            with torch.cuda.graph(g, stream=st, capture_error_mode='thread_local'):
                fwd_bwd(True)
            gb_capturing[0] = False
            for e in log:
                print('LAUNCH', e, flush=True)
            g.replay()
            torch.cuda.synchronize()
            capd = [p.grad.detach().clone() for p in params]
    bad_e = bad_c = 0
    for j, (k, _) in enumerate(named):
        r = float(ref[j].norm()) + 1e-12
        de = float((eager[j] - ref[j]).norm()) / r
        if de > 1e-3:
            bad_e += 1
            if bad_e <= 5:
                print('EAGER', k, de, flush=True)
        if cap_on:
            dc = float((capd[j] - ref[j]).norm()) / r
            if dc > 1e-3:
                bad_c += 1
                if bad_c <= 5:
                    print('CAPT', k, dc, float(capd[j].norm()), r, flush=True)
    print('bad eager', bad_e, 'bad captured', bad_c, 'of', len(named), flush=True)
    if cap_on:
        for j, (k, p) in enumerate(named):
            bi = gb.of.get(id(p))
            r = float(ref[j].norm()) + 1e-12
            dc = float((capd[j] - ref[j]).norm()) / r
            print('P', j, k, 'bucket', bi, 'launch', order.get(bi), 'BAD' if dc > 1e-3 else 'ok',
                  flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
