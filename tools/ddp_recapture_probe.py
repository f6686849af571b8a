"""Probe: repeated data-parallel captures on a one-rank 'nccl' group.
  python tools/ddp_recapture_probe.py CAPTURES BUCKET_MB
(UMAMD_CAPTURE_MODE picks the capture mode; progress goes to stdout.)"""
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
    captures, mb = int(sys.argv[1]), sys.argv[2]
    os.environ['UMAMD_GRAD_BUCKET_MB'] = mb
    from test_gpu_model import _cfg, _model, _uniform_pair
    from train.graph import CapturedTrainStep
    from train.loss import TukraUncertaintyLoss
    from train.parallel import data_parallel
    from umamd.functional import BNSync
    from umamd.optim import Adam
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1)
    BNSync.force = True
    cfg = _cfg()
    cfg['loss']['error_loss_config']['loss_type'] = 'l1'
    left, right = _uniform_pair(2, 64, 128)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        m = data_parallel(_model(cfg).train(), 0)
    torch.cuda.current_stream().wait_stream(st)
    opt = Adam(m.parameters(), 1e-4)
    cap = None
    for i in range(captures):
        if cap is not None:
            cap.close()
        print(f'capture {i} start', flush=True)
        cap = CapturedTrainStep(m, TukraUncertaintyLoss(**cfg['loss']), opt, left.cuda(),
                                right.cuda(), 0.3, warmup=1, stream=st)
        print(f'capture {i} ok, buckets {len(cap._buckets.buckets)}', flush=True)
        dl, el = cap()
        torch.cuda.synchronize()
        print(f'replay {i}', float(dl), float(el), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
