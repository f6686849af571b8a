#!/usr/bin/env python3
"""Benchmark: stereo-pairs/sec of the self-supervised depth+uncertainty
training step (BASELINE.json metric) at 256x512, batch 8 per GPU, bayesian
error loss, bf16 compute (BASELINE config 2 / config 4 per-GPU shape).

A step = reference train/train.py:116-129 on synthetic device-resident U[0,1)
pairs: image pyramid -> model forward -> reconstruct -> 4-scale loss ->
backward -> Adam.  N>1: one process per GPU (torchrun), DDP over RCCL with
SyncBatchNorm semantics (reference parallel_main.py:156-158), weak scaling.

Prints ONE JSON line (rank 0) with a ``roofline`` object for the dominant
kernel (measured with HIP events around its launches on the launch stream)
and a ``cpu_baseline`` (the oracle's CPU train step on a bounded sample,
rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(REPO, 'uncertainty-model_amd'), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import yaml  # noqa: E402

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_PEAK_TFLOPS = 2500.0   # dense bf16 MFMA
F32_PEAK_TFLOPS = 157.3     # f32 MFMA


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=8, help='pairs per GPU')
    ap.add_argument('--height', type=int, default=256)
    ap.add_argument('--width', type=int, default=512)
    ap.add_argument('--dtype', default='bf16', choices=['bf16', 'fp32'])
    ap.add_argument('--loss-type', default='bayesian', choices=['l1', 'bayesian', 'log_bayesian'])
    ap.add_argument('--config', default='config.yml')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-roofline', action='store_true')
    ap.add_argument('--loader-steps', type=int, default=20,
                    help='N=1: also time this many steps fed by the PNG/DataLoader/GPU-augment '
                         'input pipeline (loader_line; 0 = off)')
    ap.add_argument('--no-loss-delta', action='store_true',
                    help='skip the loss-delta-vs-reference leg (fp32 + bf16 10-step trajectories)')
    ap.add_argument('--no-graph', action='store_true',
                    help='eager launches instead of the captured HIP graph')
    ap.add_argument('--eager-steps', type=int, default=3,
                    help='N=1: also time this many eagerly launched steps (reported beside)')
    ap.add_argument('--cpu-steps', type=int, default=5,
                    help='CPU baseline: best of this many timed steps at C2 (BASELINE.md: 5)')
    ap.add_argument('--fp32-steps', type=int, default=5,
                    help='N=1: also time the fp32 (parity-mode) captured step, reported beside')
    return ap.parse_args()


def spawn_ranks(n: int, cmd=None) -> int:
    """``--gpus N`` without a launcher: start N copies of this script as
    rank processes (one GPU each, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in
    their environment; reference parallel_main.py:265-279 does the same with
    mp.spawn) before this process touches the GPU, wait for all of them and
    return the worst exit status.  Rank 0 prints the JSON line."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        argv = cmd or [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
        procs.append(subprocess.Popen(argv, env=env, start_new_session=True))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0:
                    rc = rc or code
                    for q in procs:  # one rank failed: the others would hang
                        os.killpg(q.pid, signal.SIGTERM)
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
    return rc if rc >= 0 else 128 - rc


def load_cfg(path, loss_type):
    with open(os.path.join(REPO, path)) as f:
        cfg = yaml.safe_load(f)
    lg = cfg['model']['encoder'].get('load_graph')
    if lg and not os.path.isabs(lg):
        cfg['model']['encoder']['load_graph'] = os.path.join(REPO, lg)
    cfg['loss']['error_loss_config']['loss_type'] = loss_type
    return cfg


def build(cfg, dtype, device, world, dp=None, stream=None):
    import model as M
    from train.loss import TukraUncertaintyLoss
    from umamd.optim import Adam
    torch.manual_seed(0)
    m = M.RandomlyConnectedModel(**cfg['model'], dtype=dtype).to(device).train()
    if dp is None:
        dp = world > 1
    if dp:
        from train.parallel import data_parallel
        m = data_parallel(m, device.index, stream=stream)
    lf = TukraUncertaintyLoss(**cfg['loss'])
    opt = Adam(m.parameters(), 1e-4)
    return m, lf, opt


def step(m, lf, opt, left, right, scale):
    import train.utils as u
    images = torch.cat([left, right], 1)
    pyr = u.scale_pyramid(images, 4)
    opt.zero_grad(set_to_none=True)
    d = m(left, scale)
    from umamd import lossfn as LF
    with LF.deferred_recon():  # as train.train.train_step: the loss forward writes the recon
        recon = u.reconstruct_pyramid(d, pyr)
    dl, el = lf(pyr, d, recon, 0, None)
    (dl + el).backward()
    opt.step()
    return dl, el


def baseline_config(a, world, cfg):
    """which BASELINE.json config the run's shape is"""
    nodes = cfg['model']['encoder'].get('nodes')
    if nodes == 10 and (a.height, a.width) == (512, 1024):
        return '5'
    if (a.height, a.width) == (128, 256):
        return '1'
    if world == 1:
        return '2'
    # C4: 8 GPUs x B=8 (global 64); N=2/4 run C4's per-GPU shape
    return '4' if world == 8 else f'4 per-GPU shape, {world} GPUs'


def time_eager(m, lf, opt, left, right, scale, batch, steps):
    """The same step launched eagerly from Python, for comparison with the
    captured graph (after the timed region; the graphs are not replayed
    again)."""
    step(m, lf, opt, left, right, scale)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(steps):
        step(m, lf, opt, left, right, scale)
    torch.cuda.synchronize()
    te = (time.perf_counter() - t1) / steps
    return {'value': round(batch / te, 2), 'ms_per_step': round(te * 1e3, 3), 'steps': steps}


# ------------------------------------------------------------- roofline ----
def loss_pixels(n, N, H, W):
    """pixels summed over the n pyramid levels of one fused-loss launch"""
    return sum(N * (H >> i) * (W >> i) for i in range(n))


# Algorithmic HBM bytes per pixel of the fused all-scale loss launches (f32):
# forward reads the 6 image channels + the 4 prediction channels; backward
# also writes the 4 gradient channels.  SURVEY 8d prices the whole fused
# stack (fwd + bwd as one pass) at 56 B/px all-f32.
LOSS_BYTES_PER_PX = {'um_loss_fwd': 4 * (6 + 4), 'um_loss_bwd': 4 * (6 + 4 + 4)}
# (a differentiated step: the forward launch computes the loss terms and the
# gradient partials, the backward is the scatter that completes them)
LOSS_KERNELS = {'um_loss_fwd': 'loss_grad_kernel<true> + loss_reduce_kernel',
                'um_loss_bwd': 'loss_scatter_kernel<true>'}


CONV_ENTRIES = {
    # C-ABI entry -> the kernel templates it launches (rocprof names)
    'um_conv2d_fwd': 'igemm_kernel<T,...,CLS=0> / halo_conv_kernel<R,BN,0,REFLECT>',
    'um_conv2d_dgrad': 'igemm_kernel<T,...,CLS> (parity classes) / halo_conv_kernel<R,BN,1,...>',
    'um_conv2d_wgrad': 'hwgrad (wgrad_halo) / wgrad_tr_kernel + wgrad_reduce',
}


def conv_min_bytes(name, a):
    """Compulsory HBM bytes of one conv-entry launch (each operand touched
    once): fwd reads x and the packed weights, writes y (f32 pre-BN or T);
    dgrad reads dy and wT, writes dx (read-modify-write when accumulating).
    None for the weight gradient (its f32 slabs are an implementation choice)."""
    if name == 'um_conv2d_dgrad':
        dt, N, H, W, C, _, _, acc, _, K, R, _, _, _, P, Q = a[:16]
        es = 4 if dt == 0 else 2
        return es * (N * P * Q * K + K * R * R * C + N * H * W * C * (2 if acc else 1))
    if name == 'um_conv2d_fwd':
        dt, N, H, W, C, _, _, _, _, K, R, _, _, _, P, Q, ydt = a[:17]
        es = 4 if dt == 0 else 2
        return es * (N * H * W * C + K * R * R * C) + (4 if ydt == 0 else 2) * N * P * Q * K
    return None


# the one-pass disparity heads (csrc/disphead.hip), HBM-bound
# (their weight gradients stay in um_conv2d_wgrad, the MFMA paths)
HEAD_ENTRIES = {'um_disp_head_fwd': 'dhead_fwd_dpp_kernel / dhead_fwd_kernel',
                'um_disp_head_dgrad': 'dhead_dgrad_col_kernel / dhead_dgrad_kernel'}


def head_min_bytes(name, a):
    """compulsory HBM bytes of one head launch: fwd reads x (bf16, C) and
    writes d (4 f32); dgrad reads dlogit (8 bf16) and writes dx (read too
    when accumulating)"""
    N, H, W, C = a[0], a[1], a[2], a[3]
    M = N * H * W
    if name == 'um_disp_head_fwd':
        return M * (2 * C + 16)
    return M * (16 + 2 * C * (2 if a[9] else 1))


def heads_report(groups):
    rows, tot = [], 0.0
    for name in HEAD_ENTRIES:
        for a, ms, _ in groups.get(name, []):
            b = head_min_bytes(name, a)
            gbs = b / (ms * 1e-3) / 1e9
            rows.append({'entry': name, 'N': a[0], 'H': a[1], 'W': a[2], 'C': a[3],
                         'ms': round(ms, 4), 'min_hbm_bytes': b, 'achieved_gbs': round(gbs, 1),
                         'frac': round(gbs / HBM_PEAK_GBS, 4)})
            tot += ms
    if not rows:
        return None
    return {'bound': 'hbm', 'launches_per_step': len(rows), 'total_ms_per_step': round(tot, 4),
            'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'launches': rows,
            'note': 'HIP events around each entry on the launch stream (one eager step)'}


def conv1x1_report(groups, peak):
    """Every 1x1 conv launch (forward and data gradient) against its own
    attainable rate min(P, AI * BW), AI = algorithmic FLOPs / compulsory
    HBM bytes (the 1x1 convs are HBM-bound at these shapes)."""
    rows = []
    for name in ('um_conv2d_fwd', 'um_conv2d_dgrad'):
        for a, ms, work in groups.get(name, []):
            if a[10] != 1:
                continue
            b = conv_min_bytes(name, a)
            ai = work / b
            att = min(peak, ai * HBM_PEAK_GBS / 1e3)  # TFLOP/s
            ach = work / (ms * 1e-3) / 1e12
            rows.append({'entry': name, 'N': a[1], 'H': a[2], 'W': a[3], 'C': a[4], 'K': a[9],
                         'ms': round(ms, 4), 'tflops': round(ach, 2), 'ai_flop_per_byte': round(ai, 1),
                         'attainable_tflops': round(att, 1), 'frac': round(ach / att, 4)})
    if not rows:
        return None
    tot_ms = sum(r['ms'] for r in rows)
    # time-weighted fraction of attainable = sum(work / attainable) / sum(time)
    ideal_ms = sum(r['ms'] * r['frac'] for r in rows)
    rows.sort(key=lambda r: -r['ms'])
    return {'launches_per_step': len(rows), 'total_ms_per_step': round(tot_ms, 4),
            'frac_of_attainable': round(ideal_ms / tot_ms, 4), 'peak_tflops': peak,
            'hbm_gbs': HBM_PEAK_GBS, 'layers': rows}


def measure_roofline(m, lf, opt, left, right, scale, dtype):
    """Time every launch of the candidate kernels with HIP events on the
    launch stream (one eager step); the entry with the largest total time is
    the dominant kernel.  Conv work = algorithmic FLOPs with the real channel
    counts (2*N*P*Q*K*R*R*C per pass, attached at each call site)."""
    from umamd import _lib
    rec = _lib.Recorder(set(CONV_ENTRIES) | set(LOSS_KERNELS) | set(HEAD_ENTRIES))
    with rec:
        step(m, lf, opt, left, right, scale)
    torch.cuda.synchronize()
    groups = {}
    for name, args, ms, work in rec.results():
        groups.setdefault(name, []).append((args, ms, work))
    peak = BF16_PEAK_TFLOPS if dtype == 'bf16' else F32_PEAK_TFLOPS
    table = {}
    for name, items in groups.items():
        if name in HEAD_ENTRIES:
            continue
        tot_ms = sum(ms for _, ms, _ in items)
        if name in LOSS_KERNELS:
            # args: nscales, N, H, W, ...
            work = sum(LOSS_BYTES_PER_PX[name] * loss_pixels(a[0], a[1], a[2], a[3])
                       for a, _, _ in items)
            ach = work / (tot_ms * 1e-3) / 1e9
            table[name] = {'kernel': LOSS_KERNELS[name], 'bound': 'hbm',
                           'achieved': round(ach, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                           'frac': round(ach / HBM_PEAK_GBS, 4)}
        else:
            work = sum(w for _, _, w in items)
            ach = work / (tot_ms * 1e-3) / 1e12
            table[name] = {'kernel': CONV_ENTRIES[name], 'bound': 'mfma',
                           'achieved': round(ach, 2), 'peak': peak, 'unit': 'TFLOP/s',
                           'frac': round(ach / peak, 4)}
            mb = [conv_min_bytes(name, a) for a, _, _ in items]
            if all(b is not None for b in mb):
                table[name]['min_hbm_bytes_per_launch'] = round(sum(mb) / len(mb))
        table[name].update({'launches_per_step': len(items),
                            'avg_launch_ms': round(tot_ms / len(items), 4),
                            'total_ms_per_step': round(tot_ms, 3),
                            'work_per_launch': work / len(items)})
    dom = max(table, key=lambda k: table[k]['total_ms_per_step'])
    out = dict(table[dom])
    out['entry'] = dom
    out['traffic'] = None
    # HBM bytes per launch of this entry from the committed rocprofv3 PMC
    # passes (tools/pmc_traffic.py: 2*FETCH_SIZE + WRITE_SIZE, separate passes)
    # -- only while the library loaded here is the one they were taken on
    pmc = os.path.join(REPO, 'profiles', 'pmc_traffic.json')
    if os.path.exists(pmc):
        with open(pmc) as f:
            t = json.load(f)
        lib = lib_digest()
        out['traffic_digest'] = t.get('lib_digest')
        if t.get('entry') != dom:
            out['traffic_note'] = f'PMC traffic is of {t.get("entry")}, not the dominant entry'
        elif not t.get('lib_digest') or t.get('lib_digest') != lib:
            out['traffic_note'] = ('PMC traffic was taken on another library build '
                                   f'({t.get("lib_digest")} vs loaded {lib}): not reported')
        else:
            out['traffic'] = round(t['traffic_bytes_per_launch'])
            out['traffic_unit'] = 'bytes/launch (rocprofv3 PMC, ' + t.get('source', '') + ')'
    out['candidates'] = {k: {kk: v[kk] for kk in ('achieved', 'unit', 'frac', 'avg_launch_ms',
                                                  'launches_per_step', 'total_ms_per_step')}
                         for k, v in table.items()}
    out['conv1x1'] = conv1x1_report(groups, peak)
    out['disp_heads'] = heads_report(groups)
    if all(k in groups for k in LOSS_KERNELS):
        # the fused loss stack (forward + backward launches) priced as SURVEY
        # 8d does: 56 B/px all-f32 (6 image + 4 prediction reads, 4 gradient
        # writes) over every scale
        a0 = groups['um_loss_fwd'][0][0]
        px = loss_pixels(a0[0], a0[1], a0[2], a0[3])
        t = table['um_loss_fwd']['total_ms_per_step'] + table['um_loss_bwd']['total_ms_per_step']
        ach = 56 * px / (t * 1e-3) / 1e9
        out['loss_stack'] = {'kernels': ' + '.join(LOSS_KERNELS.values()), 'bound': 'hbm',
                             'bytes_per_px': 56, 'pixels': px, 'ms_per_step': round(t, 4),
                             'achieved': round(ach, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                             'frac': round(ach / HBM_PEAK_GBS, 4)}
        out['loss_stack']['valu'] = loss_valu_report(
            {k: (table[k]['launches_per_step'], table[k]['total_ms_per_step'])
             for k in LOSS_KERNELS})
    return out


# VALU issue peak (MI355X_MICROARCH.md: a wave issues each VALU instruction
# over 2 cycles on its SIMD): CUs x 4 SIMDs x clock / 2 wave-instructions/s
CU_COUNT, SIMDS_PER_CU, VALU_CYCLES_PER_INST, CLOCK_GHZ = 256, 4, 2, 2.4


def loss_valu_report(launches):
    """The loss stack against its VALU-issue bound (the counters say it is
    VALU-bound): SQ_INSTS_VALU wave-instructions per launch from
    the committed rocprofv3 pass (tools/gpu_pmc_valu.sh, digest-checked like
    ``traffic``) over the HIP-event time of the same launches.
    ``launches``: entry -> (launches per step, ms per step)."""
    path = os.path.join(REPO, 'profiles', 'pmc_loss_valu.json')
    if not os.path.exists(path):
        return None
    with open(path) as f:
        pmc = json.load(f)
    lib = lib_digest()
    peak = CU_COUNT * SIMDS_PER_CU * CLOCK_GHZ * 1e9 / VALU_CYCLES_PER_INST  # wave-inst/s
    rows, insts, ms = {}, 0.0, 0.0
    for k, (n, t) in launches.items():
        e = pmc.get(k)
        if e is None or e.get('lib_digest') != lib:
            return {'note': f'VALU counters of {k} missing or taken on another library build '
                            f'({None if e is None else e.get("lib_digest")} vs loaded {lib})'}
        i = e['per_launch'] * n
        rows[k] = {'valu_insts_per_launch': round(e['per_launch']),
                   'frac': round(i / (peak * t * 1e-3), 4)}
        insts += i
        ms += t
    return {'bound': 'valu', 'valu_insts_per_step': round(insts), 'ms_per_step': round(ms, 4),
            'peak_insts_per_s': peak, 'frac': round(insts / (peak * ms * 1e-3), 4),
            'entries': rows,
            'peak_basis': f'{CU_COUNT} CUs x {SIMDS_PER_CU} SIMDs x {CLOCK_GHZ} GHz / '
                          f'{VALU_CYCLES_PER_INST} cycles per wave64 VALU instruction',
            'source': pmc[next(iter(launches))].get('source')}


def lib_digest():
    """content digest of the loaded libumamd.so (its build stamp)"""
    path = os.path.join(REPO, 'uncertainty-model_amd', 'umamd', 'libumamd.so.stamp')
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


# --------------------------------------------------------- CPU baseline ----
def _cpu_step_rate(cfg, H, W, batch, steps, seed=1234):
    """best-of-``steps`` oracle train steps (1 warm-up) -> (pairs/s, s/step,
    step-0 losses).  The warm-up step is step 0 from the formula weights on
    the bench's own synthetic pair (oracle.step.bench_inputs), so its losses
    are the oracle's side of the loss delta."""
    from oracle import model as OM, step as OS
    graphs = OM.load_stage_graphs(cfg['model']['encoder'])
    P = OS.formula_state_dict(OS.param_specs(cfg['model'], graphs))
    left, right = OS.bench_inputs(batch, H, W, seed)
    st = {}
    r0 = OS.train_step(P, left, right, 0.3, cfg['model'], cfg['loss'], graphs, st)
    best = float('inf')
    for _ in range(steps):
        t0 = time.perf_counter()
        OS.train_step(P, left, right, 0.3, cfg['model'], cfg['loss'], graphs, st)
        best = min(best, time.perf_counter() - t0)
    return batch / best, best, (r0['disp_loss'], r0['error_loss'])


def physical_cores():
    """(physical cores among the CPUs this process may run on, physical
    cores of the machine) from /sys topology: (package, core) pairs; (0, 0)
    when the topology is not readable."""
    def core_of(c):
        base = f'/sys/devices/system/cpu/cpu{c}/topology/'
        with open(base + 'physical_package_id') as f:
            pkg = f.read().strip()
        with open(base + 'core_id') as f:
            return pkg, f.read().strip()
    try:
        allowed = os.sched_getaffinity(0)
        online = [int(d[3:]) for d in os.listdir('/sys/devices/system/cpu')
                  if d.startswith('cpu') and d[3:].isdigit()]
        host = {core_of(c) for c in online}
        mine = {core_of(c) for c in allowed}
        return len(mine), len(host)
    except (OSError, ValueError):
        return 0, 0


def cpu_baseline(config, steps):
    """The oracle's CPU train step (plain-PyTorch restatement of the
    reference, pinned to its goldens) on the host cores, BASELINE.md
    protocol.  The thread count is swept (4..64) on C1 (B=2 128x256 l1, 1
    warm-up + best of 2) and the best one times C2 (B=8 256x512 bayesian, the
    GPU workload's shape: ``value``), 1 warm-up + best of ``steps``.  On the
    GPU box os.cpu_count() shows the whole machine while a job's share is
    smaller, so the sweep, not the core count, picks the threads.  The C1
    winner and its neighbours in the sweep (half, double) are then tried on
    C2 itself (1 warm-up + 1 step each): C2's own best count times ``value``."""
    ncpu = os.cpu_count() or 1
    counts = [t for t in (4, 8, 16, 32, 64) if t <= ncpu] or [ncpu]
    sweep = {}
    cfg1 = load_cfg(config, 'l1')
    for t in counts:
        torch.set_num_threads(t)
        r, _, _ = _cpu_step_rate(cfg1, 128, 256, 2, 2)
        sweep[t] = round(r, 3)
    best1 = max(sweep, key=sweep.get)
    i1 = counts.index(best1)
    cfg2 = load_cfg(config, 'bayesian')
    sweep2 = {}
    for t in counts[max(0, i1 - 1):i1 + 2]:
        torch.set_num_threads(t)
        r, _, _ = _cpu_step_rate(cfg2, 256, 512, 8, 1)
        sweep2[t] = round(r, 3)
    threads = max(sweep2, key=sweep2.get)
    torch.set_num_threads(threads)
    c2, t2, ref0 = _cpu_step_rate(cfg2, 256, 512, 8, steps)
    cpu = ''
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    cpu = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    # cores = physical cores the timed run used: its intra-op threads, capped
    # by the physical cores of the CPUs this process may run on (SMT
    # siblings count once); the machine's totals are reported beside it
    phys, host_phys = physical_cores()
    return {'value': round(c2, 3), 'unit': 'stereo-pairs/sec',
            'cores': min(threads, phys) if phys else threads,
            'threads': threads, 'host_cpu_count': ncpu, 'affinity_physical_cores': phys,
            'host_physical_cores': host_phys, 'kind': 'port',
            'sample': f'oracle fp32 train step, C2 B=8 256x512 bayesian, 1 warm-up + best of '
                      f'{steps} ({t2:.2f} s/step) at the best thread count of a C2 sweep '
                      f'around the C1 sweep\'s winner; {cpu}',
            'c1_thread_sweep_pairs_per_s': sweep, 'c2_thread_sweep': sweep2}, ref0


# ---------------------------------------------------------- loader line ----
class _PNGPairs:
    """The reference's DaVinciDataset.__getitem__ (loaders/davinci.py:70-90:
    PIL open + convert('RGB') of both views, then the transform) over PNG
    files written by ``loader_line``."""

    def __init__(self, files, transform):
        self.files, self.transform = files, transform

    def __len__(self):
        return len(self.files)

    def __getitem__(self, i):
        from PIL import Image
        lf, rf = self.files[i]
        return self.transform({'left': Image.open(lf).convert('RGB'),
                               'right': Image.open(rf).convert('RGB')})


def loader_line(run, batch, steps, warmup=3, pairs=64, src=(288, 384)):
    """pairs/s of the captured step fed by a real input pipeline: PNG pairs
    of the Hamlyn da Vinci frame size (288x384), decoded by DataLoader
    workers (PIL, as the reference's loaders), augmentation draws in the
    workers and resize / flip / ToTensor / augment on the GPU
    (train.transforms.DeviceAugment), pinned-memory uint8 batches."""
    import tempfile
    import numpy as np
    from PIL import Image
    from torch.utils.data import DataLoader
    import train.transforms as T
    from umamd.imageprep import to_device
    tmp = tempfile.mkdtemp(prefix='umamd_png_')
    rng = np.random.default_rng(0)
    files = []
    base = rng.integers(0, 256, (src[0] // 8, src[1] // 8, 3), dtype=np.uint8)
    for i in range(pairs):
        # smooth-ish textures (PNG of pure noise would not compress like frames)
        img = np.kron(np.roll(base, i, axis=1), np.ones((8, 8, 1), np.uint8))
        img = (img.astype(np.int16) + rng.integers(-8, 8, img.shape)).clip(0, 255)
        paths = []
        for v in ('l', 'r'):
            pth = os.path.join(tmp, f'{i:04d}_{v}.png')
            Image.fromarray(img.astype(np.uint8)).save(pth)
            paths.append(pth)
        files.append(tuple(paths))
    workers = max(1, min(8, (os.cpu_count() or 2) - 1))
    dl = DataLoader(_PNGPairs(files, T.DeviceAugment((256, 512))), batch_size=batch,
                    shuffle=True, num_workers=workers, pin_memory=True, drop_last=True,
                    persistent_workers=True, prefetch_factor=4)
    dev = torch.device('cuda', torch.cuda.current_device())

    def batches():
        while True:
            for b in dl:
                yield b
    it = batches()
    for _ in range(warmup):
        run(*to_device(next(it), dev))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run(*to_device(next(it), dev))
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / steps
    del dl
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)
    return {'value': round(batch / t, 2), 'ms_per_step': round(t * 1e3, 3), 'steps': steps,
            'workers': workers,
            'source': f'{src[0]}x{src[1]} PNG pairs, PIL decode in DataLoader workers, '
                      f'flip/augment draws in workers, resize+flip+ToTensor+augment on the GPU '
                      f'(train.transforms.DeviceAugment), hip-graph step'}


# ------------------------------------------------------------ loss delta ----
def _golden_traj():
    path = os.path.join(REPO, 'tests', 'golden', 'traj_c2.npz')
    if not os.path.exists(path):
        return None
    import numpy as np
    z = np.load(path)
    n = sum(1 for k in z.files if k.startswith('disp_loss_'))
    return [(float(z[f'disp_loss_{i}']), float(z[f'error_loss_{i}'])) for i in range(n)]


def loss_trajectory(cfg, dtype, device, steps):
    """``steps`` captured train steps of a ``dtype`` model with the formula
    weights on the bench's synthetic pair (C2: B=8 256x512 bayesian, scale
    0.3) -> [(disp_loss, error_loss)] per step."""
    from oracle import model as OM, step as OS
    from train.graph import CapturedTrainStep
    graphs = OM.load_stage_graphs(cfg['model']['encoder'])
    sd = OS.formula_state_dict(OS.param_specs(cfg['model'], graphs))
    left, right = OS.bench_inputs(8, 256, 512)
    left, right = left.to(device), right.to(device)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        m, lf, opt = build(cfg, dtype, device, 1, False)
        m.load_state_dict(sd)
    torch.cuda.current_stream().wait_stream(st)
    cap = CapturedTrainStep(m, lf, opt, left, right, 0.3, warmup=1, stream=st)
    out = []
    for _ in range(steps):
        dl, el = cap()
        out.append((float(dl), float(el)))
    del cap, m, lf, opt
    torch.cuda.synchronize()
    return out


def loss_delta(cfg, device, ref0):
    """BASELINE metric's "loss delta vs ref" (SURVEY 8d): |loss - ref| / |ref|
    of both scalars, at C2 with identical inputs and weights.  ``step0``
    against the oracle's fp32 step 0 timed in the cpu_baseline leg (None
    when that leg did not run); ``traj`` over the reference's own 10-step fp32
    trajectory (tests/golden/traj_c2.npz, made by importing the reference)."""
    gold = _golden_traj()
    nsteps = len(gold) if gold else 1
    res = {'config': 'C2 B=8 256x512 bayesian, formula weights, bench synthetic pair, scale 0.3'}
    for dt in ('fp32', 'bf16'):
        tr = loss_trajectory(cfg, dt, device, nsteps)
        r = {'step0': {'disp': tr[0][0], 'error': tr[0][1]}}
        if ref0 is not None:
            r['step0_vs_oracle'] = {'disp': abs(tr[0][0] / ref0[0] - 1),
                                    'error': abs(tr[0][1] / ref0[1] - 1)}
        if gold:
            dd = [abs(a[0] / b[0] - 1) for a, b in zip(tr, gold)]
            de = [abs(a[1] / b[1] - 1) for a, b in zip(tr, gold)]
            r['vs_reference_traj'] = {'steps': len(gold), 'step0_disp': dd[0], 'step0_error': de[0],
                                      'max_disp': max(dd), 'max_error': max(de)}
        res[dt] = r
    if gold:
        res['reference_step0'] = {'disp': gold[0][0], 'error': gold[0][1]}
    return res


def time_fp32(cfg, device, left, right, scale, batch, warmup, steps):
    """The fp32 (parity-mode, INTEGRATION.md default) captured step on the
    same inputs: reported beside the bf16 headline."""
    from train.graph import CapturedTrainStep
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        m, lf, opt = build(cfg, 'fp32', device, 1, False)
    torch.cuda.current_stream().wait_stream(st)
    cap = CapturedTrainStep(m, lf, opt, left, right, scale, warmup=max(1, warmup), stream=st)
    cap()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        cap()
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / steps
    return {'value': round(batch / t, 2), 'ms_per_step': round(t * 1e3, 3), 'steps': steps,
            'dtype': 'fp32'}


def main():
    a = parse()
    if a.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(spawn_ranks(a.gpus))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if 'WORLD_SIZE' in os.environ and a.gpus not in (1, world):
        print(f'bench: --gpus {a.gpus} but WORLD_SIZE={world}; using {world} ranks',
              file=sys.stderr)
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # UMAMD_DIST=1 (under torchrun) runs the data-parallel path even with one
    # rank: the DDP wrapper and the captured RCCL all-reduce on a 1-GPU box
    dp = world > 1 or os.environ.get('UMAMD_DIST') == '1'
    # the ONE JSON line goes to the original stdout; everything else the
    # libraries print there (RCCL's version banner at communicator init)
    # is sent to stderr
    json_out = os.fdopen(os.dup(1), 'w')
    sys.stdout.flush()
    os.dup2(2, 1)
    if dp:
        # 'nccl' is RCCL; UMAMD_DIST_BACKEND=gloo rehearses the N>1 path with
        # several ranks on one GPU (RCCL needs a GPU per rank)
        dist.init_process_group(os.environ.get('UMAMD_DIST_BACKEND', 'nccl'),
                                init_method='env://')
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device('cuda', local)
    cfg = load_cfg(a.config, a.loss_type)
    backend = dist.get_backend() if dp else None
    # a gloo collective (host-staged) cannot be captured in a HIP graph: the
    # gloo rehearsal of the N>1 path steps eagerly
    use_graph = not a.no_graph and backend in (None, 'nccl')
    # the graph is captured on this stream; DDP is constructed under it (it
    # keeps the parameters' AccumulateGrad nodes, which remember their stream)
    cap_stream = torch.cuda.Stream() if use_graph else torch.cuda.current_stream()
    with torch.cuda.stream(cap_stream):
        m, lf, opt = build(cfg, a.dtype, device, world, dp, stream=cap_stream)
    torch.cuda.current_stream().wait_stream(cap_stream)
    g = torch.Generator(device='cpu').manual_seed(1234 + rank)
    left = torch.rand(a.batch, 3, a.height, a.width, generator=g).to(device)
    right = torch.rand(a.batch, 3, a.height, a.width, generator=g).to(device)
    scale = 0.3  # adjust_disparity(0)

    launch = 'hip-graph' if use_graph else 'eager'
    run = None
    if use_graph:
        from train.graph import CapturedTrainStep
        # the capture's own eager warm-up steps count toward W; one replay warms the graph
        # (N>1: SyncBN and the gradient all-reduce are RCCL nodes inside the graph)
        err = None
        try:
            cap = CapturedTrainStep(m, lf, opt, left, right, scale, warmup=max(1, a.warmup - 1),
                                    stream=cap_stream)
            run = cap
        except Exception as e:  # noqa: BLE001 -- reported in the JSON line
            err = f'{type(e).__name__}: {e}'[:300]
            print(f'bench rank {rank}: capture failed: {err}', file=sys.stderr)
        if world > 1:  # every rank takes the same path, or the collectives hang
            ok = torch.tensor([0 if run is None else 1], dtype=torch.int32, device=device)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok) == 0:
                run = None
                err = err or 'capture failed on another rank'
        if run is None:
            launch = f'eager (capture failed: {err})'
            use_graph = False
        else:
            run()
    if run is None:
        with torch.cuda.stream(cap_stream):
            opt.zero_grad(set_to_none=True)

        def run():
            with torch.cuda.stream(cap_stream):
                return step(m, lf, opt, left, right, scale)
        for _ in range(a.warmup):
            run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        dl, el = run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    losses = (float(dl.detach()), float(el.detach()))
    total = a.batch * world * a.steps
    out = {
        'metric': 'stereo-pairs/sec (train step) at 256x512, 1/2/4/8 MI355X; loss delta vs ref',
        'value': round(total / elapsed, 2),
        'unit': 'stereo-pairs/sec',
        'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
        'ms_per_step': round(elapsed / a.steps * 1e3, 3),
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': a.dtype, 'data': 'synthetic U[0,1) stereo pairs (device-resident), '
                                  'formula-free random init (torch.manual_seed(0))',
        'config': {'workload': f'depth+uncertainty train step (BASELINE config '
                               f'{baseline_config(a, world, cfg)}): '
                               f'fwd+4-scale loss+bwd+Adam',
                   'global_batch': a.batch * world, 'per_gpu_batch': a.batch,
                   'height': a.height, 'width': a.width, 'loss': a.loss_type,
                   'parallelism': f'dp{world}' + ('+syncbn' if dp else ''),
                   'process_group': ({'backend': backend, 'world_size': dist.get_world_size()}
                                     if dp else None),
                   'launch': launch,
                   'graph': f'{a.config} (nodes={cfg["model"]["encoder"].get("nodes")} '
                            f'stage graphs)'},
        'final_losses': {'disp': round(losses[0], 5), 'error': round(losses[1], 5)},
    }
    if world > 1:
        # N>1: the line goes out right after the timed loop; the reported
        # legs beside it (eager, roofline, CPU, loss delta) are N=1 legs
        if rank == 0:
            out['legs'] = 'N>1: measured value only (the roofline / CPU / loss-delta legs run at N=1)'
            print(json.dumps(out), file=json_out, flush=True)
        dist.destroy_process_group()
        return
    errors = {}
    legs = post_timing_legs(a, run, use_graph, m, lf, opt, left, right, scale, cfg, device,
                            cap_stream, errors)
    out.update(legs)
    if errors:
        out['leg_errors'] = errors
    print(json.dumps(out), file=json_out, flush=True)
    if dp:
        dist.destroy_process_group()


def run_leg(name, fn, errors):
    """One reported leg after the timed region: a failure is recorded in the
    line (``leg_errors``) instead of losing the measured value."""
    try:
        return fn()
    except Exception as e:  # noqa: BLE001
        errors[name] = f'{type(e).__name__}: {e}'[:300]
        print(f'bench: {name} leg failed: {errors[name]}', file=sys.stderr, flush=True)
        return None


def post_timing_legs(a, run, use_graph, m, lf, opt, left, right, scale, cfg, device, cap_stream,
                     errors):
    """The N=1 legs reported beside the measured value (each one guarded)."""
    res = {}
    if use_graph and a.loader_steps > 0 and (a.height, a.width) == (256, 512):
        res['loader_line'] = run_leg('loader_line',
                                     lambda: loader_line(run, a.batch, a.loader_steps), errors)
    # the eager comparison and the roofline pass run on the stream the model
    # was built on (DDP keeps AccumulateGrad nodes bound to it)

    def on_stream(fn):
        def g():
            with torch.cuda.stream(cap_stream):
                r = fn()
                torch.cuda.synchronize()
                return r
        return g
    if use_graph and a.eager_steps > 0:
        res['eager_launch'] = run_leg('eager_launch', on_stream(
            lambda: time_eager(m, lf, opt, left, right, scale, a.batch, a.eager_steps)), errors)
    if not a.no_roofline:
        res['roofline'] = run_leg('roofline', on_stream(
            lambda: measure_roofline(m, lf, opt, left, right, scale, a.dtype)), errors)
    if a.dtype == 'bf16' and a.fp32_steps > 0:
        res['fp32_line'] = run_leg('fp32_line', lambda: time_fp32(
            cfg, device, left, right, scale, a.batch, 2, a.fp32_steps), errors)
    ref0 = None
    if not a.no_cpu_baseline:
        r = run_leg('cpu_baseline', lambda: cpu_baseline(a.config, a.cpu_steps), errors)
        if r is not None:
            res['cpu_baseline'], ref0 = r
        else:
            res['cpu_baseline'] = None
    if not a.no_loss_delta and (a.height, a.width, a.batch, a.loss_type) == \
            (256, 512, 8, 'bayesian'):
        res['loss_delta'] = run_leg('loss_delta', lambda: loss_delta(
            load_cfg(a.config, 'bayesian'), device, ref0), errors)
    return res


if __name__ == '__main__':
    main()
