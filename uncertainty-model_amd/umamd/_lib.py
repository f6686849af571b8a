"""ctypes binding of libumamd.so (the C ABI declared in include/umamd.h).

The product path has no fallback: if the library is missing or no HIP device
is present, ``lib()`` raises.  Every wrapper passes torch's *current* stream.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libumamd.so')

UM_F32, UM_BF16 = 0, 1
# OR'ed into the dtype of the um_bn_elu_* entries / um_conv2d_fwd_up2: the
# pre-BN y is stored in the activation dtype (include/umamd.h)
Y_ACT = 0x100
PAD_ZERO, PAD_REFLECT = 0, 1
EPI_NONE, EPI_STATS, EPI_SIGMOID_SCALE, EPI_RESIDUAL, EPI_STAT_SLOTS = 0, 1, 2, 3, 4
STAT_SLOTS = 16  # UM_STAT_SLOTS (include/umamd.h)
CAT_COPY, CAT_UP2, CAT_PSHUF = 0, 1, 2

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float
_D = ctypes.c_double


class CatSrc(ctypes.Structure):
    _fields_ = [('ptr', _P), ('scale', _P), ('C', _I), ('ld', _I), ('op', _I),
                ('coff', _I), ('dtype', _I), ('h', _I), ('w', _I)]


MWG_MAX, MWG_SRC = 24, 8  # UM_MWG_MAX, UM_MWG_SRC
CSUM_MAX = 24  # UM_CSUM_MAX


class CsumDesc(ctypes.Structure):
    """um_csum_desc: one bias gradient (column sum) of um_colsum_batch"""
    _fields_ = [('y', _P), ('parts', _P), ('out', _P), ('M', _I), ('C', _I), ('ld', _I),
                ('nparts', _I), ('creal', _I)]


class MwgDesc(ctypes.Structure):
    """um_mwg_desc: one merge-weight gradient of um_merge_wgrad_batch"""
    _fields_ = [('parts', _P), ('w', _P), ('dw', _P), ('nparts', _I), ('nsrc', _I), ('nw', _I),
                ('accumulate', _I), ('widx', _I * 8)]


# name -> (restype, argtypes); 's' = stream
_SIG = {
    'um_last_error': (ctypes.c_char_p, []),
    'um_version': (_I, []),
    'um_set_tuning': (_I, [ctypes.c_char_p, _I]),
    'um_conv_stats_parts': (_I, [_I, _I]),
    'um_conv2d_fwd': (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I,
                           _I, _P, _I, _I, _F, _P, _I, _P, _P, _L, 's']),
    'um_conv2d_dgrad': (_I, [_I, _I, _I, _I, _I, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I,
                             _P, _I, _P, _L, 's']),
    'um_conv2d_fwd_up2': (_I, [_I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _I, _I, _P, _I, _I, _P,
                               _P, _I, _I, _I, 's']),
    'um_conv_fwd_ws': (_L, [_I, _I, _I, _I, _I, _I, _I]),
    'um_conv_dgrad_ws': (_L, [_I, _I, _I, _I, _I, _I, _I, _I]),
    'um_conv_dgrad_ws_pad': (_L, [_I, _I, _I, _I, _I, _I, _I, _I, _I, _I]),
    'um_conv_wgrad_splits': (_I, [_I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I]),
    'um_conv2d_wgrad': (_I, [_I, _I, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _P, _I,
                             _P, _I, 's']),
    'um_conv_wgrad_reduce': (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _I, 's']),
    'um_pack_weight': (_I, [_I, _P, _I, _I, _I, _I, _P, _P, _I, 's']),
    'um_pack_batch': (_I, [_I, _P, _I, _P, _I, 's']),
    'um_pack_desc_size': (_I, []),
    'um_pack_tiles': (_I, [_I, _I, _I]),
    'um_pack_weight_seg': (_I, [_I, _P, _I, _I, _I, _I, _P, _P, _I, _I, _P, _P, _P, 's']),
    'um_conv_wgrad_reduce_seg': (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _I, _I, _P, _P, _P, 's']),
    'um_colsum_parts': (_I, [_I]),
    'um_colsum_batch': (_I, [_I, _P, _I, 's']),
    'um_colsum': (_I, [_I, _I, _I, _I, _P, _P, 's']),
    'um_reduce_rows': (_I, [_P, _I, _I, _I, _P, _I, _P, 's']),
    'um_colred_ws': (_L, [_I, _I, _I]),
    'um_bn_stats_reduce': (_I, [_P, _I, _I, _P, _P, 's']),
    'um_bn_stats_coeffs': (_I, [_P, _I, _I, _P, _D, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _P,
                                's']),
    'um_bn_bwd_stats_coeffs': (_I, [_P, _I, _I, _P, _D, _P, _P, _P, _P, _P, _P, _P, _P, 's']),
    'um_bn_coeffs': (_I, [_P, _D, _I, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _P, 's']),
    'um_bn_fwd_pool_parts': (_I, [_L, _L]),
    'um_bn_fwd_pool_parts_c': (_I, [_L, _L, _I]),
    'um_bn_elu_fwd': (_I, [_I, _L, _I, _P, _I, _P, _P, _P, _I, _I, _L, _P, 's']),
    'um_bn_elu_fwd_slots': (_I, [_I, _L, _I, _P, _I, _P, _D, _P, _P, _F, _F, _P, _P, _P, _P, _P,
                                 _P, _P, _P, _I, _I, _L, _P, 's']),
    'um_bn_elu_fwd_slots_merge': (_I, [_I, _L, _I, _P, _I, _P, _D, _P, _P, _F, _F, _P, _P, _P,
                                       _P, _P, _P, _P, _P, _I, _I, _I, _P, _P, _P, _I, _P,
                                       's']),
    'um_bn_elu_bwd_reduce_slots': (_I, [_I, _L, _I, _L, _P, _I, _P, _I, _P, _P, _P, _P, _P, _I,
                                        _P, 's']),
    'um_bn_elu_bwd_apply_slots': (_I, [_I, _L, _I, _L, _P, _I, _P, _I, _P, _P, _P, _P, _P, _I,
                                       _P, _D, _P, _P, _P, _P, _P, _F, _P, _I, 's']),
    'um_bn_bwd_parts': (_I, [_L]),
    'um_bn_elu_bwd_reduce': (_I, [_I, _L, _I, _L, _P, _I, _P, _I, _P, _P, _P, _P, _P, _I, _P,
                                  's']),
    'um_bn_bwd_coeffs': (_I, [_P, _D, _I, _P, _P, _P, _P, _P, _P, _F, _I, _P, _P, _P, 's']),
    'um_bn_elu_bwd_apply': (_I, [_I, _L, _I, _L, _P, _I, _P, _I, _P, _P, _P, _P, _P, _I, _P,
                                 _P, _P, _P, _I, _P, 's']),
    'um_merge_fwd': (_I, [_I, _I, _P, _P, _P, _P, _L, _P, 's']),
    'um_merge_parts': (_I, [_L]),
    'um_merge_bwd': (_I, [_I, _I, _P, _P, _P, _P, _P, _P, _L, _P, _P, 's']),
    'um_merge_bn_parts': (_I, [_L]),
    'um_merge_bwd_bn': (_I, [_I, _I, _P, _P, _P, _P, _P, _P, _L, _P, _P, _I, _P, _I, _P, _P, _P,
                             _P, _I, _P, 's']),
    'um_merge_wgrad': (_I, [_P, _I, _I, _P, _P, _P, _I, _I, 's']),
    'um_merge_wgrad_batch': (_I, [_P, _I, 's']),
    'um_image_to_nhwc': (_I, [_I, _P, _I, _I, _I, _I, _I, _P, 's']),
    'um_axpy': (_I, [_I, _L, _F, _P, _P, 's']),
    'um_sigmoid_scale_bwd': (_I, [_I, _L, _I, _P, _I, _P, _I, _F, _P, _I, 's']),
    'um_sigmoid_scale_bwd_split': (_I, [_I, _L, _I, _P, _I, _P, _I, _F, _P, _I, 's']),
    'um_head_split_fin': (_I, [_L, _I, _P, _I, _P, _F, _P, _I, 's']),
    'um_disp_head_ok': (_I, [_I, _I, _I, _I, _I]),
    'um_bnx_bytes': (_L, [_I, _I]),
    'um_bnx_alloc': (_I, [_L, _P, _P]),
    'um_bnx_open': (_I, [_P, _P]),
    'um_bnx_close': (_I, [_P]),
    'um_bnx_free': (_I, [_P]),
    'um_bnx_status': (_I, [_P]),
    'um_bnx_allreduce': (_I, [_P, _I, _P, _I, _I, _I, _I, _I, 's']),
    'um_disp_head_fwd': (_I, [_I, _I, _I, _I, _P, _I, _P, _P, _F, _P, _I, 's']),
    'um_disp_head_dgrad': (_I, [_I, _I, _I, _I, _P, _I, _P, _P, _I, _I, 's']),
    'um_pack_weight_split': (_I, [_P, _I, _I, _I, _I, _P, _P, _I, 's']),
    'um_attn_ws_kstats': (_L, [_I, _I, _I]),
    'um_attn_ws_ctx': (_L, [_I, _I, _I, _I]),
    'um_attn_ws_tiles': (_L, [_I, _I, _I, _I]),
    'um_attn_fwd': (_I, [_I, _I, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _I, 's']),
    'um_attn_bwd': (_I, [_I, _I, _I, _I, _I, _P, _I, _P, _P, _P, _P, _I, _P, _I, _P, _P, _P,
                         _P, 's']),
    'um_concat_build': (_I, [_I, _I, _I, _I, _P, _I, _I, _I, _P, 's']),
    'um_concat_bwd_ws': (_L, [_I, _I, _I, _I]),
    'um_concat_bwd_src': (_I, [_I, _I, _I, _I, _P, _I, _P, _P, _I, _I, _I, _P, _P, 's']),
    'um_channel_mean': (_I, [_I, _I, _L, _I, _P, _I, _P, 's']),
    'um_se_mlp_fwd': (_I, [_I, _I, _I, _P, _I, _F, _P, _P, _P, _P, _P, 's']),
    'um_se_mlp_bwd': (_I, [_I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F, 's']),
    'um_pyramid': (_I, [_P, _I, _I, _I, _I, _P, 's']),
    'um_warp': (_I, [_P, _I, _I, _I, _I, _P, _L, _L, _F, _P, 's']),
    'um_warp_bwd': (_I, [_P, _I, _I, _I, _I, _P, _L, _L, _F, _P, _P, _L, _L, 's']),
    'um_recon_pyramid': (_I, [_I, _I, _I, _I, _P, _P, _P, _P, 's']),
    'um_loss_ws': (_L, [_I, _I, _I, _I]),
    'um_loss_fwd': (_I, [_I, _I, _I, _I, _P, _P, _F, _I, _F, _F, _F, _F, _F, _F, _P, _P, _P,
                         _P, _P, _P, _P, 's']),
    'um_loss_bwd': (_I, [_I, _I, _I, _I, _P, _P, _F, _I, _F, _F, _F, _F, _F, _F, _P, _P, _P,
                         _P, 's']),
    'um_image_error': (_I, [_P, _P, _I, _I, _I, _F, _P, 's']),
    'um_nhwc_to_image': (_I, [_I, _P, _I, _I, _I, _I, _I, _P, 's']),
    'um_disc_head_fwd': (_I, [_I, _P, _I, _I, _I, _P, _P, _P, 's']),
    'um_disc_head_bwd': (_I, [_I, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, 's']),
    'um_l1_mean_ws': (_L, []),
    'um_l1_mean': (_I, [_I, _P, _P, _L, _P, _P, 's']),
    'um_l1_mean_bwd': (_I, [_I, _P, _P, _L, _P, _P, _P, 's']),
    'um_ssim_ws': (_L, [_I, _I, _I]),
    'um_ssim_gauss': (_I, [_P, _P, _I, _I, _I, _I, _F, _F, _P, _P, 's']),
    'um_avgpool_valid': (_I, [_P, _I, _I, _I, _I, _P, 's']),
    'um_spars_sort_ws': (_L, [_I, _I]),
    'um_spars_sort': (_I, [_P, _P, _I, _I, _P, _P, _P, _L, 's']),
    'um_spars_curve': (_I, [_P, _I, _I, _I, _P, _P, 's']),
    'um_stereo_prep_ws': (_L, [_I, _I, _I]),
    'um_stereo_prep': (_I, [_I, _I, _I, _P, _P, _I, _I, _P, _P, _I, _P, _P, _I, _P, _P, _P, _P,
                            's']),
    'um_adam_chunk': (_I, []),
    'um_adam_step': (_I, [_P, _P, _I, _F, _F, _F, _F, _F, _I, 's']),
    'um_adam_step_dev': (_I, [_P, _P, _I, _F, _P, _F, _F, _F, _F, _P, 's']),
}

_lib: Optional[ctypes.CDLL] = None


class UmamdError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load the HIP library (raises if it is missing: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    from . import _build
    if _build.needs_build():
        # missing or built from other sources: build now (under the build
        # lock, so concurrent ranks neither race nor load a half-written
        # .so) and a compile error surfaces with hipcc's own message
        if not _build.can_build():
            raise UmamdError(f'{LIB_PATH} is missing or stale and hipcc is not available to '
                             f'rebuild it (run `python uncertainty-model_amd/umamd/_build.py`)')
        try:
            _build.ensure_built()
        except RuntimeError as e:
            raise UmamdError(f'building {LIB_PATH} failed:\n{e}') from None
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIG.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = [_P if a == 's' else a for a in args]
    _lib = L
    return L


def exported_symbols():
    return sorted(_SIG)


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


class Recorder:
    """Context manager timing the launches of selected C-ABI entries with
    HIP events recorded on the launch stream (torch's current stream)."""

    _active = None

    def __init__(self, names, marker=False):
        """``marker=True`` brackets each selected launch with a one-cycle
        ``spin_kernel`` (torch.cuda._sleep) instead of timing it, so a
        rocprofv3 ``--pmc`` pass can attribute the dispatches in between to
        the entry (tools/pmc_traffic.py)."""
        self.names = set(names)
        self.marker = marker
        self.items = []

    def __enter__(self):
        Recorder._active = self
        return self

    def __exit__(self, *exc):
        Recorder._active = None

    def results(self):
        """[(name, args, ms, work)] -- synchronises on the events.  ``work``
        is the algorithmic FLOP count the caller attached (or None)."""
        out = []
        for name, args, e0, e1, work in self.items:
            e1.synchronize()
            out.append((name, args, e0.elapsed_time(e1), work))
        return out


def call(name: str, *args, work=None):
    """Call a C-ABI entry; the trailing stream argument is appended.
    ``work`` (algorithmic FLOPs of this launch) is only kept for a Recorder."""
    fn = getattr(lib(), name)
    rec = Recorder._active
    if rec is not None and name in rec.names and rec.marker:
        torch.cuda._sleep(1)
        rc = fn(*args, stream())
        torch.cuda._sleep(1)
        rec.items.append((name, args, None, None, work))
    elif rec is not None and name in rec.names:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = fn(*args, stream())
        e1.record()
        rec.items.append((name, args, e0, e1, work))
    else:
        rc = fn(*args, stream())
    if rc != 0:
        msg = lib().um_last_error().decode(errors='replace')
        raise UmamdError(f'{name} failed ({rc}): {msg}')


def query(name: str, *args):
    """Call a pure host-side query entry (no stream)."""
    return getattr(lib(), name)(*args)


def require_device(t: torch.Tensor):
    if not t.is_cuda:
        raise UmamdError('umamd kernels need tensors on a HIP device (got CPU tensor); '
                         'the HIP path has no CPU fallback')


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return UM_F32
    if dt == torch.bfloat16:
        return UM_BF16
    raise UmamdError(f'unsupported activation dtype {dt}')
