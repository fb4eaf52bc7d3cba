"""ctypes binding of libacmi.so (the C-ABI in include/acmi.h).

The library is the product path: there is no CPU or PyTorch fallback.  If the
shared object is missing or fails to load, every entry point raises.
"""

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), 'libacmi.so')
if os.environ.get('ACMI_LIB'):  # A/B timing of another build (scripts/kbench.py)
    LIB_PATH = os.environ['ACMI_LIB']

c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_u32 = ctypes.c_uint32
c_float = ctypes.c_float
c_vp = ctypes.c_void_p


class AcmiError(RuntimeError):
    """A libacmi entry point returned a non-zero status."""


class Net(ctypes.Structure):
    # mode fields: the mode + 1, 0 = the process default (acmi.h acmi_net_t)
    _fields_ = [('num_actions', c_int), ('conv3_filters', c_int), ('params', c_vp), ('conv_prep', c_vp),
                ('gemm_mode', c_int), ('forward_mode', c_int), ('conv_stats_mode', c_int)]


class Acts(ctypes.Structure):
    _fields_ = [('a1', c_vp), ('a2', c_vp), ('a3', c_vp), ('a4', c_vp),
                ('logits', c_vp), ('value', c_vp), ('ld_logits', c_int),
                ('ws', c_vp), ('ws_floats', c_i64), ('m1', c_vp), ('m2', c_vp), ('m3', c_vp)]


class Bwd(ctypes.Structure):
    _fields_ = [('d1', c_vp), ('d2', c_vp), ('d3', c_vp), ('d4', c_vp),
                ('dhead', c_vp), ('ldh', c_int)]


class EnvState(ctypes.Structure):
    _fields_ = [('episode', c_vp), ('step', c_vp), ('length', c_vp), ('total', c_vp), ('done', c_vp),
                ('game', c_vp)]


class RolloutIO(ctypes.Structure):
    _fields_ = [('seed', c_u32), ('stream_id', c_u32), ('counter', c_u32), ('counter_dev', c_vp),
                ('row_offset', c_int), ('actions', c_vp), ('bad_rows', c_vp), ('state', EnvState),
                ('env_offset', c_int), ('env_seed', c_u32), ('obs_out', c_vp), ('out_stride', c_i64),
                ('rewards', c_vp), ('terminals', c_vp), ('episode_rewards', c_vp), ('ld', c_i64),
                ('tower_done', c_int), ('next_acts', c_vp), ('next_act_stride', c_i64), ('obs_copy', c_vp)]


# name -> (restype, argtypes)
_SIGS = {
    'acmi_last_error': (ctypes.c_char_p, []),
    'acmi_abi_version': (c_int, []),
    'acmi_abi_struct_sizes': (c_int, [c_vp, c_int]),
    'acmi_set_forward_mode': (c_int, [c_int]),
    'acmi_get_forward_mode': (c_int, []),
    'acmi_set_gemm_mode': (c_int, [c_int]),
    'acmi_get_gemm_mode': (c_int, []),
    'acmi_set_conv_stats_mode': (c_int, [c_int]),
    'acmi_get_conv_stats_mode': (c_int, []),
    'acmi_band_info': (c_int, [c_int, c_int, c_i64, ctypes.POINTER(c_i64)]),
    'acmi_param_count': (c_i64, [c_int, c_int]),
    'acmi_conv_prep_bytes': (c_i64, [c_int]),
    'acmi_kfac_packed_floats': (c_i64, [c_int, c_int, c_int]),
    'acmi_kfac_pack': (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    'acmi_kfac_unpack': (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    'acmi_conv_prepare': (c_int, [ctypes.POINTER(Net), c_vp, c_vp]),
    'acmi_param_offsets': (c_int, [c_int, c_int, ctypes.POINTER(c_i64)]),
    'acmi_kfac_layout': (c_int, [c_int, c_int, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64),
                                 ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]),
    'acmi_forward': (c_int, [ctypes.POINTER(Net), c_vp, c_i64, c_int, ctypes.POINTER(Acts), c_int, c_vp]),
    'acmi_forward_ws_floats': (c_i64, [c_int]),
    'acmi_forward_strided': (c_int, [ctypes.POINTER(Net), c_vp, c_i64, c_int, ctypes.POINTER(Acts), c_int,
                                     c_i64, c_vp]),
    'acmi_sample_actions': (c_int, [c_vp, c_int, c_int, c_int, c_u32, c_u32, c_u32, c_vp, c_int, c_vp,
                                    c_vp, c_vp]),
    'acmi_sample_actions_at': (c_int, [c_vp, c_int, c_int, c_int, c_u32, c_u32, c_u32, c_int, c_vp, c_int,
                                       c_vp, c_vp, c_vp]),
    'acmi_sample_actions_dev': (c_int, [c_vp, c_int, c_int, c_int, c_u32, c_u32, c_vp, c_u32, c_int, c_vp,
                                        c_int, c_vp, c_vp, c_vp]),
    'acmi_rollout_step': (c_int, [ctypes.POINTER(Net), c_vp, c_i64, c_int, ctypes.POINTER(Acts), c_i64,
                                  ctypes.POINTER(RolloutIO), c_vp]),
    'acmi_categorical': (c_int, [c_vp, c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    'acmi_returns': (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp]),
    'acmi_gae': (c_int, [c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_float, c_float, c_vp, c_vp, c_vp]),
    'acmi_adv_moments_ws_doubles': (c_i64, [c_i64]),
    'acmi_adv_moments': (c_int, [c_vp, c_i64, c_vp, c_vp, c_vp]),
    'acmi_adv_normalize': (c_int, [c_vp, c_i64, c_vp, ctypes.c_double, ctypes.c_double, c_vp]),
    'acmi_a2c_loss_ws_floats': (c_i64, [c_int]),
    'acmi_a2c_loss': (c_int, [c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_float, c_float, c_float,
                              c_vp, c_int, c_vp, c_vp, c_vp]),
    'acmi_backward_ws_floats': (c_i64, [c_int, c_int, c_int]),
    'acmi_backward': (c_int, [ctypes.POINTER(Net), c_vp, c_i64, c_int, ctypes.POINTER(Acts),
                              ctypes.POINTER(Bwd), c_vp, c_vp, c_vp, c_i64, c_vp]),
    'acmi_kfac_output_stats': (c_int, [ctypes.POINTER(Net), c_int, ctypes.POINTER(Acts), ctypes.POINTER(Bwd),
                                       c_u32, c_u32, c_u32, c_vp, c_vp, c_i64, c_vp]),
    'acmi_backward_stacked': (c_int, [ctypes.POINTER(Net), c_vp, c_i64, c_int, ctypes.POINTER(Acts),
                                      ctypes.POINTER(Bwd), c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(Bwd), c_u32, c_u32,
                                      c_u32, c_vp, c_i64, c_vp]),
    'acmi_kfac_output_stats_finish': (c_int, [ctypes.POINTER(Net), c_int, ctypes.POINTER(Acts), ctypes.POINTER(Bwd),
                                              c_vp, c_vp, c_i64, c_vp]),
    'acmi_debug_ws_flushes': (c_int, []),
    'acmi_debug_convt2': (c_int, [ctypes.POINTER(Net), c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp, c_vp,
                                  c_vp]),
    'acmi_kfac_ema': (c_int, [c_vp, c_vp, c_vp, c_i64, c_float, c_float, c_float, c_vp]),
    'acmi_kfac_inverse_layout': (c_int, [c_int, c_int, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]),
    'acmi_kfac_inverse_floats': (c_i64, [c_int, c_int]),
    'acmi_kfac_inverse_ws_doubles': (c_i64, [c_int, c_int]),
    'acmi_kfac_inverse': (c_int, [c_int, c_int, c_vp, c_float, c_int, c_vp, c_vp, c_vp]),
    'acmi_kfac_eig_ws_doubles': (c_i64, [c_int, c_int]),
    'acmi_kfac_eigvals': (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp]),
    'acmi_kfac_step_ws_floats': (c_i64, [c_int, c_int]),
    'acmi_kfac_step': (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_float, c_float, c_float, c_vp, c_vp,
                               c_vp, c_vp]),
    'acmi_opt_ws_floats': (c_i64, [c_i64]),
    'acmi_momentum_apply': (c_int, [c_vp, c_vp, c_vp, c_i64, c_float, c_float, c_float, c_vp, c_vp, c_vp]),
    'acmi_rmsprop_apply': (c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_float, c_float, c_float, c_float, c_float,
                                   c_vp, c_vp, c_vp]),
    'acmi_env_reset': (c_int, [ctypes.POINTER(EnvState), c_int, c_int, c_u32, c_vp, c_i64, c_vp]),
    'acmi_env_step': (c_int, [ctypes.POINTER(EnvState), c_int, c_int, c_u32, c_vp, c_vp, c_i64, c_vp, c_i64,
                              c_vp, c_vp, c_vp, c_i64, c_vp]),
    'acmi_atari_preprocess': (c_int, [c_vp, c_i64, c_i64, c_vp, c_int, c_int, c_int, c_vp, c_i64, c_vp]),
    'acmi_atari_stack': (c_int, [c_vp, c_i64, c_i64, c_vp, c_int, c_int, c_int, c_vp, c_int, c_vp, c_vp,
                                 c_i64, c_vp]),
    'acmi_stream_wait_backward_dx': (c_int, [c_vp]),
    'acmi_selftest_plans': (c_int, [c_int]),
    'acmi_gemm_f32': (c_int, [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_vp]),
    'acmi_prof_enable': (c_int, [c_int, c_int]),
    'acmi_prof_collect': (c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_int)]),
}

GEMM_F32 = 0  # acmi_set_gemm_mode: v_mfma_f32_32x32x2_f32
GEMM_X3 = 1   # bf16x3 split operands on the bf16 matrix cores (default)
FWD_F32 = 0   # acmi_set_forward_mode: the conv tower f32-accurate (default)
FWD_BF16 = 1  # one bf16 MFMA per product (BASELINE configs[4] "bf16 forward")

CONV_STATS_PATCHES = 0  # acmi_set_conv_stats_mode: im2col patch rows
CONV_STATS_BAND = 1     # pixel-pair band reduction (default)

PROF_CONV1_WGRAD = 1
PROF_CONV2_WGRAD = 2
PROF_CONV1_FWD = 3
PROF_CONV1_AFACTOR = 4
PROF_CONV2_DX = 5

EXPORTED = tuple(_SIGS)

_lib = None


def load():
    """Loads libacmi.so once; raises ImportError if it is missing (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError('libacmi.so not found at {} - build it with `python __graft_entry__.py build` '
                              '(hipcc --offload-arch=gfx950); there is no CPU fallback'.format(LIB_PATH))
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if os.environ.get('ACMI_LIB') and not hasattr(lib, name):
                continue  # an older build under A/B timing: entry points added since stay unbound
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.acmi_abi_version() != 4:
            raise ImportError('libacmi ABI mismatch')
        _lib = lib
    return _lib


def check(status, what=''):
    if status != 0:
        msg = load().acmi_last_error().decode(errors='replace')
        raise AcmiError('{} failed ({}): {}'.format(what, status, msg))


def call(name, *args):
    """Calls a status-returning entry point and raises AcmiError on failure."""
    check(getattr(load(), name)(*args), name)


def ptr(t):
    """Device (or host) pointer of a contiguous tensor, or None."""
    if t is None:
        return None
    assert t.is_contiguous(), 'libacmi needs contiguous buffers'
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None):
    """hipStream_t of torch's current stream (graph-capture friendly)."""
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError('actorcritic (MI355X) needs a ROCm GPU: torch.cuda.is_available() is False; '
                           'there is no CPU fallback for the hot path')
