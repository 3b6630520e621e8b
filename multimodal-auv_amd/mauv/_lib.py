"""ctypes binding of libmauv_hip.so — the C-ABI declared in include/mauv.h.

The library is the product: there is no fallback.  If it is missing or was built for
another architecture, importing ``mauv`` raises immediately.  torch is imported first so
that the HIP runtime the library links against (soname libamdhip64.so.7) resolves to the
one PyTorch-ROCm already loaded — stream handles are then interchangeable.
"""
import ctypes
import os

import torch  # noqa: F401  (must load libamdhip64 before the extension)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MAUV_LIB", os.path.join(_HERE, "libmauv_hip.so"))

P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
F = ctypes.c_float
U64 = ctypes.c_ulonglong
U32 = ctypes.c_uint

# name -> argtypes (restype is int unless listed in _RESTYPES)
SIGNATURES = {
    "mauv_abi_version": [],
    "mauv_last_error": [],
    "mauv_get_route": [P],
    "mauv_set_route": [P],
    # conv_gemm.hip
    "mauv_conv2d_fwd_f32": [P, P, P, P, I, P, P, P] + [I] * 10 + [P, P, P, P],
    "mauv_conv2d_fwd_stat_blocks": [I] * 10,
    "mauv_conv2d_bwd_data_f32": [P, P, P, P, P] + [I] * 11 + [P] * 7 + [I, P, P, P],
    "mauv_conv2d_bwd_data_stat_blocks": [I] * 10,
    "mauv_conv2d_wgrad_splits": [I, I, I, I, I, I, I, I, I, I],
    "mauv_conv2d_bwd_weight_f32": [P, P, P, P, I, P, P] + [I] * 11 + [P],
    # conv_gemm16.hip
    "mauv_conv2d_fwd_h16": [I, P, P, P, P, I, P, P] + [I] * 10 + [P, P, P, P, P],
    "mauv_conv2d_fwd_fold_h16": [I] + [P] * 10 + [I] * 6 + [P, P, P, P, P],
    "mauv_conv2d_bwd_data_h16": [I, P, P, P, P, I] + [I] * 10 + [P],
    "mauv_conv2d_bwd_data_bn_h16": [I, P, P, P, P, I] + [I] * 10 + [P] * 8 + [I, P, P, P],
    "mauv_reparam_sample_ex": [I, P, P, P, ctypes.c_ulonglong, ctypes.c_ulonglong, P, ctypes.c_uint,
                               I, I, I, I, I, P, LL, P],
    "mauv_conv2d_bwd_weight_h16": [I, P, P, P, P, I, P, P, I] + [I] * 10 + [P],
    # reparam.hip
    "mauv_reparam_sample": [P, P, P, U64, U64, U32, I, I, I, I, P, LL, P],
    "mauv_reparam_bwd": [P, I, LL, LL, P, P, P, U64, U64, U32, I, I, I, I, I, P, P, LL, P],
    "mauv_reparam_sample_h16": [I, P, P, P, U64, U64, U32, I, I, I, I, I, P, LL, P],
    "mauv_reparam_sample_padded": [P, P, P, U64, U64, U32, I, I, I, I, I, P, LL, P],
    "mauv_kl_workspace_bytes": [I],
    "mauv_kl_fwd": [P, I, P, F, P, P],
    "mauv_kl_bwd": [P, I, P, F, P],
    "mauv_philox_raw": [U64, U64, U32, I, P, P, P],
    # adam.hip
    "mauv_adam_step": [P, I, F, F, F, F, F, LL, P],
    "mauv_adam_step_gated": [P, I, F, F, F, F, F, P, P],
    # bn.hip
    "mauv_bn_workspace_floats": [I, LL, I],
    "mauv_bn_fwd_train": [P, I, LL, I, P, P, P, P, F, F, P, P, P, P, P, P, I, P, P],
    "mauv_bn_stats_finalize": [I, I, I, P, P, P, P, P, P, P, F, F, P, P, P, P, P, P, P],
    "mauv_bn_stats_workspace_floats": [I, I, I],
    "mauv_bn_apply": [P, P, P, P, P, P, I, P, I, LL, I, P],
    "mauv_bn_eval_params": [I, I, P, P, P, P, F, P, P, P],
    "mauv_bn_bwd": [P, P, P, I, P, P, P, P, I, LL, I, P, P, P, P, P, P, P, I, P],
    "mauv_bn_apply_h16": [I, P, P, P, P, P, P, I, P, I, LL, I, P],
    "mauv_bn_bwd_h16": [I, P, P, P, I, P, P, P, P, I, LL, I, P, P, P, P, P, P],
    # pool.hip
    "mauv_maxpool_fwd": [P, I, I, I, I, P, P, P],
    "mauv_maxpool_bwd": [P, P, I, I, I, I, P, P],
    "mauv_maxpool_bn_fwd": [P, P, P, I, I, I, I, I, P, P, P],
    "mauv_bn_apply_mask": [I, P, P, P, P, P, P, P, P, I, LL, I, P],
    "mauv_bn_bwd_mask": [I, P, P, P, P, P, P, I, LL, I, P, P, P, P, P, P],
    "mauv_bn_bwd_ex": [I, P, P, P, P, I, P, P, P, P, I, LL, I, P, P, P, P, P, P, P, I, P],
    "mauv_avgpool_fwd": [P, I, I, I, P, P],
    "mauv_avgpool_bwd": [P, I, I, I, P, P],
    "mauv_maxpool_fwd_h16": [I, P, I, I, I, I, P, P, P],
    "mauv_maxpool_bwd_h16": [I, P, P, I, I, I, I, P, P],
    "mauv_maxpool_bn_fwd_h16": [I, P, P, P, I, I, I, I, I, P, P, P],
    "mauv_avgpool_fwd_h16": [I, P, I, I, I, P, P],
    "mauv_avgpool_bwd_h16": [I, P, I, I, I, P, P],
    "mauv_pack_nchw_h16": [I, P, I, I, I, I, I, P, P],
    "mauv_pack_nchw_f32": [P, I, I, I, I, I, P, P],
    # stem.hip
    "mauv_stem_im2col": [I, P] + [I] * 9 + [P, P],
    "mauv_stem_fwd_f32": [P, P, P, I, I, I, I, P, P, P, P],
    "mauv_stem_fwd_h16": [I, P, P, P, I, I, I, I, P, P, P, P, P],
    # head.hip
    "mauv_attn_t": [P, I, I, P, P],
    "mauv_attn_t_bwd": [P, P, I, I, P, P],
    "mauv_attn_out": [P, P, I, I, P, I, I, P],
    "mauv_attn_out_bwd": [P, I, I, P, P, I, I, P, P, P],
    "mauv_colsum": [P, I, I, I, P, I, P],
    "mauv_mc_mean_ce": [P, P, I, I, I, P, P, P, P],
    "mauv_mc_mean_bwd": [P, P, P, P, I, I, I, P, P],
    "mauv_mc_stats": [P, I, I, I, F, P, I, P],
    "mauv_mc_finalize": [P, I, I, I, F, P, P, P, P, P, P],
    "mauv_nonfinite_count": [P, LL, P, P],
    # staging.hip
    "mauv_stage_u8": [P, I, I, I, I, P, P, P, P, P, F, P, P],
    "mauv_uifm": [P, I, I, I, I, P, P, P, F, P, P],
    "mauv_resize_workspace_bytes": [I, I, I, I, I, I],
    "mauv_resize_u8": [P, I, I, I, I, I, I, P, P, P, P, P, P, P, F, P, P],
    # metrics.hip
    "mauv_confusion_update": [P, P, I, I, P, P],
    "mauv_calibration_update": [P, P, I, I, I, P, P, P],
    "mauv_auroc_pairs": [P, P, I, P, P],
}
_RESTYPES = {"mauv_last_error": ctypes.c_char_p, "mauv_bn_workspace_floats": LL,
             "mauv_bn_stats_workspace_floats": LL, "mauv_resize_workspace_bytes": LL}


class MauvRoute(ctypes.Structure):
    """include/mauv.h MauvRoute: the library's process-wide kernel routing."""
    _fields_ = [("f32_math", I), ("halo3", I), ("big16", I), ("big16_min_k", I),
                ("haloc16", I), ("expand16", I), ("reparam_kernels", I),
                ("reserved", I * 9)]


class MauvError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libmauv_hip.so not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950). "
            "There is no CPU/PyTorch fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    # an explicitly chosen older library (MAUV_LIB, same-box A/B against a previous build) may
    # lack entry points added since: those raise when called, every other binding is checked
    older_ok = "MAUV_LIB" in os.environ
    for name, argt in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if not older_ok:
                raise

            def missing(*a, _n=name):
                raise MauvError(f"{_n} is not in {LIB_PATH} (an older library, MAUV_LIB)")
            setattr(lib, name, missing)
            continue
        fn.argtypes = argt
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    return lib


lib = _load()


def check(rc, what=""):
    if rc != 0:
        msg = lib.mauv_last_error().decode(errors="replace")
        raise MauvError(f"{what or 'mauv'} failed ({rc}): {msg}")
    return rc


def exported_symbols():
    return list(SIGNATURES)
