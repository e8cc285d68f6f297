"""ctypes binding of librpst.so (the C ABI declared in include/rpst.h).

The library is built in-tree (`make -C rp-style-transfer_amd/csrc`, or
`__graft_entry__.build()`) and loaded from there; RPST_LIB overrides the path.
There is no fallback: if the library is missing or a call fails, a RuntimeError is
raised with the library's own message (rpst_last_error()).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RPST_LIB", os.path.join(os.path.dirname(_HERE), "csrc", "librpst.so"))

_c_float_p = ctypes.c_void_p
_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_F = ctypes.c_float
_D = ctypes.c_double
_SZ = ctypes.c_size_t

# name -> (restype, argtypes); must match include/rpst.h exactly
SIGNATURES = {
    "rpst_version": (_I, []),
    "rpst_last_error": (ctypes.c_char_p, []),
    "rpst_calc_mean_std": (_I, [_P, _P, _P, _I, _I, _I64, _F, _P]),
    "rpst_adain_workspace_size": (_SZ, [_I, _I]),
    "rpst_adain": (_I, [_P, _P, _P, _I, _I, _I64, _F, _P, _SZ, _P]),
    "rpst_mean_variance_norm": (_I, [_P, _P, _I, _I, _I64, _F, _P, _SZ, _P]),
    "rpst_conv2d_packed_size": (_SZ, [_I, _I, _I]),
    "rpst_conv2d_pack": (_I, [_P, _P, _I, _I, _I, _P]),
    "rpst_conv2d_grid_threads": (_I64, [_I, _I, _I, _I, _I, _I, _I]),
    "rpst_conv2d_algorithm": (_I, [_I, _I, _I, _I, _I, _I]),
    "rpst_conv2d_set_precise": (_I, [_I]),
    "rpst_conv2d_set_quarter": (_I, [_I]),
    "rpst_conv2d_quarter": (_I, [_I, _I, _I, _I, _I, _I]),
    "rpst_conv2d_stats_workspace_size": (_SZ, [_I, _I, _I, _I, _I, _I, _I]),
    "rpst_conv2d_stats": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I,
                               _P, _P, _F, _P, _SZ, _P]),
    "rpst_conv2d_stats_store": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I,
                                     _I, _P, _P, _F, _I, _P, _SZ, _P]),
    "rpst_conv2d": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "rpst_conv2d_pool": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "rpst_conv2d_masked": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "rpst_conv2d_pair": (_I, [_P, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "rpst_conv2d_workspace_size": (_SZ, [_I, _I, _I, _I, _I, _I, _I]),
    "rpst_conv2d_ws": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I,
                            _P, _SZ, _P]),
    "rpst_conv2d_skip_adain": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "rpst_maxpool2x2_ceil": (_I, [_P, _P, _I, _I, _I, _I, _P]),
    "rpst_upsample_nearest2x": (_I, [_P, _P, _I, _I, _I, _I, _P]),
    "rpst_add_upsample_nearest2x": (_I, [_P, _P, _P, _I, _I, _I, _I, _P]),
    "rpst_sanet_attention_workspace_size": (_SZ, [_I, _I]),
    "rpst_sanet_attention_workspace_size_c": (_SZ, [_I, _I, _I]),
    "rpst_sanet_attention": (_I, [_P, _P, _P, _P, _I, _I, _I, _P, _SZ, _P]),
    "rpst_conv_weight_flip": (_I, [_P, _P, _I, _I, _I, _P]),
    "rpst_relu_backward": (_I, [_P, _P, _P, _I64, _P]),
    "rpst_leaky_relu_backward": (_I, [_P, _P, _P, _I64, _F, _P]),
    "rpst_maxpool2x2_ceil_backward": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "rpst_reflect_pad_border_grad_workspace_size": (_SZ, [_I, _I, _I, _I]),
    "rpst_reflect_pad_border_grad": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    "rpst_reflect_pad_border_grad_masked": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ,
                                                 _P]),
    "rpst_conv_wgrad_workspace_size": (_SZ, [_I, _I, _I, _I, _I]),
    "rpst_conv_wgrad": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    "rpst_conv_wgrad_pad": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    "rpst_adain_backward": (_I, [_P, _P, _P, _P, _P, _P, _I, _I64, _P, _SZ, _P]),
    "rpst_style_content_loss_grad": (_I, [_P, _P, _P, _P, _P, _I, _I64, _I, _P]),
    "rpst_sq_diff_workspace_size": (_SZ, []),
    "rpst_sq_diff_sum": (_I, [_P, _P, _I64, _D, _P, _P, _SZ, _P]),
    "rpst_pad1": (_I, [_P, _P, _I64, _I, _I, _I, _P]),
    "rpst_upsample_nearest2x_backward": (_I, [_P, _P, _I64, _I, _I, _P]),
    "rpst_mean_variance_norm_backward": (_I, [_P, _P, _P, _P, _I64, _I64, _I, _P]),
    "rpst_softmax_rows": (_I, [_P, _P, _I64, _I, _P]),
    "rpst_softmax_rows_backward": (_I, [_P, _P, _P, _I64, _I, _P]),
    "rpst_sanet_attention_backward_workspace_size": (_SZ, [_I, _I, _I]),
    "rpst_sanet_attention_backward": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _SZ,
                                           _P]),
    "rpst_sanet_attention_backward_chunked_workspace_size": (_SZ, [_I, _I, _I, _I]),
    "rpst_sanet_attention_backward_chunked": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I,
                                                   _P, _SZ, _P]),
    "rpst_adaptive_attention_backward_workspace_size": (_SZ, [_I, _I, _I, _I]),
    "rpst_adaptive_attention_backward": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _F, _F,
                                              _F, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I,
                                              _P, _SZ, _P]),
    "rpst_conv1x1_wgrad_workspace_size": (_SZ, [_I, _I, _I]),
    "rpst_conv1x1_wgrad": (_I, [_P, _P, _P, _P, _I, _I, _I64, _I, _P, _SZ, _P]),
    "rpst_u8hwc_to_f32nchw": (_I, [_P, _P, _I, _I, _I, _P]),
    "rpst_f32nchw_to_u8_tile": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "rpst_png_filter_up": (_I, [_P, _P, _I, _I, _I, _P]),
    "rpst_cosine_affinity_workspace_size": (_SZ, [_I, _I, _I]),
    "rpst_cosine_affinity": (_I, [_P, _P, _P, _I, _I, _I, _P, _SZ, _P]),
    "rpst_aea_clamp_workspace_size": (_SZ, [_I, _I, _I]),
    "rpst_aea_clamp": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _F, _F, _F, _P, _P, _I, _I, _P, _SZ,
                            _P]),
    "rpst_adaptive_attention_workspace_size": (_SZ, [_I, _I, _I, _I]),
    "rpst_adaptive_attention": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _F, _F, _F, _P,
                                     _P, _P, _P, _I, _I, _I, _P, _SZ, _P]),
    "rpst_matrix_power_workspace_size": (_SZ, [_I, _I]),
    "rpst_matrix_power_psd_f64": (_I, [_P, _P, _I, _I, _I, _P, _P, _SZ, _P]),
    "rpst_wct_workspace_size": (_SZ, [_I, _I, _I64]),
    "rpst_whiten_and_color_f64": (_I, [_P, _P, _P, _I, _I64, _P, _P, _SZ, _P]),
    "rpst_wct_fuse": (_I, [_P, _P, _P, _I, _I, _I64, _P, _P, _SZ, _P]),
    "rpst_wct_params": (_I, [_P, _P, _P, _P, _P, _I, _I, _I64, _P, _P, _SZ, _P]),
    "rpst_wct_status": (_I, [_P, _I, _I, _I64, _P, _P]),
    "rpst_wct_phase_timing": (_I, [_I]),
    "rpst_wct_phase_ms": (_I, [_P, _P]),
    "rpst_whiten_and_color_original_f64": (_I, [_P, _P, _P, _I, _I64, _P, _SZ, _P]),
    "rpst_whiten_and_color_status": (_I, [_P, _I, _I64, _P, _P]),
    "rpst_conv2d_mix_workspace_size": (_SZ, [_I, _I, _I, _I, _I, _I]),
    "rpst_conv2d_mix": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _SZ,
                             _P]),
}

_lib = None
_lock = threading.Lock()


class RpstError(RuntimeError):
    pass


def load():
    """Load librpst.so once; raise RpstError if it is absent (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RpstError(
                f"rpst: HIP library not found at {LIB_PATH}; build it with "
                "`make -C rp-style-transfer_amd/csrc` or __graft_entry__.build()")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(status: int, what: str) -> None:
    if status != 0:
        msg = load().rpst_last_error().decode(errors="replace")
        raise RpstError(f"{what} failed (status {status}): {msg}")


def call(name: str, *args):
    """Call an rpst_* entry point that returns a status code; raise on failure."""
    st = getattr(load(), name)(*args)
    check(st, name)
