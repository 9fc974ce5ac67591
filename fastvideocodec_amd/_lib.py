"""ctypes binding of libfvc.so (the C-ABI in include/fvc.h).

The product path has exactly one compute backend: these HIP kernels. If the shared
library is missing or fails to load, every op raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FVC_LIB_PATH") or os.path.join(_HERE, "libfvc.so")  # override: experiments only

c_int = ctypes.c_int
c_float = ctypes.c_float
c_size_t = ctypes.c_size_t
vp = ctypes.c_void_p

# name -> (restype, argtypes)
_SIGS = {
    "fvc_version": (c_int, []),
    "fvc_device_arch_ok": (c_int, []),
    "fvc_conv_wpack_floats": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "fvc_conv_pack_weight": (c_int, [vp, vp, c_int, c_int, c_int, c_int, c_int]),
    "fvc_conv2d_nhwc_f32": (c_int, [vp, vp, vp, vp, vp] + [c_int] * 10 + [vp]),
    "fvc_deconv2d_nhwc_f32": (c_int, [vp, vp, vp, vp, vp] + [c_int] * 10 + [vp]),
    "fvc_conv_x3_supported": (c_int, [c_int] * 5),
    "fvc_deconv_x3_all_classes": (c_int, [c_int] * 4),
    "fvc_conv_x3_wpack_bytes": (c_size_t, [c_int] * 5),
    "fvc_conv_x3_layout_id": (ctypes.c_uint, [c_int] * 5),
    "fvc_conv_x3_pack_weight": (c_int, [vp, vp, vp] + [c_int] * 5),
    "fvc_conv2d_nhwc_x3": (c_int, [vp, vp, c_float, vp, vp, vp] + [c_int] * 11 + [vp, vp, c_int, vp]),
    "fvc_deconv2d_nhwc_x3": (c_int, [vp, vp, c_float, vp, vp, vp] + [c_int] * 11 + [vp, vp, c_int, vp]),
    "fvc_conv_x3_tap_supported": (c_int, [c_int] * 6),
    "fvc_conv_x3_pool_supported": (c_int, [c_int] * 3),
    "fvc_conv2d_nhwc_x3_pool": (c_int, [vp, vp, c_float, vp, vp, vp, vp] + [c_int] * 8 + [vp, vp, c_int, vp]),
    "fvc_x3_tap_wpack_bytes": (c_size_t, [c_int, c_int]),
    "fvc_x3_tap_pack_weight": (c_int, [vp, vp, vp, c_int, c_int]),
    "fvc_conv2d_nhwc_x3_tap": (c_int, [vp, vp, c_float, vp, vp, vp] + [c_int] * 8 + [vp, c_float]
                               + [c_int] * 2 + [vp, vp, c_int, vp]),
    "fvc_deconv2d_nhwc_x3_tap": (c_int, [vp, vp, c_float, vp, vp, vp] + [c_int] * 8 + [vp, c_float]
                                 + [c_int] * 2 + [vp, vp, c_int, vp]),
    "fvc_conv_wino_supported": (c_int, [c_int] * 5),
    "fvc_conv_wino_wpack_bytes": (c_size_t, []),
    "fvc_conv_wino_pack_weight": (c_int, [vp, vp, vp]),
    "fvc_conv2d_nhwc_wino": (c_int, [vp, vp, c_float, vp, vp, vp, vp] + [c_int] * 6 + [vp, vp, c_int, vp]),
    "fvc_conv2d_nhwc_wino_up": (c_int, [vp, vp, vp, vp, c_float, vp, vp] + [c_int] * 6 + [vp, vp, c_int, vp]),
    "fvc_conv_wino128_supported": (c_int, [c_int] * 5),
    "fvc_conv_wino128_wpack_bytes": (c_size_t, []),
    "fvc_conv_wino128_pack_weight": (c_int, [vp, vp, vp]),
    "fvc_conv2d_nhwc_wino128": (c_int, [vp, vp, vp, vp, vp] + [c_int] * 6 + [vp, vp, c_int, vp]),
    "fvc_conv_wr7_supported": (c_int, [c_int] * 5),
    "fvc_conv_wr7_wpack_bytes": (c_size_t, [c_int]),
    "fvc_conv_wr7_pack_weight": (c_int, [vp] + [c_int] * 5 + [vp, vp]),
    "fvc_conv2d_nhwc_wr7": (c_int, [vp, c_int, vp, c_int, c_float, vp, vp] + [c_int] * 7 + [vp, vp, c_int, vp]),
    "fvc_conv_stem_supported": (c_int, [c_int] * 5),
    "fvc_conv_stem_wpack_bytes": (c_size_t, [c_int] * 3),
    "fvc_conv_stem_pack_weight": (c_int, [vp] + [c_int] * 3 + [vp, vp]),
    "fvc_conv2d_nhwc_stem": (c_int, [vp, vp, c_float, vp, vp] + [c_int] * 8 + [vp, vp]),
    "fvc_wino_tap_wpack_bytes": (c_size_t, [c_int]),
    "fvc_wino_tap_pack_weight": (c_int, [vp, vp, vp, c_int]),
    "fvc_conv2d_nhwc_wino_tap": (c_int, [vp, vp, c_float, vp, vp, vp] + [c_int] * 4 + [vp, c_float, c_int, c_int, vp, vp,
                                                                                      c_int, vp]),
    "fvc_nchw_to_nhwc": (c_int, [vp, vp, c_int, c_int, c_int, c_int, c_int, vp]),
    "fvc_nhwc_to_nchw": (c_int, [vp, vp, c_int, c_int, c_int, c_int, c_int, c_int, vp]),
    "fvc_avgpool2_nhwc": (c_int, [vp, vp, c_int, c_int, c_int, c_int, vp]),
    "fvc_warp_nhwc": (c_int, [vp, vp, vp, c_int, c_int, c_int, c_int, vp]),
    "fvc_upsample2x_add_nhwc": (c_int, [vp, vp, vp, c_int, c_int, c_int, c_int, c_int, c_float, vp]),
    "fvc_spynet_assemble": (c_int, [vp, vp, vp, vp, vp, c_int, c_int, c_int, vp]),
    "fvc_mc_assemble": (c_int, [vp, vp, vp, vp, c_int, c_int, c_int, vp]),
    "fvc_sub_f32": (c_int, [vp, vp, vp, c_size_t, vp]),
    "fvc_tap_gather_nhwc": (c_int, [vp, c_int, vp, vp, vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_int, c_int, vp]),
    "fvc_gdn_nhwc": (c_int, [vp, vp, vp, vp, c_int, c_int, c_int, c_int, c_int, vp]),
    "fvc_gdn_tap_nhwc": (c_int, [vp, vp, vp, vp, vp, vp] + [c_int] * 7 + [vp, vp]),
    "fvc_reduce_ws_doubles": (c_size_t, []),
    "fvc_recon_finalize": (c_int, [vp] * 7 + [c_int, c_int, c_int, vp]),
    "fvc_bits_laplace": (c_int, [vp] * 4 + [c_int] * 5 + [vp]),
    "fvc_bits_factorized": (c_int, [vp] * 4 + [c_int] * 5 + [vp]),
    "fvc_latent_to_symbols": (c_int, [vp, vp] + [c_int] * 5 + [vp]),
    "fvc_symbols_to_latent": (c_int, [vp, vp] + [c_int] * 5 + [vp]),
    "fvc_build_indexes": (c_int, [vp, vp, c_int, vp] + [c_int] * 5 + [vp]),
    "fvc_channel_indexes": (c_int, [vp, c_int, c_int, c_int, vp]),
    "fvc_quantize_symbols": (c_int, [vp, vp, vp, c_size_t, vp]),
    "fvc_dequantize_symbols": (c_int, [vp, vp, vp, c_size_t, vp]),
    "fvc_build_indexes_flat": (c_int, [vp, vp, c_int, vp, c_size_t, vp]),
    "fvc_pmf_to_quantized_cdf": (c_int, [vp, c_int, c_int, vp]),
    "fvc_rans_encode_ws_bytes": (c_size_t, [ctypes.c_int64]),
    "fvc_rans_encode": (c_int, [vp, vp, vp, c_int, ctypes.c_int64, vp, c_int, vp, vp, vp, vp, vp, vp, vp]),
    "fvc_rans_lut_bytes": (c_size_t, [c_int, c_int]),
    "fvc_rans_build_lut": (c_int, [vp, c_int, vp, c_int, vp, vp]),
    "fvc_rans_pack": (c_int, [vp, vp, vp, c_int, vp, vp, vp, vp]),
    "fvc_rans_decode": (c_int, [vp, vp, vp, vp, c_int, c_int, c_int, vp, vp, vp, vp, vp, c_int, vp]),
    "fvc_iframe_rct_fwd": (c_int, [vp, vp, c_int, c_int, c_int, vp]),
    "fvc_iframe_rct_inv": (c_int, [vp, vp, c_int, c_int, c_int, vp]),
    "fvc_iframe_dwt53": (c_int, [vp, vp, c_int, c_int, c_int, c_int, c_int, vp]),
    "fvc_iframe_quant": (c_int, [vp, c_int, c_int, c_int, c_int, c_int, c_int, vp]),
    "fvc_iframe_block_index": (c_int, [vp, vp, c_int, vp, vp, c_int, c_int, c_int, c_int, vp]),
    "fvc_iframe_expand_index": (c_int, [vp, vp, c_int, c_int, c_int, c_int, vp]),
    "fvc_gdn_nhwc_cai": (c_int, [vp, vp, vp, vp] + [c_int] * 5 + [vp]),
    "fvc_lstm_gates": (c_int, [vp] * 7 + [c_size_t, ctypes.c_float, vp]),
    "fvc_rpm_scale": (c_int, [vp, vp, c_size_t, vp]),
    "fvc_eb_forward": (c_int, [vp] * 6 + [c_int] * 5 + [vp]),
    "fvc_gc_forward": (c_int, [vp] * 6 + [c_int] * 5 + [vp]),
    "fvc_torchac_normalize": (c_int, [vp, ctypes.c_int64, c_int, c_int, vp, vp]),
    "fvc_torchac_rows_bounds": (c_int, [vp, vp, ctypes.c_int64, c_int, vp, vp, vp, vp]),
    "fvc_torchac_laplace_rows": (c_int, [vp] + [c_int] * 6 + [vp, vp]),
    "fvc_torchac_laplace_bounds": (c_int, [vp, vp] + [c_int] * 6 + [vp, vp, vp, vp]),
    "fvc_torchac_bitest_table": (c_int, [vp, c_int, c_int, vp, vp]),
    "fvc_torchac_table_bounds": (c_int, [vp, vp] + [c_int] * 6 + [vp, vp, vp, vp]),
    "fvc_torchac_max_bytes": (c_size_t, [ctypes.c_int64]),
    "fvc_torchac_encode": (c_int, [vp, vp, ctypes.c_int64, vp, c_size_t, vp]),
    "fvc_torchac_decode": (c_int, [vp, c_int, vp, ctypes.c_int64, ctypes.c_int64, vp, c_size_t, vp]),
}

EXPORTED = tuple(_SIGS)

_lib = None
_err = None


class FvcError(RuntimeError):
    pass


def load():
    """Load libfvc.so (once). Raises FvcError if it is missing or lacks a symbol."""
    global _lib, _err
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FvcError(f"libfvc.so not built at {LIB_PATH}; run __graft_entry__.build() "
                       "(no CPU fallback exists for the codec path)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)  # AttributeError if a symbol is missing
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def call(name, *args):
    """Call a status-returning entry point; raise on a non-zero status."""
    st = getattr(load(), name)(*args)
    if st != 0:
        raise FvcError(f"{name} failed with status {st}")
    return st
