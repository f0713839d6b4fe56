"""ctypes binding of libsa_hip.so (the C ABI declared in include/stereoanywhere_hip.h).

The library is built in-tree (``make`` or ``stereoanywhere_amd._native.build()``) so the
.so travels with the repo snapshot to the GPU box.  There is no fallback: if the
library is missing every op raises, loudly.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("SA_HIP_LIB") or os.path.join(_HERE, "lib", "libsa_hip.so")  # override: A/B runs
HEADER = os.path.join(ROOT, "include", "stereoanywhere_hip.h")

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
F = ctypes.c_float

# name -> (restype, argtypes); must match include/stereoanywhere_hip.h exactly
class SaWinoProblem(ctypes.Structure):
    """include/stereoanywhere_hip.h: one convolution of sa_conv2d_k3_wino_multi."""
    _fields_ = [("in_", P), ("in_bs", L), ("N", I), ("Cin", I), ("H", I), ("W", I), ("U", P), ("Cout", I),
                ("bias", P), ("relu", I), ("in_m", P), ("in_s", P), ("in_t", P), ("in_pstride", I),
                ("in_act", I), ("out", P), ("out_bs", L), ("stats_partial", P), ("pitch", I),
                ("skip", P), ("skip_bs", L), ("skip_s", P), ("skip_t", P), ("skip_act", I), ("out_act", I)]


class SaGateEpilogue(ctypes.Structure):
    """include/stereoanywhere_hip.h: ConvGRU gate epilogue of sa_conv2d_k3_wino4_multi_gate."""
    _fields_ = [("mode", I), ("ctx", P), ("ctx_bs", L), ("h", P), ("h_bs", L), ("z", P), ("z_bs", L),
                ("add", P), ("add_bs", L), ("out2", P), ("out2_bs", L), ("head_w", P), ("head_part", P),
                ("head_part_bs", L)]


class SaResampleJob(ctypes.Structure):
    """include/stereoanywhere_hip.h: one pool2x / interp job of sa_resample_multi."""
    _fields_ = [("kind", I), ("in_", P), ("in_bs", L), ("in_pitch", I), ("B", I), ("C", I), ("H", I), ("W", I),
                ("Ho", I), ("Wo", I), ("out", P), ("out_bs", L), ("out_pitch", I)]


class SaFeatureGateJob(ctypes.Structure):
    """include/stereoanywhere_hip.h: one DoubleFeatureAtt branch of sa_feature_gates."""
    _fields_ = [("in_", P), ("in_bs", L), ("B", I), ("H", I), ("W", I), ("w3", P), ("w1", P), ("b1", P),
                ("C", I), ("out", P), ("out_bs", L)]


SIGNATURES = {
    "sa_feature_gates_ws_size": (L, [I, P]),
    "sa_feature_gates": (I, [I, P, P, P]),
    "sa_abi_version": (I, []),
    "sa_conv1x1_weights_size": (L, [I, I]),
    "sa_conv1x1_weights": (I, [P, I, I, P, P]),
    "sa_conv1x1": (I, [P, L, I, I, I, I, P, I, P, F, P, L, P]),
    "sa_conv1x1_redo_blocks": (L, [I]),
    "sa_tile_gather_pad": (I, [P, I, I, I, P, I, I, I, I, I, I, I, P, P]),
    "sa_tile_stitch": (I, [P, L, I, P, I, I, I, P, I, I, I, P, P, P]),
    "sa_last_error": (ctypes.c_char_p, []),
    "sa_pyramid_level_width": (I, [I, I]),
    "sa_pyramid_level_offset": (I, [I, I]),
    "sa_pyramid_row_stride": (L, [I, I]),
    "sa_corr_volume_pyramid": (I, [P, P, I, I, I, I, I, F, P, P, F, I, P, L, P]),
    "sa_corr_pyramid_from_volume": (I, [P, L, I, L, I, P, L, P]),
    "sa_corr_pyramid_from_volume_strided": (I, [P, I, I, I, I, L, L, L, I, P, L, P]),
    "sa_corr_lookup": (I, [P, P, I, L, I, I, P, L, I, I, I, P, L, P]),
    "sa_corr_lookup_conv1x1": (I, [P, P, I, L, I, I, P, L, I, I, I, P, P, I, P, P]),
    "sa_lookup_set_mfma": (None, [I]),
    "sa_lookup_set_shear_dual": (None, [I]),
    "sa_lookup_get_shear_dual": (I, []),
    "sa_lookup_get_mfma": (I, []),
    "sa_shear_slice_size": (L, [I, I, I]),
    "sa_shear_row_pitch": (L, [I]),
    "sa_corr_shear_supported": (I, [I, I, I, I, I]),
    "sa_shear_level_offset": (L, [I, I, I, I]),
    "sa_corr_pyramid_shear": (I, [P, L, I, I, I, I, I, P, P]),
    "sa_corr_volume_pyramid_sheared": (I, [P, P, I, I, I, I, I, F, P, P, F, I, P, P]),
    "sa_corr_pyramid_from_volume_strided_sheared": (I, [P, I, I, I, I, L, L, L, I, P, P]),
    "sa_corr_lookup_conv1x1_sheared": (I, [P, P, I, I, I, P, L, I, I, I, P, P, I, P, P]),
    "sa_mono_normals": (I, [P, I, I, I, F, P, P]),
    "sa_mono_masked_volume": (I, [P, P, P, P, I, I, I, I, I, F, P, P]),
    "sa_mono_bin_records": (I, [P, P, I, I, I, I, P, P]),
    "sa_softargmin_conf": (I, [P, P, I, I, I, I, L, L, L, L, P, P, P, P, L, P]),
    "sa_softargmin_set_one_pass": (None, [I]),
    "sa_softargmin_get_one_pass": (I, []),
    "sa_split_redo_blocks": (L, [I]),
    "sa_conv2d_k3_wino4_launch": (I, [I, P, P, I, I, P]),
    "sa_flow_head_part_size": (L, [I, I, I, I]),
    "sa_clock_probe": (I, [I, I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "sa_flow_head_reduce": (I, [P, I, I, I, I, P, P, P, L, P, L, P]),
    "sa_softlrc": (I, [P, P, P, P, I, I, I, L, F, P, P, P]),
    "sa_weighted_lsq": (I, [P, P, P, I, I, F, F, P, P, P]),
    "sa_weighted_lsq_ws_size": (L, [I, I]),
    "sa_weighted_lsq_ws": (I, [P, P, P, I, I, F, F, P, P, P, P]),
    "sa_mono_scale_mirror": (I, [P, P, P, P, P, P, I, I, I, L, F, F, P, P, P, P, P]),
    "sa_gru_zr": (I, [P, L, P, P, L, P, P, L, P, L, I, I, I, P, P, P]),
    "sa_gru_out": (I, [P, L, P, P, L, P, L, P, I, I, I, P, L, P]),
    "sa_gru_out_split": (I, [P, L, P, P, P, L, P, L, P, I, I, I, P, L, P]),
    "sa_pool2x": (I, [P, L, I, I, I, I, P, L, P]),
    "sa_interp_bilinear_ac": (I, [P, L, I, I, I, I, I, I, P, L, P]),
    "sa_pool2x_p": (I, [P, L, I, I, I, I, I, P, L, I, P]),
    "sa_interp_bilinear_ac_p": (I, [P, L, I, I, I, I, I, I, I, P, L, I, P]),
    "sa_resample_multi": (I, [I, P, P]),
    "sa_relu_copy": (I, [P, L, I, I, I, P, L, P]),
    "sa_flow_update": (I, [P, P, L, I, I, I, P, L, P, L, P]),
    "sa_convex_upsample": (I, [P, P, L, I, I, I, I, P, P]),
    "sa_conv3d_stat_parts": (L, [I, I, I, I, I]),
    "sa_conv3d": (I, [P, I, I, I, I, I, I, P, I, P, P, I, F, P, P, P, P, P]),
    "sa_conv2d_k3_narrow": (I, [P, L, I, I, I, I, P, P, I, P, L, P]),
    "sa_conv2d_wino_weights": (I, [P, I, I, P, P]),
    "sa_conv2d_k3_wino": (I, [P, L, I, I, I, I, P, I, P, I, P, L, P]),
    "sa_conv2d_k3_wino_stat_parts": (L, [I, I]),
    "sa_conv2d_k3_wino_ex": (I, [P, L, I, I, I, I, P, I, P, I, P, P, P, I, I, P, L, P, P]),
    "sa_conv2d_k3_wino_multi": (I, [I, P, P]),
    "sa_conv2d_wino4_weights": (I, [P, I, I, P, P]),
    "sa_conv2d_wino4_weights_split": (I, [P, I, I, P, P]),
    "sa_conv2d_k3_wino4_stat_parts": (L, [I, I]),
    "sa_conv2d_k3_wino4_multi": (I, [I, P, P]),
    "sa_conv2d_k3_wino4_multi_gate": (I, [I, P, P, I, P]),
    "sa_conv_direct_weights": (I, [P, I, I, I, I, I, P, P]),
    "sa_conv_direct_weights_size": (L, [I, I, I, I, I]),
    "sa_conv_direct_weights_split": (I, [P, L, P, P]),
    "sa_conv_direct_stat_parts": (L, [I, I]),
    "sa_conv_direct": (I, [P, L, I, I, I, I, I, I, P, P, I, P, L, P, L, P, P, P]),
    "sa_conv_direct_split": (I, [P, L, I, I, I, I, I, I, P, P, I, P, L, P, L, P, P, P]),
    "sa_conv_direct_close_supported": (I, [I, I, I]),
    "sa_conv_direct_close": (I, [P, L, P, L, P, P, I, I, I, I, I, I, P, P, I, I, P, L, P, L, P, P, P]),
    "sa_plane_stats": (I, [P, L, I, I, L, F, P, P, P]),
    "sa_norm_act": (I, [P, L, I, I, L, P, P, P, I, I, P, L, P, P, P, I, I, I, P, L, P]),
    "sa_conv3d_upcat_stat_parts": (L, [I, I, I]),
    "sa_conv3d_wd_stat_parts": (L, [I, I, I, I]),
    "sa_conv3d_pointwise": (I, [P, I, I, I, I, I, P, P, I, F, P, P, P, I, P, P]),
    "sa_conv3d_pointwise_upcat": (I, [P, I, P, P, I, P, P, P, I, I, I, I, I, I, I, F, P, I, P, P, P]),
    "sa_instnorm_finalize": (I, [P, I, L, L, F, P, P, P]),
    "sa_conv3d_wd": (I, [P, I, I, I, I, I, P, I, P, P, I, F, P, P, P, P, P]),
    "sa_conv3d_wd_set_variant": (None, [I]),
    "sa_conv3d_wd_get_variant": (I, []),
    "sa_conv3d_mf_weights_size": (L, [I, I]),
    "sa_conv3d_mf_weights": (I, [P, I, I, P, P]),
    "sa_conv3d_mf_stat_parts": (L, [I, I, I, I, I, I]),
    "sa_conv3d_mf": (I, [P, I, I, I, I, I, P, I, P, P, F, P, P, P]),
    "sa_conv3d_mf_set_planes": (None, [I]),
    "sa_conv3d_mf_get_planes": (I, []),
    "sa_struct_size": (L, [I]),
    "sa_conv3d_s2mf_weights_size": (L, []),
    "sa_conv3d_s2mf_weights": (I, [P, P, P]),
    "sa_conv3d_s2mf_stat_parts": (L, [I, I, I]),
    "sa_conv3d_s2mf": (I, [P, I, I, I, I, P, P, P, F, P, P, P, P, P]),
    "sa_conv3d_onehot_stat_parts": (L, [I, I, I]),
    "sa_conv3d_onehot": (I, [P, P, I, I, I, I, I, I, F, P, I, P, P, P]),
    "sa_conv3d_pointwise_upcat_onehot": (I, [P, P, I, F, P, I, I, I, I, I, I, I, P, I, P, P, P]),
    "sa_vol_apply": (I, [P, I, I, I, I, I, P, P, I, F, P, P, P, P]),
    "sa_conv2d_small": (I, [P, L, I, I, I, I, P, P, I, I, I, P, L, P]),
    "sa_timing_enable": (I, [I]),
    "sa_timing_read": (I, [I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_long)]),
    "sa_kernel_name": (ctypes.c_char_p, [I]),
}

KERNEL_IDS = {
    "corr_volume_pyramid": 0, "corr_lookup": 1, "mono_masked_volume": 2, "softargmin_conf": 3,
    "weighted_lsq": 4, "gru_zr": 5, "gru_out": 6, "convex_upsample": 7, "misc": 8, "conv3d_fused": 9,
    "norm_act": 10, "conv2d_wino": 11, "conv2d_direct": 12, "conv2d_wino4": 13, "corr_shear": 14,
    "mono_pyramid": 15, "gru_plumbing": 16, "conv2d_small": 17, "conv2d_narrow": 18, "conv1x1": 19,
}

_lib: Optional[ctypes.CDLL] = None


class NativeError(RuntimeError):
    pass


def build(verbose: bool = False) -> str:
    """Compile libsa_hip.so for gfx950 with hipcc (via the repo Makefile)."""
    cmd = ["make", "-C", ROOT, "-j8"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise NativeError(f"building libsa_hip.so failed:\n{res.stdout}\n{res.stderr}")
    if verbose:
        print(res.stdout)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"{LIB_PATH} is missing: the HIP hot path has no fallback. Build it with `make` "
                "or stereoanywhere_amd._native.build().")
        h = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name, None)
            if fn is None:
                if os.environ.get("SA_HIP_LIB"):   # an older library of an A/B run: bind what it has
                    continue
                raise NativeError(f"{LIB_PATH} does not export {name}")
            fn.restype = res
            fn.argtypes = args
        _check_abi(h)
        _lib = h
    return _lib


# include/stereoanywhere_hip.h SA_ABI_VERSION: the library must be built from the same header as
# these bindings (the struct arrays are read at the library's stride)
ABI_VERSION = 7


def _check_abi(h) -> None:
    if not hasattr(h, "sa_abi_version"):
        if os.environ.get("SA_HIP_LIB"):   # an older library of an A/B run
            return
        raise NativeError(f"{LIB_PATH} has no sa_abi_version: rebuild it (`make`)")
    v = int(h.sa_abi_version())
    if v != ABI_VERSION:
        raise NativeError(f"{LIB_PATH} implements ABI version {v}, these bindings {ABI_VERSION}: rebuild it")
    for which, st in ((0, SaWinoProblem), (1, SaGateEpilogue), (2, SaResampleJob), (3, SaFeatureGateJob)):
        got = int(h.sa_struct_size(which))
        if got != ctypes.sizeof(st):
            raise NativeError(f"{LIB_PATH}: {st.__name__} is {got} bytes in the library, "
                              f"{ctypes.sizeof(st)} in the bindings")


def call(name: str, *args) -> None:
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().sa_last_error().decode(errors="replace")
        raise NativeError(f"{name} failed ({rc}): {msg}")


def timing_enable(on: bool) -> None:
    call("sa_timing_enable", 1 if on else 0)


def timing_read(kernel: str):
    """(total_ms, launches) of one kernel since timing_enable / the last read."""
    ms = ctypes.c_double()
    n = ctypes.c_long()
    call("sa_timing_read", KERNEL_IDS[kernel], ctypes.byref(ms), ctypes.byref(n))
    return ms.value, n.value
