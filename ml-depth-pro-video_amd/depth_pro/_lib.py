"""ctypes binding of libdp_mi355x.so (the C ABI declared in include/dp_mi355x.h).

The library is the only compute path of this package: if it is missing or was
built for another ABI, importing the engine raises instead of falling back to
anything else.
"""

from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch  # noqa: F401  (loads the HIP runtime first; libdp links the same SONAME)

DP_BF16, DP_F16, DP_F32 = 0, 1, 2
DP_ACT_NONE, DP_ACT_RELU, DP_ACT_GELU = 0, 1, 2
DP_A_DENSE, DP_A_CONV = 0, 1
DP_STORE_ROWS, DP_STORE_DECONV2X2, DP_STORE_HEAD_PS = 0, 1, 2
DP_CV_INTER_LINEAR, DP_CV_INTER_AREA = 1, 3
DP_INTERP_BILINEAR, DP_INTERP_BICUBIC = 0, 1
DP_DEPTH_IMG_COLOR, DP_DEPTH_IMG_RAW16 = 0, 1
INTERP_MODES = {"bilinear": DP_INTERP_BILINEAR, "bicubic": DP_INTERP_BICUBIC}
(DP_TILE_AUTO, DP_TILE_128x128, DP_TILE_256x64, DP_TILE_256x32, DP_TILE_BIG_256x256, DP_TILE_BIG_256x128,
 DP_TILE_BIG_256x256_K32, DP_TILE_BIG_256x128_K32, DP_TILE_8PH_256x256, DP_TILE_DEEP4_256x256,
 DP_TILE_DEEP5_256x256, DP_TILE_DEEP_256x128, DP_TILE_STREAMK_256x256, DP_TILE_BIG_320x256,
 DP_TILE_BIG_512x128, DP_TILE_PBIG_320x256, DP_TILE_PBIG_256x256, DP_TILE_DUAL_256x128,
 DP_TILE_P8PH_256x256, DP_TILE_8PH_320x256, DP_TILE_CV3_256x256, DP_TILE_SPLITK_256x256,
 DP_TILE_CV3_192x256, DP_TILE_CV3_384x128) = range(24)
DP_ABI_VERSION = 14

_ERRORS = {1000: "DP_ERR_ARG", 1001: "DP_ERR_SHAPE", 1002: "DP_ERR_ALIGN", 1003: "DP_ERR_DTYPE"}

LIB_PATH = os.environ.get(
    "DP_MI355X_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libdp_mi355x.so")
)

# (name, ctypes type) in header order
EXPORTS = (
    "dp_abi_version", "dp_gemm", "dp_gemm_grouped", "dp_layernorm", "dp_layernorm_grouped", "dp_layernorm_stats", "dp_attention",
    "dp_attention_log2q", "dp_normalize_u8",
    "dp_resize_bilinear", "dp_resize", "dp_patchify_pyramid", "dp_vit_cls_rows", "dp_merge_windows",
    "dp_merge_windows_range", "dp_fov_tail", "dp_infer_epilogue", "dp_infer_epilogue_mode", "dp_gemm_workspace_size", "dp_gemm_plan",
    "dp_depth_to_points", "dp_gemm_workspace_check", "dp_resize_u8_cv", "dp_depth_to_image",
)


class GemmArgs(ctypes.Structure):
    """Mirror of `dp_gemm_args` (include/dp_mi355x.h)."""

    _fields_ = [
        ("M", ctypes.c_int32), ("N", ctypes.c_int32), ("K", ctypes.c_int32),
        ("dtype", ctypes.c_int32),
        ("A", ctypes.c_void_p), ("lda", ctypes.c_int64),
        ("B", ctypes.c_void_p), ("ldb", ctypes.c_int64),
        ("a_mode", ctypes.c_int32), ("relu_a", ctypes.c_int32),
        ("in_h", ctypes.c_int32), ("in_w", ctypes.c_int32), ("in_c", ctypes.c_int32),
        ("k_h", ctypes.c_int32), ("k_w", ctypes.c_int32), ("stride", ctypes.c_int32),
        ("pad", ctypes.c_int32), ("out_h", ctypes.c_int32), ("out_w", ctypes.c_int32),
        ("bias", ctypes.c_void_p), ("act", ctypes.c_int32),
        ("gamma", ctypes.c_void_p),
        ("pos", ctypes.c_void_p), ("ldpos", ctypes.c_int64),
        ("pos_group", ctypes.c_int32), ("pos_off", ctypes.c_int32),
        ("R1", ctypes.c_void_p), ("ldr1", ctypes.c_int64),
        ("R2", ctypes.c_void_p), ("ldr2", ctypes.c_int64),
        ("C", ctypes.c_void_p), ("ldc", ctypes.c_int64),
        ("c_dtype", ctypes.c_int32), ("accumulate", ctypes.c_int32),
        ("store_mode", ctypes.c_int32),
        ("dc_h", ctypes.c_int32), ("dc_w", ctypes.c_int32), ("dc_cout", ctypes.c_int32),
        ("row_group", ctypes.c_int32), ("row_group_out", ctypes.c_int32), ("row_off", ctypes.c_int32),
        ("head_w", ctypes.c_void_p), ("head_b", ctypes.c_float), ("head_corr", ctypes.c_void_p),
        ("tile", ctypes.c_int32),
        ("workspace", ctypes.c_void_p), ("workspace_bytes", ctypes.c_int64),
        ("ln_part_out", ctypes.c_void_p), ("ln_xb_out", ctypes.c_void_p), ("ln_part_in", ctypes.c_void_p),
        ("ln_colsum", ctypes.c_void_p), ("ln_eps", ctypes.c_float), ("ln_xl", ctypes.c_void_p),
        ("ln_rs_out", ctypes.c_void_p), ("ln_rs_in", ctypes.c_void_p),
    ]


class DPError(RuntimeError):
    pass


_lib: Optional[ctypes.CDLL] = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load and type the library once; raise DPError if it is absent or stale."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise DPError(
            f"libdp_mi355x.so not found at {path}: build it with "
            f"`make -C ml-depth-pro-video_amd/csrc` (or __graft_entry__.build()). "
            f"There is no fallback compute path."
        )
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name in EXPORTS:
        if not hasattr(lib, name):
            raise DPError(f"{path} does not export {name}")
    vp, i32, i64, f32, f64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_double
    sig = {
        "dp_abi_version": [],
        "dp_gemm": [ctypes.POINTER(GemmArgs), vp],
        "dp_gemm_grouped": [ctypes.POINTER(GemmArgs), i32, vp],
        "dp_layernorm_grouped": [vp, i64, vp, vp, i32, vp, i64, i32, i32, f32, i32, vp],
        "dp_layernorm": [vp, i64, vp, vp, vp, i64, i32, i32, f32, i32, vp],
        "dp_layernorm_stats": [vp, i64, i32, i32, vp, i64, vp, vp, i32, vp],
        "dp_attention": [vp, vp, i32, i32, i32, i32, f32, i32, vp],
        "dp_attention_log2q": [vp, vp, i32, i32, i32, i32, i32, vp],
        "dp_normalize_u8": [vp, i32, i32, vp, i32, vp],
        "dp_resize_bilinear": [vp, i32, i32, i32, i32, vp, i32, i32, vp],
        "dp_resize": [vp, i32, i32, i32, i32, vp, i32, i32, i32, vp],
        "dp_patchify_pyramid": [vp, vp, i32, vp],
        "dp_vit_cls_rows": [vp, vp, vp, i32, vp],
        "dp_merge_windows": [vp, i32, i64, i32, i32, i32, vp, i32, vp],
        "dp_merge_windows_range": [vp, i32, i64, i32, i32, i32, i32, i32, vp, i32, vp],
        "dp_fov_tail": [vp, i32, vp, f32, vp, vp],
        "dp_infer_epilogue": [vp, i32, i32, vp, i32, f64, i32, i32, vp, vp, vp, vp],
        "dp_infer_epilogue_mode": [vp, i32, i32, vp, i32, f64, i32, i32, vp, vp, vp, i32, vp],
        "dp_gemm_workspace_size": [],
        "dp_gemm_workspace_check": [vp, vp, vp],
        "dp_resize_u8_cv": [vp, i32, i32, vp, i32, i32, i32, vp],
        "dp_depth_to_points": [vp, i32, i32, vp, f64, i32, vp, vp, vp, vp, vp],
        "dp_depth_to_image": [vp, i64, vp, vp, i32, i32, vp, vp],
        "dp_gemm_plan": [ctypes.POINTER(GemmArgs), ctypes.POINTER(i32), ctypes.POINTER(i32)],
    }
    for name, argtypes in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int
    lib.dp_gemm_workspace_size.restype = ctypes.c_int64
    lib.dp_gemm_debug_flags.argtypes = [ctypes.c_int]
    lib.dp_gemm_debug_flags.restype = ctypes.c_int
    ver = lib.dp_abi_version()
    if ver != DP_ABI_VERSION:
        raise DPError(f"{path} has ABI version {ver}, expected {DP_ABI_VERSION}; rebuild it")
    dbg = int(os.environ.get("DP_GEMM_DEBUG", "0") or 0)   # ablation / A-B switches (tools, bench)
    if dbg:
        lib.dp_gemm_debug_flags(dbg)
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        name = _ERRORS.get(rc, f"hipError {rc}")
        raise DPError(f"{what} failed: {name}")
