"""The C-ABI library loads and exports exactly what include/dp_mi355x.h declares (no GPU needed)."""

import ctypes
import os
import re
import subprocess

import pytest

from depth_pro import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "dp_mi355x.h")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int64_t) (dp_\w+)\(", src, flags=re.M)))


def test_header_and_python_export_lists_agree():
    assert declared() == sorted(_lib.EXPORTS)


def test_library_loads_and_exports_every_symbol():
    lib = _lib.load()
    for name in declared():
        assert hasattr(lib, name), name
    assert lib.dp_abi_version() == _lib.DP_ABI_VERSION


def test_gemm_args_struct_layout_matches_c(tmp_path):
    """ctypes GemmArgs == sizeof/offsetof of the C struct (compiled with gcc)."""
    fields = [f for f, _ in _lib.GemmArgs._fields_]
    prog = tmp_path / "lay.c"
    body = "".join(f'printf("%zu\\n", offsetof(dp_gemm_args, {f}));' for f in fields)
    prog.write_text(f'#include <stdio.h>\n#include <stddef.h>\n#include "{HEADER}"\n'
                    f'int main(void){{printf("%zu\\n", sizeof(dp_gemm_args));{body}return 0;}}\n')
    exe = tmp_path / "lay"
    subprocess.run(["gcc", "-std=c11", str(prog), "-o", str(exe)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(_lib.GemmArgs)
    for f, off in zip(fields, vals[1:]):
        assert getattr(_lib.GemmArgs, f).offset == off, f


def test_argument_errors_are_reported_before_launch():
    """Shape/alignment errors return DP_ERR_* without touching the GPU (null stream, no device)."""
    lib = _lib.load()
    a = _lib.GemmArgs()
    a.M, a.N, a.K = 16, 16, 60  # K % 64 != 0
    a.A = a.B = a.C = 16
    a.lda = a.ldb = 64
    assert lib.dp_gemm(ctypes.byref(a), None) == 1001
    a.K = 64
    a.ldb = 12
    assert lib.dp_gemm(ctypes.byref(a), None) == 1002
    assert lib.dp_attention(16, 16, 1, 577, 16, 128, 0.1, 0, None) == 1001
    with pytest.raises(_lib.DPError, match="DP_ERR_SHAPE"):
        _lib.check(1001, "x")


def test_gemm_plan_tile_choice():
    """dp_gemm_plan (host-only): engine choice for the frame's GEMM shapes (tile, workgroups)."""
    lib = _lib.load()
    t, g = ctypes.c_int32(), ctypes.c_int32()

    def plan(M, N, K, **kw):
        a = _lib.GemmArgs()
        a.M, a.N, a.K = M, N, K
        a.A = a.B = a.C = 256
        a.lda, a.ldb, a.ldc = K, K, N
        for k, v in kw.items():
            setattr(a, k, v)
        rc = lib.dp_gemm_plan(ctypes.byref(a), ctypes.byref(t), ctypes.byref(g))
        return rc, t.value, g.value

    # ViT-L patch encoder (M = 35 x 577 = 20195 = 64 tiles of 320 rows)
    # qkv / proj: the 8-phase 320 x 256 engine; fc1: the persistent 8-phase engine (one workgroup per CU)
    assert plan(20195, 3072, 1024)[1:] == (_lib.DP_TILE_8PH_320x256, 64 * 12)
    assert plan(20195, 1024, 1024)[1:] == (_lib.DP_TILE_8PH_320x256, 64 * 4)     # one round on 256 CUs
    assert plan(20195, 4096, 1024)[1:] == (_lib.DP_TILE_P8PH_256x256, 256)
    # the previous engines stay reachable (A/B switches in the planner, explicit tile hints)
    assert plan(20195, 4096, 1024, tile=_lib.DP_TILE_8PH_256x256)[1:] == (_lib.DP_TILE_8PH_256x256, 79 * 16)
    assert plan(20195, 1024, 1024, tile=_lib.DP_TILE_BIG_320x256)[1:] == (_lib.DP_TILE_BIG_320x256, 64 * 4)
    assert plan(577, 3072, 1024)[1:] == (_lib.DP_TILE_BIG_256x128, 3 * 24)       # side encoders
    assert plan(768 * 768, 128, 2304)[1:] == (_lib.DP_TILE_BIG_512x128, 1152)     # head.0 conv (N = 128)
    # past 2^31 elements of A (M * lda) or B (N * ldb): only the engines with 64-bit operand
    # pointers (the 8-phase 320 x 256 and the persistent engines keep 32-bit element offsets)
    big_m = (1 << 21) + 5                                   # 2097157 x 1024 >= 2^31
    assert plan(big_m, 1024, 1024)[1:] == (_lib.DP_TILE_BIG_320x256, 6554 * 4)
    off32 = {_lib.DP_TILE_8PH_320x256, _lib.DP_TILE_P8PH_256x256, _lib.DP_TILE_PBIG_320x256,
             _lib.DP_TILE_PBIG_256x256}
    assert plan(big_m, 4096, 1024)[1] not in off32
    assert plan(big_m, 1024, 1024, tile=_lib.DP_TILE_8PH_320x256)[0] == 1000
    assert plan(big_m, 4096, 1024, tile=_lib.DP_TILE_P8PH_256x256)[0] == 1000
    assert plan(big_m - 8, 1024, 1024)[1] in off32                      # 2097149 x 1024 < 2^31
    # stream-K is opt-in and needs a workspace
    assert plan(20195, 3072, 1024, tile=_lib.DP_TILE_STREAMK_256x256)[0] == 1000
    ws = lib.dp_gemm_workspace_size()
    rc, tile, wgs = plan(20195, 3072, 1024, tile=_lib.DP_TILE_STREAMK_256x256, workspace=256, workspace_bytes=ws)
    assert rc == 0 and tile == _lib.DP_TILE_STREAMK_256x256 and 1 <= wgs <= 256

    # decoder 3x3 convs: long-K projections with < 1 tile per CU go to stream-K with
    # split K ranges (needs a workspace); K = 2304 small grids stay data-parallel
    def conv(S, cin, **kw):
        return plan(S * S, 256, 9 * cin, a_mode=_lib.DP_A_CONV, in_h=S, in_w=S, in_c=cin, k_h=3, k_w=3,
                    stride=1, pad=1, out_h=S, out_w=S, **kw)
    wsk = dict(workspace=256, workspace_bytes=ws)
    assert conv(48, 1024, **wsk)[1:] == (_lib.DP_TILE_STREAMK_256x256, 9 * 6)     # 9 tiles x split 6
    assert conv(96, 1024, **wsk)[1:] == (_lib.DP_TILE_STREAMK_256x256, 36 * 6)    # 36 tiles x split 6
    # 192^2 x 512 channels: 144 tiles of 16 x 16 px would leave 112 CUs idle -- 12-row patch-conv tiles
    # (192 workgroups, one round; the planner rule of DP_TILE_CV3_192x256)
    assert conv(192, 512, **wsk)[1:] == (_lib.DP_TILE_CV3_192x256, 192)
    assert conv(48, 1024)[1] != _lib.DP_TILE_STREAMK_256x256                        # no workspace
    assert conv(48, 256, **wsk)[1] == _lib.DP_TILE_BIG_256x128                     # K = 2304
    # split-K + reduce: an explicit hint (needs a workspace); split = min(CUs / tiles, K steps / 2,
    # workspace slabs, 32)
    SPK = _lib.DP_TILE_SPLITK_256x256
    assert conv(48, 1024, tile=SPK, **wsk)[1:] == (SPK, 9 * 28)
    assert conv(96, 1024, tile=SPK, **wsk)[1:] == (SPK, 36 * 7)                      # 7 slabs of 9.4 MB
    assert conv(48, 256, tile=SPK, **wsk)[1:] == (SPK, 9 * 18)                       # 36 K steps / 2
    assert conv(48, 256, tile=SPK)[0] == 1000                                        # no workspace
    assert conv(768, 256, tile=SPK, **wsk)[0] == 1001                                # 2304 tiles: no split
    # the 768^2 ResidualBlock convs (2304 tiles of 256 pixels): the 3x3 patch-conv engine; 384^2 not
    assert conv(768, 256, **wsk)[1:] == (_lib.DP_TILE_CV3_256x256, 2304)
    assert conv(384, 256, **wsk)[1] != _lib.DP_TILE_CV3_256x256
    # the head convs at 768^2 (128 output channels): the composed out_conv∘head.0 with its border
    # correction on the patch-conv engine (debug 4096: the 512 x 128 engine); the composed depth
    # head (HEAD_PS) on the 512 x 128 engine unless the patch-conv engine is asked for
    def head(**kw):
        return plan(768 * 768, 128, 9 * kw.pop("cin"), a_mode=_lib.DP_A_CONV, in_h=768, in_w=768, k_h=3, k_w=3,
                    stride=1, pad=1, out_h=768, out_w=768, head_corr=256, **kw)
    h0c = dict(cin=256, in_c=256)
    hps = dict(cin=128, in_c=128, store_mode=_lib.DP_STORE_HEAD_PS, head_w=256, c_dtype=_lib.DP_F32)
    assert head(**h0c)[1:] == (_lib.DP_TILE_CV3_384x128, 1536)                       # 24 x 16-pixel tiles
    assert head(**h0c, tile=_lib.DP_TILE_CV3_256x256)[1:] == (_lib.DP_TILE_CV3_256x256, 2304)
    assert head(**hps)[1:] == (_lib.DP_TILE_BIG_512x128, 1152)
    assert head(**hps, tile=_lib.DP_TILE_CV3_256x256)[1:] == (_lib.DP_TILE_CV3_256x256, 2304)
    assert head(**hps, tile=_lib.DP_TILE_CV3_384x128)[1:] == (_lib.DP_TILE_CV3_384x128, 1536)
    assert head(**hps, tile=_lib.DP_TILE_BIG_256x128)[1:] == (_lib.DP_TILE_BIG_256x128, 2304)
    assert head(**hps, tile=_lib.DP_TILE_BIG_256x256)[1:] == (_lib.DP_TILE_BIG_512x128, 1152)    # not a HEAD_PS engine
    # the decoder's 2x2 deconvs with >= 128 tiles of 256 x 256: the persistent 8-phase engine with
    # the pixel-shuffle store; fewer tiles stay where they were
    def deconv(S, cin, cout, **kw):
        return plan(S * S, 4 * cout, cin, store_mode=_lib.DP_STORE_DECONV2X2, dc_h=S, dc_w=S, dc_cout=cout,
                    ldc=cout, dtype=_lib.DP_F16, c_dtype=_lib.DP_F16, bias=256, **kw)
    assert deconv(384, 256, 256, **wsk)[1:] == (_lib.DP_TILE_P8PH_256x256, 256)
    assert deconv(192, 256, 256, **wsk)[1:] == (_lib.DP_TILE_P8PH_256x256, 256)
    assert deconv(96, 512, 512, **wsk)[1:] == (_lib.DP_TILE_P8PH_256x256, 256)     # 288 tiles
    assert deconv(96, 256, 256, **wsk)[1:] == (_lib.DP_TILE_P8PH_256x256, 144)     # 144 tiles, one round
    assert deconv(48, 256, 256, **wsk)[1] != _lib.DP_TILE_P8PH_256x256             # 36 tiles
    assert deconv(384, 256, 256, act=_lib.DP_ACT_RELU, **wsk)[1] != _lib.DP_TILE_P8PH_256x256
    lib.dp_gemm_debug_flags(4096)
    try:
        assert head(**h0c)[1:] == (_lib.DP_TILE_BIG_512x128, 1152)
        assert head(**hps)[1:] == (_lib.DP_TILE_BIG_512x128, 1152)
    finally:
        lib.dp_gemm_debug_flags(0)
    lib.dp_gemm_debug_flags(1 << 23)
    try:
        assert deconv(384, 256, 256, **wsk)[1] == _lib.DP_TILE_STREAMK_256x256
    finally:
        lib.dp_gemm_debug_flags(0)


def test_empty_inputs_are_refused_before_launch():
    """Zero-size inputs (no rows / images / pixels) return DP_ERR_SHAPE (DP_ERR_ARG for an empty
    group list) from every entry point that takes a size, before any launch (no GPU here: a launch
    would return a HIP error instead).  The reference's torch ops raise on these shapes too."""
    lib = _lib.load()
    P = 4096                      # a dummy non-null pointer: never dereferenced on the host
    f32, f64 = ctypes.c_float, ctypes.c_double
    a = _lib.GemmArgs()
    a.M, a.N, a.K = 0, 64, 64
    a.A = a.B = a.C = P
    a.lda = a.ldb = a.ldc = 64
    calls = {
        "gemm M=0": lambda: lib.dp_gemm(ctypes.byref(a), None),
        "attention batch=0": lambda: lib.dp_attention(P, P, 0, 577, 16, 64, f32(0.125), 0, None),
        "attention seq=0": lambda: lib.dp_attention(P, P, 1, 0, 16, 64, f32(0.125), 0, None),
        "attention_log2q heads=0": lambda: lib.dp_attention_log2q(P, P, 1, 577, 0, 64, 0, None),
        "layernorm rows=0": lambda: lib.dp_layernorm(P, 1024, P, P, P, 1024, 0, 1024, f32(1e-6), 0, None),
        "layernorm_stats rows=0": lambda: lib.dp_layernorm_stats(P, 1024, 0, 1024, P, 1024, None, P, 0, None),
        "normalize_u8 H=0": lambda: lib.dp_normalize_u8(P, 0, 100, P, 0, None),
        "resize_bilinear OH=0": lambda: lib.dp_resize_bilinear(P, 0, 3, 10, 10, P, 0, 10, None),
        "resize H=0": lambda: lib.dp_resize(P, 0, 3, 0, 10, P, 10, 10, 0, None),
        "vit_cls_rows n=0": lambda: lib.dp_vit_cls_rows(P, P, P, 0, None),
        "infer_epilogue H=0": lambda: lib.dp_infer_epilogue(P, 1536, 1536, P, 0, f64(0), 0, 10, P, P, P, None),
        "resize_u8_cv OH=0": lambda: lib.dp_resize_u8_cv(P, 10, 10, P, 0, 5, 3, None),
        "depth_to_points H=0": lambda: lib.dp_depth_to_points(P, 0, 10, P, f64(1.0), 1, P, P, P, P, None),
        "depth_to_image n=0": lambda: lib.dp_depth_to_image(P, 0, P, P, 256, 0, P, None),
    }
    for name, call in calls.items():
        assert call() == 1001, name
    a.M, a.N = 64, 0
    assert lib.dp_gemm(ctypes.byref(a), None) == 1001
    a.N = 64
    assert lib.dp_gemm_grouped(ctypes.byref(a), 0, None) == 1000
