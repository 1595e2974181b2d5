#!/usr/bin/env python3
"""Time dp_gemm tile engines on the Depth Pro GEMM shapes vs torch.matmul (hipBLASLt) on the same data."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ml-depth-pro-video_amd"))
from depth_pro import ops  # noqa: E402
from depth_pro._lib import (DP_TILE_128x128, DP_TILE_256x64, DP_TILE_8PH_256x256, DP_TILE_BIG_256x128,  # noqa
                            DP_TILE_BIG_256x128_K32, DP_TILE_BIG_256x256, DP_TILE_BIG_256x256_K32,
                            DP_TILE_DEEP4_256x256, DP_TILE_DEEP5_256x256, DP_TILE_DEEP_256x128,
                            DP_TILE_STREAMK_256x256, DP_TILE_BIG_320x256, DP_TILE_BIG_512x128,
                            DP_TILE_PBIG_320x256, DP_TILE_PBIG_256x256, DP_TILE_DUAL_256x128,
                            DP_TILE_P8PH_256x256, DP_TILE_8PH_320x256, DP_TILE_CV3_256x256,
                            DP_TILE_SPLITK_256x256, DP_TILE_CV3_192x256, DP_TILE_CV3_384x128)

TILES = (("auto", 0), ("big256x256", DP_TILE_BIG_256x256), ("big256x128", DP_TILE_BIG_256x128),
         ("8ph256x256", DP_TILE_8PH_256x256), ("deep4_256x256", DP_TILE_DEEP4_256x256),
         ("deep5_256x256", DP_TILE_DEEP5_256x256), ("deep6_256x128", DP_TILE_DEEP_256x128),
         ("sk256x256", DP_TILE_STREAMK_256x256), ("big320x256", DP_TILE_BIG_320x256),
         ("small128x128", DP_TILE_128x128), ("big512x128", DP_TILE_BIG_512x128), ("small256x64", DP_TILE_256x64),
         ("pbig320x256", DP_TILE_PBIG_320x256), ("pbig256x256", DP_TILE_PBIG_256x256),
         ("dual256x128", DP_TILE_DUAL_256x128), ("p8ph256x256", DP_TILE_P8PH_256x256),
         ("8ph320x256", DP_TILE_8PH_320x256), ("cv3_256x256", DP_TILE_CV3_256x256),
         ("splitk256x256", DP_TILE_SPLITK_256x256), ("cv3_192x256", DP_TILE_CV3_192x256),
         ("cv3_384x128", DP_TILE_CV3_384x128))
N256 = (DP_TILE_BIG_256x256, DP_TILE_BIG_256x256_K32, DP_TILE_8PH_256x256, DP_TILE_DEEP4_256x256,
        DP_TILE_DEEP5_256x256, DP_TILE_STREAMK_256x256, DP_TILE_BIG_320x256, DP_TILE_PBIG_320x256,
        DP_TILE_PBIG_256x256, DP_TILE_P8PH_256x256, DP_TILE_8PH_320x256, DP_TILE_CV3_256x256,
        DP_TILE_SPLITK_256x256, DP_TILE_CV3_192x256)

SHAPES = [  # (name, M, N, K, kw)
    ("qkv", 20195, 3072, 1024, {}),
    ("proj+res", 20195, 1024, 1024, {"acc": True}),
    ("fc1+gelu", 20195, 4096, 1024, {"gelu": True}),
    ("fc1 nogelu", 20195, 4096, 1024, {}),
    ("sq4096", 4096, 4096, 4096, {}),
    ("fc2+res", 20195, 1024, 4096, {"acc": True}),
    ("conv3x3 768^2 256->256", 768 * 768, 256, 2304, {"conv": 768}),
    ("conv3x3 384^2 256->256", 384 * 384, 256, 2304, {"conv": 384}),
    ("conv3x3 192^2 256->256", 192 * 192, 256, 2304, {"conv": 192}),
    ("conv3x3 96^2 256->256", 96 * 96, 256, 2304, {"conv": 96}),
    ("conv3x3 48^2 256->256", 48 * 48, 256, 2304, {"conv": 48}),
    # ResidualBlock second conv: ReLU prologue + residual epilogue (f16, as the decoder runs it)
    ("rb conv 768^2", 768 * 768, 256, 2304, {"conv": 768, "rb": True}),
    ("rb conv 384^2", 384 * 384, 256, 2304, {"conv": 384, "rb": True}),
    ("rb conv 192^2", 192 * 192, 256, 2304, {"conv": 192, "rb": True}),
    ("rb conv 96^2", 96 * 96, 256, 2304, {"conv": 96, "rb": True}),
    ("rb conv 48^2", 48 * 48, 256, 2304, {"conv": 48, "rb": True}),
    ("proj conv 48^2 1024->256", 48 * 48, 256, 9216, {"conv": 48}),
    ("proj conv 96^2 1024->256", 96 * 96, 256, 9216, {"conv": 96}),
    ("head conv 768^2 256->128", 768 * 768, 128, 2304, {"conv": 768}),
    ("composed head 768^2 128->4x32", 768 * 768, 128, 1152, {"conv": 768}),
    ("deconv 384->768 256ch", 384 * 384, 1024, 256, {"deconv": (384, 384, 256)}),
    ("plain 384^2 x 1024 K256 (the deconv's GEMM, row store)", 384 * 384, 1024, 256, {}),
    ("deconv 192->384 256ch", 192 * 192, 1024, 256, {"deconv": (192, 192, 256)}),
]


from depth_pro._lib import DPError  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None, help="substring of one shape name")
    ap.add_argument("--tile", default=None, help="128x128 | big256x256 | big256x128")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--torch-only", action="store_true", help="time only torch.matmul (hipBLASLt) on the dense shapes")
    ap.add_argument("--dbg", type=int, default=0, help="dp_gemm_debug_flags for every run (8 = direct epilogue)")
    ap.add_argument("--ablate", action="store_true", help="time the no-store / no-load / no-mfma variants")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    ws = ops.gemm_workspace(dev)
    if args.dbg:
        from depth_pro import _lib
        _lib.load().dp_gemm_debug_flags(args.dbg)
    for name, M, N, K, kw in SHAPES:
        if args.only and args.only not in name:
            continue
        dt = torch.float16 if kw.get("rb") or "proj conv" in name else torch.bfloat16
        B = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(dt)
        bias = torch.randn(N, device=dev, generator=g)
        if "conv" in kw:
            S = kw["conv"]
            cin = K // 9
            A = torch.randn(S * S, cin, device=dev, generator=g).to(dt)
            conv = dict(in_h=S, in_w=S, in_c=cin, k=3, stride=1, pad=1, out_h=S, out_w=S)
        else:
            A = torch.randn(M, K, device=dev, generator=g).to(dt)
            conv = None
        C = torch.zeros(M, N, device=dev, dtype=torch.float32 if kw.get("acc") else dt)
        R1 = torch.randn(M, N, device=dev, generator=g).to(dt) if kw.get("rb") else None
        dc = kw.get("deconv")
        flop = 2.0 * M * N * K
        res = []
        for tname, tile in (() if args.torch_only else TILES):
            if tile in N256 and N % 256:
                continue
            if args.tile and tname not in args.tile.split(","):
                continue
            f = lambda: ops.gemm(A, B, C, M=M, N=N, K=K, conv=conv, bias=bias, act=2 if kw.get("gelu") else 0,
                                 accumulate=bool(kw.get("acc")), tile=tile, workspace=ws, deconv=dc,
                                 ldc=dc[2] if dc else None, relu_a=bool(kw.get("rb")),
                                 R1=R1, ldr1=N if R1 is not None else 0)  # noqa: E731
            try:
                ms = timeit(f, args.iters)
            except DPError:
                res.append(f"{tname} n/a")
                continue
            res.append(f"{tname} {ms*1e3:8.1f}us {flop/ms/1e9:7.1f}TF")
            if args.ablate and (tname.startswith("big") or tname.startswith("8ph") or tname.startswith("p8")
                                or tname.startswith("dual") or tname.startswith("cv3")):
                from depth_pro import _lib
                parts = []
                abl = ((1, "nostore"), (2, "noload"), (3, "nostore+noload"), (4, "nomfma"), (5, "nomfma+nostore"))
                if not tname.startswith("big") and not tname.startswith("cv3"):
                    abl = abl[:1]
                for flags, lab in abl:
                    _lib.load().dp_gemm_debug_flags(flags)
                    parts.append(f"{lab} {timeit(f, args.iters)*1e3:.1f}")
                _lib.load().dp_gemm_debug_flags(args.dbg)
                res.append("[" + " ".join(parts) + "]")
        # correctness of the big engine vs the small one on this shape
        if not kw.get("acc") and not kw.get("rb") and not dc and not args.tile and not args.torch_only:
            C1 = torch.empty_like(C)
            ops.gemm(A, B, C1, M=M, N=N, K=K, conv=conv, bias=bias, tile=DP_TILE_128x128)
            C2 = torch.empty_like(C)
            d = 0.0
            for _, t in TILES:
                if t in N256 and N % 256:
                    continue
                try:
                    ops.gemm(A, B, C2, M=M, N=N, K=K, conv=conv, bias=bias, tile=t, workspace=ws)
                except DPError:
                    continue
                d = max(d, (C1.float() - C2.float()).abs().max().item())
            res.append(f"max|small-big|={d:.2e}")
        if conv is None and not dc and (not args.tile or args.torch_only):
            ms = timeit(lambda: torch.matmul(A, B.t()))
            res.append(f"torch.matmul {ms*1e3:8.1f}us {flop/ms/1e9:7.1f}TF")
        print(f"{name:28s} " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
