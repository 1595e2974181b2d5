#!/usr/bin/env python3
"""Where a tile's time goes in the persistent 8-phase engine (the ViT fc1 and qkv: folded-LN
consumer epilogue, GELU for fc1), from per-tile s_memrealtime stamps of the timing-only build
(`make -C ml-depth-pro-video_amd/csrc stamps` -> libdp_mi355x_stamps.so; dp_gemm_impl.h DP_STAMPS).

Per workgroup and tile: [K loop start, K loop done, epilogue done (its stores issued)].  Reports, in
us (100 MHz stamps), the medians over all tiles of the K loop, the epilogue (folded LN + GELU + the
slab round trip + store issue), the boundary (epilogue done -> the next tile's K loop start: the
next tile's first A / constant DMA issue), the launch span and the share of it in K loops.

    DP_MI355X_LIB=.../libdp_mi355x_stamps.so python tools/p8ph_stamps.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("DP_MI355X_LIB", os.path.join(ROOT, "ml-depth-pro-video_amd", "depth_pro", "_lib",
                                                    "libdp_mi355x_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "ml-depth-pro-video_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from depth_pro import _lib, ops  # noqa: E402
from depth_pro._lib import DP_ACT_GELU, DP_TILE_P8PH_256x256  # noqa: E402

TILES, W = 8, 3 * 8 + 1


def analyse(st: np.ndarray, ntiles: np.ndarray) -> str:
    us = 0.01
    kl, ep, bd = [], [], []
    t0 = st[:, 0].astype(np.int64).min()
    t_end = 0
    for w in range(len(st)):
        n = int(ntiles[w])
        for i in range(min(n, TILES)):
            a, b, c = (int(st[w, 3 * i + j]) for j in range(3))
            kl.append((b - a) * us)
            ep.append((c - b) * us)
            t_end = max(t_end, c)
            if i + 1 < min(n, TILES):
                bd.append((int(st[w, 3 * (i + 1)]) - c) * us)
    span = (t_end - t0) * us
    busy = sum(kl) / (len(st) * span)
    q = lambda v: f"{np.median(v):6.2f} (p10 {np.percentile(v, 10):6.2f} p90 {np.percentile(v, 90):6.2f})"  # noqa: E731
    return (f"tiles/wg {int(ntiles.min())}-{int(ntiles.max())} | K loop {q(kl)} | epilogue {q(ep)} | boundary "
            f"{q(bd) if bd else '-'} | span {span:.1f} us | K-loop share of the CU-span {busy:.2f}")


def main():
    lib = _lib.load()
    fn = lib.dp_p8_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    M, K = 20195, 1024
    ws = ops.gemm_workspace(dev)
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--more", action="store_true",
                    help="also the fc1 shape without GELU, the qkv shape with it, and fc1 on 8- / 2-row tile bands")
    args = ap.parse_args()
    runs = [("fc1 (LN + GELU)", 4096, DP_ACT_GELU, 0), ("qkv (LN)", 3072, 0, 0)]
    if args.more:
        runs += [("fc1 shape, no GELU", 4096, 0, 0), ("qkv shape + GELU", 3072, DP_ACT_GELU, 0),
                 ("fc1, 8-row bands", 4096, DP_ACT_GELU, 1 << 18), ("fc1, 2-row bands", 4096, DP_ACT_GELU, 1 << 19)]
    for name, N, act, dbg in runs:
        lib.dp_gemm_debug_flags(dbg)
        A = torch.randn(M, K, device=dev, generator=g).to(dt)
        B = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(dt)
        bias = torch.randn(N, device=dev, generator=g)
        colsum = B.float().sum(1).contiguous()
        rs = torch.rand((M + 1) // 2 * 2 + 256, 2, device=dev, generator=g) + 0.5
        C = torch.empty(M, N, device=dev, dtype=dt)
        kw = dict(M=M, N=N, K=K, bias=bias, act=act, ln_in=(None, colsum), ln_rs_in=rs,
                  tile=DP_TILE_P8PH_256x256, workspace=ws)
        _, wgs = ops.gemm(A, B, C, plan_only=True, **kw)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            ops.gemm(A, B, C, **kw)
        e0.record()
        for _ in range(10):
            ops.gemm(A, B, C, **kw)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        st = np.zeros((wgs, W), dtype=np.uint64)
        assert fn(st.ctypes.data, wgs) == 0
        T = ((M + 255) // 256) * (N // 256)
        ntiles = np.array([(T - w + wgs - 1) // wgs for w in range(wgs)])
        print(f"{name:20s} {ms * 1e3:7.1f} us/launch (stamped build) | {analyse(st, ntiles)}", flush=True)
    lib.dp_gemm_debug_flags(0)


if __name__ == "__main__":
    main()
