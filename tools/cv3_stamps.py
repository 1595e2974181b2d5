#!/usr/bin/env python3
"""Per-workgroup clock stamps of the 3x3 patch-conv engine (debug bit 8, a diagnostic build of the
kernel: stamps at start, after the prologue DMA, after the K loop, after the epilogue's stores):
where a tile's time goes, in shader cycles, and the in-kernel clock under load.

    python tools/cv3_stamps.py [--size 768] [--no-res]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ml-depth-pro-video_amd"))
from depth_pro import _lib, ops  # noqa: E402
from depth_pro._lib import DP_TILE_CV3_192x256, DP_TILE_CV3_256x256  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=768)
    ap.add_argument("--no-res", action="store_true", help="no residual (a ResidualBlock's first conv)")
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--th", type=int, default=16, help="tile rows: 16 (DP_TILE_CV3_256x256) or 12 (..._192x256)")
    ap.add_argument("--abl", type=int, default=0, help="extra ablation bits with the stamps: 2 no loads, 4 no MFMA, "
                    "16 no barriers (timing only)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    S, cin, N = args.size, 256, 256
    g = torch.Generator(device=dev).manual_seed(0)
    dt = torch.float16
    A = torch.randn(S * S, cin, device=dev, generator=g).to(dt)
    B = (torch.randn(N, 9 * cin, device=dev, generator=g) * (9 * cin) ** -0.5).to(dt)
    bias = torch.randn(N, device=dev, generator=g)
    C = torch.empty(S * S, N, device=dev, dtype=dt)
    R1 = None if args.no_res else torch.randn(S * S, N, device=dev, generator=g).to(dt)
    conv = dict(in_h=S, in_w=S, in_c=cin, k=3, stride=1, pad=1, out_h=S, out_w=S)
    lib = _lib.load()

    def run():
        ops.gemm(A, B, C, M=S * S, N=N, K=9 * cin, conv=conv, bias=bias, relu_a=True, act=0 if R1 is not None else 1,
                 R1=R1, ldr1=N if R1 is not None else 0, tile=DP_TILE_CV3_256x256 if args.th == 16 else DP_TILE_CV3_192x256)

    # (the cv3 ablation / stamp variants are selected only with debug bit 1 << 24, dp_gemm_cv3.hip)
    for flags, lab in (((0, "plain"),) if not args.abl else ()) + (((1 << 24) | 8 | args.abl,
                                                                   f"stamped (bits {8 | args.abl})"),):
        lib.dp_gemm_debug_flags(flags)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 0
        e0.record()
        while True:
            for _ in range(20):
                run()
            n += 20
            e1.record()
            torch.cuda.synchronize()
            if e0.elapsed_time(e1) > 1000 * args.seconds:
                break
        print(f"{lab}: {1000 * e0.elapsed_time(e1) / n:.1f} us per launch ({n} launches)")
    lib.dp_gemm_debug_flags(0)
    nwg = (S // 16) * (S // args.th)
    buf = (ctypes.c_ulonglong * (nwg * 10))()
    lib.dp_cv3_stamps.restype = ctypes.c_int
    assert lib.dp_cv3_stamps(buf, nwg) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(nwg, 10).astype(np.float64)
    clk = (st[:, 3] - st[:, 0]) / ((st[:, 5] - st[:, 4]) / 100e6)   # shader cycles / s
    mhz = np.median(clk) / 1e6
    pro, loop, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
    tot = st[:, 3] - st[:, 0]
    kt = 9 * cin // 64
    print(f"in-kernel clock (median over workgroups): {mhz:.0f} MHz; tiles {nwg}")
    for lab, v in (("prologue (patch + 2 weight steps)", pro), ("K loop", loop), ("epilogue incl. store drain", epi),
                   ("workgroup", tot)):
        print(f"  {lab:36s} median {np.median(v):9.0f} cyc = {np.median(v) / mhz:7.2f} us  "
              f"(p10 {np.percentile(v, 10) / mhz:6.2f}, p90 {np.percentile(v, 90) / mhz:6.2f})")
    if args.abl & 256:
        for j, lab in ((6, "vmcnt waits"), (7, "barriers"), (8, "lgkmcnt waits before MFMAs"), (9, "MFMA issue")):
            print(f"  wave 0, K loop: {lab:28s} {np.median(st[:, j]) / kt:7.0f} cyc per step")
    print(f"  K loop per step: {np.median(loop) / kt:.0f} cyc (MFMA floor 2 waves x {8 * args.th // 2} MFMAs x 16 = {128 * args.th})")
    # workgroup rounds: start-time spread
    t0 = st[:, 0] - st[:, 0].min()
    print(f"  launch span {(st[:, 3].max() - st[:, 0].min()) / mhz:.1f} us")


if __name__ == "__main__":
    main()
