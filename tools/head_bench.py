#!/usr/bin/env python3
"""The depth head's two 768^2 convs alone (the composed out_conv∘head.0 conv, N = 128 with its
border correction; the composed ConvTranspose + conv + ReLU + 1x1 head with the pixel-shuffle
store, DP_STORE_HEAD_PS), on random operands: average launch time over 2 s of launches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ml-depth-pro-video_amd"))
from depth_pro import ops  # noqa: E402


def timeit(fn, seconds=1.5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 0
    e0.record()
    while True:
        for _ in range(10):
            fn()
        n += 10
        e1.record()
        torch.cuda.synchronize()
        if e0.elapsed_time(e1) > 1000 * seconds:
            return 1000 * e0.elapsed_time(e1) / n


def main():
    dev = torch.device("cuda:0")
    dt = torch.float16
    g = torch.Generator(device=dev).manual_seed(0)
    S = 768
    feats = torch.randn(S * S, 256, device=dev, generator=g).to(dt)
    w0 = (torch.randn(128, 9 * 256, device=dev, generator=g) * 0.02).to(dt)
    b0 = torch.randn(128, device=dev, generator=g)
    corr0 = torch.randn(9 * 128, device=dev, generator=g) * 0.01
    h0 = torch.empty(S * S, 128, device=dev, dtype=dt)
    wps = (torch.randn(128, 9 * 128, device=dev, generator=g) * 0.03).to(dt)
    bps = torch.randn(128, device=dev, generator=g)
    corr = torch.randn(9 * 32, device=dev, generator=g) * 0.01
    hw = torch.randn(32, device=dev, generator=g)
    out = torch.empty(1, 1, 2 * S, 2 * S, device=dev)
    conv = lambda cin: dict(in_h=S, in_w=S, in_c=cin, k=3, stride=1, pad=1, out_h=S, out_w=S)  # noqa: E731
    f0 = lambda: ops.gemm(feats, w0, h0, M=S * S, N=128, K=9 * 256, conv=conv(256), bias=b0,  # noqa: E731
                          border_corr=corr0)
    ps_tile = int(os.environ.get("HEAD_PS_TILE", "0"))   # an explicit tile for head.ps (A/B)
    f1 = lambda: ops.gemm(h0, wps, out, M=S * S, N=128, K=9 * 128, conv=conv(128), bias=bps,  # noqa: E731
                          head_w=hw, head_b=0.1, head_corr=corr, tile=ps_tile)
    for lab, f, fl in (("head.0c (composed out_conv∘head.0)", f0, 2.0 * S * S * 128 * 2304),
                       ("head.ps (composed deconv + conv + 1x1)", f1, 2.0 * S * S * 128 * 1152)):
        us = timeit(f)
        print(f"{lab:40s} {us:7.1f} us  {fl / us / 1e6:6.1f} TF", flush=True)
    if "--ablate" in sys.argv:
        # the big engine's timing ablations (dp_gemm_debug_flags; results are wrong): what bounds head.ps
        from depth_pro import _lib
        lib = _lib.load()
        for lab, dbg in (("no epilogue", 1), ("no loads in the K loop", 2), ("no MFMA (one fragment read)", 4),
                         ("no loads, no epilogue", 3)):
            lib.dp_gemm_debug_flags(dbg)
            us = timeit(f1)
            lib.dp_gemm_debug_flags(0)
            print(f"head.ps, {lab:34s} {us:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
