#!/usr/bin/env python3
"""Per-workgroup timeline of the big GEMM engine from in-kernel s_memrealtime stamps.

Needs the timing-only build: `make -C ml-depth-pro-video_amd/csrc stamps`
(-> depth_pro/_lib/libdp_mi355x_stamps.so).  For each shape it reports, in us,
the prologue (kernel entry -> first tile visible in LDS), the K loop and the
epilogue of each workgroup, the idle gap between consecutive workgroups on the
same CU, and the share of CU-time spent inside K loops over the kernel span.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("DP_MI355X_LIB", os.path.join(ROOT, "ml-depth-pro-video_amd", "depth_pro", "_lib",
                                                    "libdp_mi355x_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "ml-depth-pro-video_amd"))

import ctypes  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from depth_pro import _lib, ops  # noqa: E402
from depth_pro._lib import DP_TILE_BIG_256x128, DP_TILE_BIG_256x256  # noqa: E402

SHAPES = [  # (name, M, N, K, kw)
    ("qkv", 20195, 3072, 1024, {}),
    ("proj+res", 20195, 1024, 1024, {"acc": True}),
    ("fc1+gelu", 20195, 4096, 1024, {"gelu": True}),
    ("fc2+res", 20195, 1024, 4096, {"acc": True}),
    ("conv3x3 768^2 256->256", 768 * 768, 256, 2304, {"conv": 768}),
]


def analyse(st: np.ndarray) -> str:
    t0, t1, t2, t3, hw = (st[:, i].astype(np.int64) for i in range(5))
    us = 0.01  # 100 MHz ticks
    origin = t0.min()
    span = (t3.max() - origin) * us
    pro, loop, epi = (t1 - t0) * us, (t2 - t1) * us, (t3 - t2) * us
    hwid = hw & 0xFFFFFFFF
    cu = (hw >> 32) * 4096 + ((hwid >> 13) & 7) * 256 + ((hwid >> 12) & 1) * 16 + ((hwid >> 8) & 15)
    gaps, per_cu = [], {}
    for c in np.unique(cu):
        idx = np.where(cu == c)[0]
        idx = idx[np.argsort(t0[idx])]
        per_cu[c] = len(idx)
        for a, b in zip(idx[:-1], idx[1:]):
            gaps.append((t0[b] - t3[a]) * us)
    gaps = np.array(gaps) if gaps else np.zeros(1)
    ncu = len(per_cu)
    busy = loop.sum() / (ncu * span)
    first = (t0 - origin) * us
    return (f"wg={len(st)} cus={ncu} span={span:.1f}us | pro {np.median(pro):.2f} (p90 {np.percentile(pro, 90):.2f})"
            f" loop {np.median(loop):.2f} (p10 {np.percentile(loop, 10):.2f} p90 {np.percentile(loop, 90):.2f})"
            f" epi {np.median(epi):.2f} (p90 {np.percentile(epi, 90):.2f}) | gap {np.median(gaps):.2f}"
            f" (p90 {np.percentile(gaps, 90):.2f}) | last-start {first.max():.1f} | K-loop share {busy:.2f}"
            f" | wg/cu {min(per_cu.values())}-{max(per_cu.values())}")


def main():
    lib = _lib.load()
    stamps_fn = lib.dp_gemm_stamps
    stamps_fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    for name, M, N, K, kw in SHAPES:
        B = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(dt)
        bias = torch.randn(N, device=dev, generator=g)
        if "conv" in kw:
            S = kw["conv"]
            A = torch.randn(S * S, K // 9, device=dev, generator=g).to(dt)
            conv = dict(in_h=S, in_w=S, in_c=K // 9, k=3, stride=1, pad=1, out_h=S, out_w=S)
        else:
            A = torch.randn(M, K, device=dev, generator=g).to(dt)
            conv = None
        C = torch.zeros(M, N, device=dev, dtype=torch.float32 if kw.get("acc") else dt)
        for tname, tile, bn in (("big256x256", DP_TILE_BIG_256x256, 256), ("big256x128", DP_TILE_BIG_256x128, 128)):
            if N % bn:
                continue
            nwg = ((M + 255) // 256) * ((N + bn - 1) // bn)
            for _ in range(4):
                ops.gemm(A, B, C, M=M, N=N, K=K, conv=conv, bias=bias, act=2 if kw.get("gelu") else 0,
                         accumulate=bool(kw.get("acc")), tile=tile)
            torch.cuda.synchronize()
            st = np.zeros((nwg, 5), dtype=np.uint64)
            rc = stamps_fn(st.ctypes.data, nwg)
            assert rc == 0, rc
            print(f"{name:24s} {tname}: {analyse(st)}", flush=True)


if __name__ == "__main__":
    main()
