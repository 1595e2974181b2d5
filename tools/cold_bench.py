#!/usr/bin/env python3
"""proj / fc2 (fp32 residual accumulate, 8-phase 320 x 256) with the residual stream cold vs warm in
the caches: between timed calls a 512 MiB buffer is rewritten (evicts L2 and MALL), the GEMM alone is
timed with HIP events.  Tells whether the epilogue's x reads pay for a cold residual stream."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ml-depth-pro-video_amd"))
from depth_pro import ops  # noqa: E402
from depth_pro._lib import DP_TILE_8PH_320x256  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    for name, M, N, K in (("proj", 20195, 1024, 1024), ("fc2", 20195, 1024, 4096)):
        A = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        B = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
        bias = torch.randn(N, device=dev, generator=g)
        gamma = torch.rand(N, device=dev, generator=g)
        X = torch.randn(M, N, device=dev, generator=g)
        f = lambda: ops.gemm(A, B, X, M=M, N=N, K=K, bias=bias, gamma=gamma, accumulate=True,  # noqa: E731
                             tile=DP_TILE_8PH_320x256)
        for _ in range(3):
            f()
        res = {}
        for mode in ("warm", "cold_all", "cold_x_only"):
            ts = []
            for _ in range(10):
                if mode == "cold_all":
                    flush.fill_(1)
                elif mode == "cold_x_only":
                    flush.fill_(1)
                    A.add_(0)          # re-touch A and B (warm), x stays cold
                    B.add_(0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            ts.sort()
            res[mode] = ts[len(ts) // 2]
        print(name, " ".join(f"{k} {v:.1f}us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
