#!/usr/bin/env python3
"""The ViT fc1 as the frame runs it (folded-LN consumer + GELU on the persistent 8-phase engine,
M = 20195, N = 4096, K = 1024, incl. the ln_merge pre-pass), against `--dbg` variants of the
library (dp_gemm_debug_flags), interleaved rounds, average launch time by HIP events.
Round 5 (profiles/r05c_fc1_half_tile/): a half-tile persistent engine (the epilogue drained one
fragment per K step of the next 128 x 256 half tile) ran 235 vs 168 us here and was removed."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ml-depth-pro-video_amd"))
from depth_pro import _lib, ops  # noqa: E402
from depth_pro._lib import DP_ACT_GELU  # noqa: E402


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--dbg", type=int, default=0, help="debug flags of the variant timed beside the default")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    M, N, K = 20195, 4096, 1024
    x = torch.randn(M, K, device=dev, generator=g) * 2
    xb = torch.empty(M, K, dtype=dt, device=dev)
    part = torch.empty(M, K // 128, 2, device=dev)
    ops.layernorm_stats(x, xb, part, M, K)
    w = torch.randn(N, K, device=dev, generator=g) * K ** -0.5
    wf, bf, sf = ops.fold_layernorm(w, torch.zeros(N, device=dev), torch.ones(K, device=dev),
                                    torch.zeros(K, device=dev), dt)
    out = torch.empty(M, N, dtype=dt, device=dev)
    ws = ops.gemm_workspace(dev)
    lib = _lib.load()
    f = lambda: ops.gemm(xb, wf, out, M=M, N=N, K=K, bias=bf, act=DP_ACT_GELU, ln_in=(part, sf), workspace=ws)  # noqa
    flop = 2.0 * M * N * K
    res = {"default": [], f"dbg {args.dbg}": []}
    for _ in range(5):
        for name, dbg in (("default", 0), (f"dbg {args.dbg}", args.dbg)):
            lib.dp_gemm_debug_flags(dbg)
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1000.0 / 20)
    lib.dp_gemm_debug_flags(0)
    for name, v in res.items():
        v = sorted(v)
        print(f"fc1 (LN consumer + GELU + merge pre-pass) {name:10s} median {v[2]:7.1f} us  min {v[0]:7.1f} us  "
              f"{flop / v[2] / 1e6:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
