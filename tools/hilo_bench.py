#!/usr/bin/env python3
"""proj / fc2 residual GEMMs (the folded-LN producers, M = 20195, N = 1024) with the fp32 residual
stream vs the split one (16-bit hi + int8 lo): average launch time, warm (operands re-used, the stream
resident in the Infinity Cache) and cold (a 512 MB write between launches evicts it, as the frame's
other kernels do)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ml-depth-pro-video_amd"))
from depth_pro import ops  # noqa: E402


def timeit(fn, iters, flush=None):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    tot = 0.0
    for _ in range(iters):
        if flush is not None:
            flush()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        tot += e0.elapsed_time(e1)
    return 1000.0 * tot / iters


def main():
    dev = torch.device("cuda:0")
    dt = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    M, N = 20195, 1024
    junk = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    flush = lambda: junk.fill_(1)  # noqa: E731
    x = torch.randn(M, N, device=dev, generator=g) * 2
    hi, lo = ops.split_residual(x, dt)      # the 16-bit high part and the int8 low part
    part = torch.empty(M, N // 128, 2, device=dev)
    # the HBM floor of an epilogue that reads and writes the split stream once (3 + 3 B per element):
    # a plain device copy of the same 62 MB
    src = torch.empty(M * N * 3, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    for cl, fl in (("warm", None), ("cold", flush)):
        us = timeit(lambda: dst.copy_(src), 20, fl)
        print(f"copy {src.numel() / 1e6:.0f} MB ({cl}): {us:6.1f} us = {2 * src.numel() / us / 1e6:5.2f} TB/s", flush=True)
    for name, K in (("proj", 1024), ("fc2", 4096)):
        A = torch.randn(M, K, device=dev, generator=g).to(dt)
        B = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(dt)
        bias = torch.randn(N, device=dev, generator=g)
        gamma = torch.full((N,), 1e-3, device=dev)
        kw = dict(M=M, N=N, K=K, bias=bias, gamma=gamma, accumulate=True)
        xb = torch.empty(M, N, dtype=dt, device=dev)
        f32 = lambda: ops.gemm(A, B, x, ln_out=(xb, part), **kw)  # noqa: E731
        spl = lambda: ops.gemm(A, B, None, ln_out=(hi, part), ln_xl=lo, **kw)  # noqa: E731
        flop = 2.0 * M * N * K
        res = []
        from depth_pro import _lib
        lib = _lib.load()
        for lab, fn, dbg in (("fp32", f32, 0), ("split", spl, 0), ("split-touch", spl, 1 << 28),
                             ("split-ahead1", spl, 1 << 27), ("no-epilogue", spl, 1)):
            lib.dp_gemm_debug_flags(dbg)
            for cl, fl in (("warm", None), ("cold", flush)):
                us = timeit(fn, 20, fl)
                res.append(f"{lab}/{cl} {us:7.1f}us {flop / us / 1e6:6.1f}TF")
        lib.dp_gemm_debug_flags(0)
        print(f"{name:5s} " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
