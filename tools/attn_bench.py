#!/usr/bin/env python3
"""Time dp_attention on the Depth Pro ViT shapes vs torch SDPA on the same data."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ml-depth-pro-video_amd"))
from depth_pro import ops  # noqa: E402


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
    ap.add_argument("--quick", action="store_true", help="only the 35 x 577 bf16 case, no torch reference")
    ap.add_argument("--log2q", action="store_true", help="time dp_attention_log2q (what the engine runs)")
    ap.add_argument("--seq", type=int, default=577, help="sequence length of the --quick case")
    ap.add_argument("--batch", type=int, default=35, help="images of the --quick case")
    ap.add_argument("--ablate", action="store_true",
                    help="35 x 577 with each stage dropped in turn (needs the ablation build: make attnexp, "
                         "DP_MI355X_LIB=.../libdp_mi355x_attnexp.so)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    H, hd = 16, 64
    if args.ablate:
        from depth_pro import _lib
        lib = _lib.load()
        batch, seq = 35, 577
        qkv = torch.randn(batch * seq, 3 * H * hd, device=dev).to(torch.bfloat16)
        out = torch.empty(batch * seq, H * hd, dtype=torch.bfloat16, device=dev)
        flop = 4.0 * batch * H * seq * seq * hd
        for flags, lab in ((0, "full"), (1, "no exp"), (16, "no row sums"), (17, "no exp+sums"), (2, "no PV"),
                           (4, "no tile wait/barrier"), (8, "no K/V DMA"), (10, "no DMA+PV"), (15, "S MFMA only")):
            lib.dp_attn_debug_flags(flags)
            ms = timeit(lambda: ops.attention(qkv, out, batch, seq, H, hd, log2q=True))
            print(f"{lab:22s} {ms*1e3:7.1f}us {flop/ms/1e9:6.1f}TF", flush=True)
        lib.dp_attn_debug_flags(0)
        return
    cases = ((args.batch, args.seq),) if args.quick else ((35, 577), (1, 577), (8, 2048))
    for batch, seq in cases:
        for dt in ((torch.bfloat16,) if args.quick else (torch.bfloat16, torch.float16)):
            qkv = torch.randn(batch * seq, 3 * H * hd, device=dev)
            if args.log2q:   # the engine's qkv epilogue scales Q by hd^-0.5 * log2 e
                qkv[:, :H * hd] *= hd ** -0.5 * 1.4426950408889634
            qkv = qkv.to(dt)
            out = torch.empty(batch * seq, H * hd, dtype=dt, device=dev)
            flop = 4.0 * batch * H * seq * seq * hd
            ms = timeit(lambda: ops.attention(qkv, out, batch, seq, H, hd, log2q=args.log2q))
            if args.quick:
                print(f"b={batch} seq={seq} dp {ms*1e3:.1f}us {flop/ms/1e9:.1f}TF", flush=True)
                continue
            q, k, v = qkv.reshape(batch, seq, 3, H, hd).permute(2, 0, 3, 1, 4).unbind(0)
            ref = F.scaled_dot_product_attention(q.float(), k.float(), v.float()).transpose(1, 2).reshape(batch * seq, -1)
            err = (out.float() - ref).abs().max().item()
            qc, kc, vc = q.contiguous(), k.contiguous(), v.contiguous()
            ms_t = timeit(lambda: F.scaled_dot_product_attention(qc, kc, vc))
            print(f"b={batch:3d} seq={seq} {str(dt):15s} dp {ms*1e3:7.1f}us {flop/ms/1e9:6.1f}TF  max|err|={err:.2e}"
                  f" | torch sdpa {ms_t*1e3:7.1f}us {flop/ms_t/1e9:6.1f}TF", flush=True)


if __name__ == "__main__":
    main()
