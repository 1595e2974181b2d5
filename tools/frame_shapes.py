#!/usr/bin/env python3
"""Per-(kernel, shape) time of one eager forward (side encoders serialised), with the
GEMM engine and grid the planner picks -- finds the launches that leave CUs idle.

    python tools/frame_shapes.py [--dbg FLAGS] [--top N]
"""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ml-depth-pro-video_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dbg", type=int, default=0, help="dp_gemm_debug_flags (32 = no small-grid stream-K)")
    ap.add_argument("--top", type=int, default=30)
    args = ap.parse_args()
    from depth_pro import _lib, ops
    from depth_pro.depth_pro import _compute_dtype
    from depth_pro.engine import Engine, pack_weights
    from depth_pro.weights import synthetic_state_dict

    _lib.load().dp_gemm_debug_flags(args.dbg)
    dev = torch.device("cuda:0")
    code = _compute_dtype(torch.float32)
    eng = Engine(pack_weights(synthetic_state_dict(0), dev, code), dev, code)
    img = torch.from_numpy(np.random.default_rng(0).integers(0, 256, (1536, 1536, 3), dtype=np.uint8)).to(dev)
    ops.normalize_u8(img, eng.x0)
    eng.serial_side = True
    eng.forward()
    ops.profile_begin()
    eng.forward()
    rec = ops.profile_end()
    groups = {}
    for kind, flops, shape, _dt, ms in rec:
        g = groups.setdefault((kind, shape), [0, 0.0, 0.0])
        g[0] += 1
        g[1] += ms
        g[2] += flops
    total = sum(g[1] for g in groups.values())
    print(f"dbg={args.dbg} eager serial forward: {total:.3f} ms in {len(rec)} launches")
    A = torch.empty(8, dtype=eng.dt, device=dev)
    for (kind, shape), (n, ms, fl) in sorted(groups.items(), key=lambda kv: -kv[1][1])[:args.top]:
        eng_s = ""
        if kind == "gemm" and len(shape) == 3:   # dense plan only (conv plans need the conv geometry)
            M, N, K = shape
            try:
                tile, wgs = ops.gemm(A, A, A, M=M, N=N, K=K, plan_only=True, workspace=eng.ws_main)
                eng_s = f"tile {tile:2d} grid {wgs:5d}"
            except Exception as e:  # noqa: BLE001
                eng_s = f"plan? {e}"
        tf = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        print(f"{kind:12s} {str(shape):24s} x{n:3d} {ms:8.3f} ms {1000 * ms / n:8.1f} us/launch {tf:7.1f} TF  {eng_s}")


if __name__ == "__main__":
    main()
