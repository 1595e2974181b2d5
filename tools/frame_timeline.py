#!/usr/bin/env python3
"""Ordered launch timeline of one eager forward (side encoders serialised) from the first
launch after the patch encoder: which post-encoder launches leave the chip idle.

    python tools/frame_timeline.py [--dbg FLAGS]
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
    ap.add_argument("--dbg", type=int, default=0)
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
    # the patch encoder's last fc2 (M = 20195, N = 1024, K = 4096) ends the encoder part
    last = max(i for i, r in enumerate(rec) if r[2] == (20195, 1024, 4096))
    tot = sum(r[4] for r in rec)
    post = rec[last + 1:]
    print(f"eager serial forward {tot:.3f} ms; after the patch encoder: {sum(r[4] for r in post):.3f} ms "
          f"in {len(post)} timed launches")
    A = torch.empty(8, dtype=eng.dt, device=dev)
    for i, (kind, fl, shape, _dt, ms) in enumerate(post):
        eng_s = ""
        if kind == "gemm" and len(shape) == 3:
            try:
                tile, wgs = ops.gemm(A, A, A, M=shape[0], N=shape[1], K=shape[2], plan_only=True, workspace=eng.ws_main)
                eng_s = f"tile {tile:2d} grid {wgs:5d}"
            except Exception:  # noqa: BLE001
                pass
        tf = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        print(f"{i:3d} {kind:12s} {str(shape):26s} {1000 * ms:8.1f} us {tf:7.1f} TF  {eng_s}")


if __name__ == "__main__":
    main()
