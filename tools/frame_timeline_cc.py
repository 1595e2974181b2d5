#!/usr/bin/env python3
"""Launch timeline of one eager forward in the product's concurrent stream layout (HIP events on
the launching stream around every launch, start / end relative to the frame start), from the
patch encoder's last fc2 on: which stream runs what when, and how long only one stream is busy.

    python tools/frame_timeline_cc.py [--all]
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
    ap.add_argument("--all", action="store_true", help="the whole frame, not only the post-encoder part")
    args = ap.parse_args()
    from depth_pro import ops
    from depth_pro.depth_pro import _compute_dtype
    from depth_pro.engine import Engine, pack_weights
    from depth_pro.weights import synthetic_state_dict

    dev = torch.device("cuda:0")
    code = _compute_dtype(torch.float32)
    eng = Engine(pack_weights(synthetic_state_dict(0), dev, code), dev, code)
    img = torch.from_numpy(np.random.default_rng(0).integers(0, 256, (1536, 1536, 3), dtype=np.uint8)).to(dev)
    ops.normalize_u8(img, eng.x0)
    for _ in range(2):
        eng.forward()
    names = {torch.cuda.current_stream(dev).cuda_stream: "main"}
    for n in ("side", "dec_a", "dec_b", "dec_c"):
        names[getattr(eng, n).cuda_stream] = n
    ops.profile_begin()
    eng.forward()
    rec = ops.profile_end(timeline=True)
    frame_end = max(r[5] for r in rec)
    last = max(i for i, r in enumerate(rec) if r[2] == (20195, 1024, 4096))
    t_enc = rec[last][5]
    sel = rec if args.all else [r for r in rec if r[5] > t_enc - 1e-6][0:]
    sel = sorted(sel, key=lambda r: r[4])
    print(f"frame (eager, concurrent) {frame_end:.3f} ms; patch encoder ends at {t_enc:.3f} ms")
    for (k, fl, sh, dt, t0, t1, st) in sel:
        tf = fl / ((t1 - t0) * 1e-3) / 1e12 if t1 > t0 else 0.0
        print(f"{names.get(st, '?'):6s} {t0:8.3f} {t1:8.3f} {1000 * (t1 - t0):8.1f} us {tf:7.1f} TF  {k:12s} {sh}")
    # occupancy of the post-encoder part by number of busy streams
    t0s = sorted({r[4] for r in sel} | {r[5] for r in sel})
    busy = {}
    for a, b in zip(t0s, t0s[1:]):
        n = len({r[6] for r in sel if r[4] <= a and r[5] >= b})
        busy[n] = busy.get(n, 0.0) + (b - a)
    print("time by number of busy streams (ms):", {k: round(v, 3) for k, v in sorted(busy.items())})


if __name__ == "__main__":
    main()
