#!/usr/bin/env python3
"""Where one eager forward's time goes, in the graph's stream layout (side encoders and decoder
chains concurrent): per-launch start / end on every stream (HIP events on the launching stream,
one device clock), the main stream's busy time vs idle gaps, and the top launches per phase.

    python tools/frame_streams.py [--top 25]
"""
import argparse
import os
import sys
from collections import defaultdict

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ml-depth-pro-video_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=25)
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
    for _ in range(3):
        eng.forward()
    torch.cuda.synchronize()
    main_id = torch.cuda.current_stream().cuda_stream
    ops.profile_begin()
    eng.forward()
    rec = ops.profile_end(timeline=True)
    names = {main_id: "main", eng.side.cuda_stream: "side", eng.dec_a.cuda_stream: "dec_a",
             eng.dec_b.cuda_stream: "dec_b", eng.dec_c.cuda_stream: "dec_c"}
    end = max(r[5] for r in rec)
    print(f"frame (eager, concurrent streams): {end:.3f} ms, {len(rec)} timed launches")
    per = defaultdict(list)
    for r in rec:
        per[names.get(r[6], str(r[6]))].append(r)
    for st, rs in per.items():
        busy = sum(r[5] - r[4] for r in rs)
        print(f"  stream {st:6s}: {len(rs):4d} launches, busy {busy:.3f} ms")
    mains = sorted(per["main"], key=lambda r: r[4])
    gaps, t = [], 0.0
    for r in mains:
        if r[4] > t + 1e-4:
            gaps.append((r[4] - t, t, r[0], r[2]))
        t = max(t, r[5])
    print(f"  main stream idle between its launches: {sum(g[0] for g in gaps):.3f} ms in {len(gaps)} gaps; largest:")
    for g in sorted(gaps, reverse=True)[:10]:
        print(f"    {1000 * g[0]:8.1f} us at {g[1]:7.3f} ms before {g[2]} {g[3]}")
    # per (kind, shape) on main: total and average
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for r in mains:
        a = agg[(r[0], r[2])]
        a[0] += 1
        a[1] += r[5] - r[4]
        a[2] += r[1]
    print("  main stream by launch group (kind, shape): n, total ms, avg us, TFLOP/s")
    for (k, sh), (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:args.top]:
        print(f"    {k:12s} {str(sh):26s} {n:4d} {ms:8.3f} {1000 * ms / n:8.1f} {fl / (ms * 1e-3) / 1e12 if ms else 0:8.1f}")


if __name__ == "__main__":
    main()
