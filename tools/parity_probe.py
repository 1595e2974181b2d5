#!/usr/bin/env python3
"""Replay-order parity probe: frame-0 depth parity after capture, eager, and after many replays
of other frames (the bench's order).  python tools/parity_probe.py  (env: DP_SIDE_MODE, ...)"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ml-depth-pro-video_amd"))
sys.path.insert(0, REPO)


def main():
    import bench
    from depth_pro import ops
    from depth_pro.depth_pro import _compute_dtype
    from depth_pro.engine import Engine, pack_weights
    from depth_pro.weights import synthetic_state_dict

    dev = torch.device("cuda:0")
    code = _compute_dtype(torch.float32)
    eng = Engine(pack_weights(synthetic_state_dict(0), dev, code), dev, code)
    frames = [torch.from_numpy(bench.frame(k)).to(dev) for k in range(4)]
    depth = torch.empty(1536, 1536, device=dev)
    fpx = torch.empty((), device=dev)

    def par(tag, graph):
        ops.normalize_u8(frames[0], eng.x0)
        c, fov = eng.run() if graph else eng.forward()
        ops.infer_epilogue(c, fov, None, 1536, 1536, depth, fpx)
        torch.cuda.synchronize()
        print(tag, bench.depth_parity(depth, c, fov)["depth_rel_l1"], flush=True)

    par("eager-first", False)
    eng.capture_graph()
    par("graph-after-capture", True)
    for i in range(20):
        ops.normalize_u8(frames[i % 4], eng.x0)
        eng.run()
    par("graph-after-20-replays", True)
    eng.serial_side = True
    par("eager-serial_side", False)
    eng.serial_side = False
    par("graph-after-eager", True)

    names = ("cols", "g", "cat", "enc4", "low", "feats", "f0", "f1", "f2", "lat0", "lat1", "fov_tok")

    def snap():
        d = {n: getattr(eng, n).clone() for n in names}
        d["vi.out"] = eng.vi.out.clone()
        d["vi.x"] = eng.vi.x.clone()
        d["vp.out"] = eng.vp.out.clone()
        return d

    for i in range(5):
        ops.normalize_u8(frames[(i % 3) + 1], eng.x0)
        eng.run()
    ops.normalize_u8(frames[0], eng.x0)
    eng.run()
    torch.cuda.synchronize()
    a = snap()
    ops.normalize_u8(frames[0], eng.x0)
    eng.forward()
    torch.cuda.synchronize()
    b = snap()
    for n in a:
        d = (a[n].float() - b[n].float()).abs().max().item()
        print(f"graph vs eager {n:8s} max|d| {d:.3e}", flush=True)


if __name__ == "__main__":
    main()
