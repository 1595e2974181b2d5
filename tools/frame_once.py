#!/usr/bin/env python3
"""Run the eager (non-graph) forward on synthetic frame 0 a few times — target for rocprofv3 --pmc passes.

Each launch is its own dispatch, so per-kernel PMC rows (FETCH_SIZE, WRITE_SIZE, SQ_*)
map one-to-one onto the frame's kernels.  The last `--frames` forwards are the ones to read.
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
    ap.add_argument("--frames", type=int, default=2)
    ap.add_argument("--serial", action="store_true",
                    help="every launch on one stream (Engine.serial_side): each launch alone on the chip -- "
                         "the frames tools/frame_budget.py sums and takes per-kernel alone times from")
    args = ap.parse_args()
    from depth_pro import ops
    from depth_pro.depth_pro import _compute_dtype
    from depth_pro.engine import Engine, pack_weights
    from depth_pro.weights import synthetic_state_dict

    dev = torch.device("cuda:0")
    code = _compute_dtype(torch.float32)
    eng = Engine(pack_weights(synthetic_state_dict(0), dev, code), dev, code)
    img = torch.from_numpy(np.random.default_rng(0).integers(0, 256, (1536, 1536, 3), dtype=np.uint8)).to(dev)
    eng.serial_side = args.serial
    for _ in range(args.frames):
        ops.normalize_u8(img, eng.x0)
        eng.forward()
    torch.cuda.synchronize()
    print("frames done", args.frames)


if __name__ == "__main__":
    main()
