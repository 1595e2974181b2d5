#!/usr/bin/env python3
"""Per-frame cost of DepthPro.infer around the graph replay: K replays of the captured forward alone
vs K infer() calls (transform + input copy + replay + depth epilogue + status) on resident frames."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ml-depth-pro-video_amd"))
from depth_pro.depth_pro import DepthPro, Transform, _compute_dtype  # noqa: E402
from depth_pro.engine import pack_weights  # noqa: E402
from depth_pro.weights import synthetic_state_dict  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    code = _compute_dtype(torch.float32)
    model = DepthPro.from_packed(pack_weights(synthetic_state_dict(0), dev, code), dev, code)
    eng = model.engine()
    eng.capture_graph()
    transform = Transform(dev, torch.float32)
    frames = [torch.from_numpy(np.random.default_rng(k).integers(0, 256, (1536, 1536, 3), dtype=np.uint8)).to(dev)
              for k in range(4)]
    K = 40

    def timed(fn):
        for i in range(3):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(K):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / K

    for r in range(2):
        t_rep = timed(lambda i: eng.run())
        with torch.no_grad():
            t_inf = timed(lambda i: model.infer(transform(frames[i % 4])))
        print(f"graph replay alone {t_rep:.3f} ms/frame; infer() {t_inf:.3f} ms/frame; difference {t_inf - t_rep:.3f} ms",
              flush=True)


if __name__ == "__main__":
    main()
