"""Step-by-step run of the engine under the current env (schedule knobs), printing each stage:
eager forward, graph capture, replays.  For locating a host-side crash (run with -X faulthandler)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ml-depth-pro-video_amd"))
from depth_pro.depth_pro import DepthPro, Transform, _compute_dtype  # noqa: E402
from depth_pro.engine import pack_weights  # noqa: E402
from depth_pro.weights import synthetic_state_dict  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    code = _compute_dtype(torch.float32)
    packed = pack_weights(synthetic_state_dict(0), dev, code)
    model = DepthPro.from_packed(packed, dev, code)
    eng = model.engine()
    eng.forward()
    torch.cuda.synchronize()
    print("eager ok", flush=True)
    eng.capture_graph()
    torch.cuda.synchronize()
    print("captured", flush=True)
    for _ in range(3):
        eng.run()
    torch.cuda.synchronize()
    print("replay ok", flush=True)
    transform = Transform(dev, torch.float32)
    img = torch.randint(0, 256, (1536, 1536, 3), dtype=torch.uint8, device=dev)
    for _ in range(5):
        with torch.no_grad():
            model.infer(transform(img))
    torch.cuda.synchronize()
    print("infer ok", model.last_status().error(), flush=True)


if __name__ == "__main__":
    main()
