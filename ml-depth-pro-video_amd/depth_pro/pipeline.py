"""Frame pipeline for video streams: frame i+1's image / FOV encoders beside frame i's decoder.

`DepthPro.infer` runs one frame at a time: its image and FOV encoders (two ViT-L at M = 577
rows, 194 latency-bound launches) run on side streams beside the same frame's patch encoder,
whose one-round GEMMs (proj / fc2: 256 workgroups on 256 CUs) then wait for the CUs they hold.
For a stream of frames (BASELINE config 3, `generate_depth_maps.py`) the frames are
independent, so `FramePipeline` keeps two engines (activations double-buffered, the packed
weights shared) and runs each frame in three captured phases (`Engine.forward(phase)`):

    main stream:  ... | enc(i) | dec(i) | enc(i+1) | dec(i+1) | ...
    side stream:      side(i+1) ........| side(i+2) .........

`side(j)` (window im2col + image encoder + FOV encoder of frame j) starts when `enc(j-1)` ends
and runs beside `dec(j-1)` (the decoder's small-grid phases leave CUs idle); `enc(j)` waits for
`side(j)`.  Every frame goes through the same kernels in the same order as `Engine.run`, so its
outputs are bit-identical to the single-frame path (tests/test_gpu_model.py).

Measured and NOT the default (round 2, `bench.py --pipeline 1`, profiles/r02z_pipeline/):
30.1 vs 23.1 ms per frame.  With the process's 4 hardware queues (GPU_MAX_HW_QUEUES, HIP's
default) the side phase ran alone between the phases (kernel trace: no overlap at all, the two
side encoders serialised too); with 8 / 16 queues the phases did overlap and the frame took
42.8 / 45.9 ms: the decoder's stream-K launches, whose workgroups wait for each other, then
share the CUs with the side encoders' 1-workgroup-per-CU GEMMs.
"""

from __future__ import annotations

from typing import Callable, List, Optional

import torch

from . import ops
from ._lib import DPError
from .engine import Engine


class FramePipeline:
    """Two `Engine`s over one set of packed weights, driven as a two-frame pipeline."""

    def __init__(self, packed, device: torch.device, dtype_code, use_fov: bool = True, graph: bool = True):
        self.dev = device
        self.E = [Engine(packed, device, dtype_code, use_fov=use_fov) for _ in range(2)]
        self.S = torch.cuda.Stream(device=device)       # side phases
        self.graph = graph
        self.G: List[Optional[dict]] = [None, None]
        self.side_done: List[Optional[torch.cuda.Event]] = [None, None]
        self.primed = False
        self.i = 0
        if graph:
            self.capture()

    def capture(self) -> None:
        """Capture side / enc / dec of both engines (one eager warm-up forward each first)."""
        for k, e in enumerate(self.E):
            s = torch.cuda.Stream(device=self.dev)
            s.wait_stream(torch.cuda.current_stream(self.dev))
            with torch.cuda.stream(s):
                e.forward()
            torch.cuda.current_stream(self.dev).wait_stream(s)
            gs = {}
            for ph in ("side", "enc", "dec"):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    e.forward(ph)
                gs[ph] = g
            self.G[k] = gs
        torch.cuda.synchronize(self.dev)

    def _phase(self, k: int, ph: str) -> None:
        if self.graph:
            self.G[k][ph].replay()
        else:
            self.E[k].forward(ph)

    def _side(self, k: int, load: Callable[[torch.Tensor], None]) -> None:
        """On the side stream: `load` fills engine k's x0 with the next frame, then side(k)."""
        with torch.cuda.stream(self.S):
            load(self.E[k].x0)
            self._phase(k, "side")
            ev = torch.cuda.Event()
            ev.record(self.S)
        self.side_done[k] = ev

    def step(self, load_this: Callable[[torch.Tensor], None], load_next: Optional[Callable[[torch.Tensor], None]]):
        """Frame i = this step's frame: `load_this(x0)` is used only on the first step (later frames
        were loaded by the previous step's `load_next`).  Enqueues enc(i), side(i+1) (if
        `load_next`), dec(i) on the current stream / the side stream and returns engine i's
        (canonical, fov_deg) buffers, valid on the current stream (until step i+2)."""
        main = torch.cuda.current_stream(self.dev)
        k = self.i & 1
        if not self.primed:
            main_ev = torch.cuda.Event()
            main_ev.record(main)
            self.S.wait_event(main_ev)
            self._side(k, load_this)
            self.primed = True
        e = self.E[k]
        e.check_status(block=False)
        main.wait_event(self.side_done[k])
        self._phase(k, "enc")
        if load_next is not None:
            ev = torch.cuda.Event()
            ev.record(main)                  # engine k^1's previous frame is done with its buffers
            self.S.wait_event(ev)
            self._side(k ^ 1, load_next)
        self._phase(k, "dec")
        e._stage_status()
        self.i += 1
        if load_next is None:
            self.primed = False              # the stream ended: the next step primes again
        return e.canonical, e.fov_deg

    def run(self, frames: List[Callable[[torch.Tensor], None]]):
        """Generator over a list of loaders (each fills an x0): yields (canonical, fov) per frame
        (the buffers are valid until two more frames have been yielded)."""
        n = len(frames)
        for j in range(n):
            yield self.step(frames[j], frames[j + 1] if j + 1 < n else None)

    def check_status(self) -> None:
        for e in self.E:
            e.check_status(block=True)


def u8_loader(img_u8: torch.Tensor) -> Callable[[torch.Tensor], None]:
    """Loader for a resident uint8 HxWx3 1536^2 frame: the `transform` (dp_normalize_u8) into x0."""
    if img_u8.shape[:2] != (1536, 1536):
        raise DPError("FramePipeline frames must be 1536 x 1536 (resize first, as DepthPro.infer does)")
    return lambda x0: ops.normalize_u8(img_u8, x0)
