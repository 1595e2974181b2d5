"""The generate_depth_maps drop-in: writers pinned to the reference colorize_depth (CPU),
and the pipelined directory loop on the GPU."""

import os
import time

import numpy as np
import pytest

os.environ.setdefault("DEPTH_PRO_SYNTHETIC", "1")  # no checkpoint offline: synthetic weights

import generate_depth_maps as G  # noqa: E402


def test_colorize_matches_reference(golden_dir):
    g = np.load(f"{golden_dir}/golden_frameloop.npz")
    for cmap in ("turbo", "viridis", "jet"):
        assert np.array_equal(G.colorize_depth(g["depth"], cmap=cmap), g[f"color_{cmap}"]), cmap
    d = np.nan_to_num(g["depth"], nan=1.0)
    assert np.array_equal(G.raw_depth_u16(d), g["raw_u16"])


def test_png_writers_roundtrip(tmp_path):
    from PIL import Image

    rgb = (np.arange(48 * 64 * 3) % 251).astype(np.uint8).reshape(48, 64, 3)
    G._write_png(str(tmp_path / "c.png"), rgb)
    assert np.array_equal(np.asarray(Image.open(tmp_path / "c.png")), rgb)
    u16 = (np.arange(48 * 64) * 20).astype(np.uint16).reshape(48, 64)
    G._write_png(str(tmp_path / "r.png"), u16)
    assert np.array_equal(np.asarray(Image.open(tmp_path / "r.png")).astype(np.uint16), u16)


@pytest.mark.gpu
def test_batch_loop_on_gpu(tmp_path, cuda):
    from PIL import Image

    import torch

    src = tmp_path / "frames"
    src.mkdir()
    rng = np.random.default_rng(0)
    for k in range(3):
        Image.fromarray(rng.integers(0, 256, (360, 640, 3), dtype=np.uint8)).save(src / f"output_{k:04d}.png")
    out = tmp_path / "depth"
    n = G.batch_generate_depth_maps(str(src), str(out), pattern="output_*.png")
    assert n == 3
    files = sorted(os.listdir(out))
    assert files == [f"output_{k:04d}_depth.png" for k in range(3)]
    img = np.asarray(Image.open(out / files[0]))
    assert img.shape == (360, 640, 3) and img.dtype == np.uint8
    # the colored PNG is exactly colorize_depth(model.infer(...)) of the same frame
    model, transform = G._model(cuda, False)
    frame = np.asarray(Image.open(src / "output_0000.png"))
    with torch.no_grad():
        depth = model.infer(transform(frame))["depth"].cpu().numpy()
    assert np.array_equal(img, G.colorize_depth(depth))
    n_raw = G.batch_generate_depth_maps(str(src), str(tmp_path / "raw"), pattern="output_*.png", colored=False)
    assert n_raw == 3
    raw = np.asarray(Image.open(tmp_path / "raw" / "output_0001_depth.png"))
    assert raw.shape == (360, 640)


@pytest.mark.gpu
def test_batch_loop_pointcloud_on_gpu(tmp_path, cuda):
    """--pointcloud: one PLY per frame == depth_to_3d(infer depth, infer f_px) with the frame's colours."""
    from PIL import Image

    import torch

    from depth_pro import pointcloud as PC
    from oracle import depth_pro_oracle as O

    src = tmp_path / "frames"
    src.mkdir()
    img = np.random.default_rng(5).integers(0, 256, (270, 480, 3), dtype=np.uint8)
    Image.fromarray(img).save(src / "output_0000.png")
    out = tmp_path / "pc"
    assert G.batch_generate_depth_maps(str(src), str(out), pattern="output_*.png", pointcloud=True) == 1
    pts, cols = PC.read_ply(str(out / "output_0000_points.ply"))
    model, transform = G._model(cuda, False)
    with torch.no_grad():
        pred = model.infer(transform(img))
    depth = pred["depth"].cpu().numpy()
    ref, valid = O.depth_to_3d(depth, float(pred["focallength_px"]), 480, 270)
    assert np.array_equal(pts, ref)
    assert np.array_equal(cols, img[valid])


def test_bad_frame_dropped_once_by_its_writer(tmp_path):
    """a bad frame whose status is already final when the NEXT frame is submitted (the
    GPU finished it before its writer thread looked at it) is reported by its own writer only.
    The loop claims each frame's status (BatchStatus.claim), so the next infer's non-blocking sweep
    of finished frames (DepthPro._check_earlier -> Engine.check_status(block=False)) skips it:
    frames 0 and 2 are written, frame 1 is dropped, and no frame is dropped in its place.  The
    engine's sweep is the real one (Engine._sweep / check_status); the forward is a CPU stub whose
    frames are finished at once."""
    import threading

    import torch
    from PIL import Image

    from depth_pro.engine import BatchStatus, Engine, FrameStatus

    class Done:   # a frame event that has completed; its writer thread is slow to look at it
        def __init__(self, delay):
            self.delay = delay

        def query(self):
            return True

        def synchronize(self):
            if threading.current_thread() is not threading.main_thread():
                time.sleep(self.delay)

    class Model:
        def __init__(self):
            self.eng = Engine.__new__(Engine)
            self.eng._recent, self.eng._unreported = [], []
            self.n, self.last = 0, None

        def infer(self, x, f_px=None):
            self.eng.check_status(block=False)          # as DepthPro.infer before each call
            words = torch.tensor([0, 7 if self.n == 1 else 0], dtype=torch.int32)
            st = FrameStatus(self.n, words, Done(0.5 if self.n == 1 else 0.0))
            self.eng._recent.append(st)
            self.last = BatchStatus([st])
            self.n += 1
            return {"depth": torch.full(x.shape[:2], 2.0), "focallength_px": torch.tensor(1000.0)}

        def last_status(self):
            return self.last

    src = tmp_path / "frames"
    src.mkdir()
    for k in range(3):
        Image.fromarray(np.full((24, 32, 3), 40 * k, np.uint8)).save(src / f"output_{k:04d}.png")
    model = Model()
    n = G.batch_generate_depth_maps(str(src), str(tmp_path / "out"), pattern="output_*.png",
                                    model=(model, lambda im: torch.as_tensor(np.asarray(im))), decode_workers=1,
                                    encode_workers=1)
    assert n == 2
    assert sorted(os.listdir(tmp_path / "out")) == ["output_0000_depth.png", "output_0002_depth.png"]
    assert model.n == 3
    model.eng.check_status(block=True)                  # nothing owed: frame 1 was reported once
