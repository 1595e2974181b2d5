"""BASELINE configs 4 and 5 on the GPU, end to end through the code paths they run.

* Config 5 (`generate_depth_maps.py` at 4K with the focal-length head and the point-cloud
  write-out, reference generate_depth_maps.py:153-206 + img_to_normalized_pointcloud.py:819-856):
  two 3840x2160 PNG frames through `batch_generate_depth_maps(..., pointcloud=True)`, checked
  against the reference's own 4K `infer` (golden_infer_4k.npz) and the reference's depth_to_3d.
* Config 4's non-root rank (one process per GPU under torchrun): rank 1 builds its model from
  rank 0's packed weights (`create_model_and_transforms_shared` -> `broadcast_packed` ->
  `DepthPro.from_packed`), which must compute bit for bit what rank 0's locally packed model
  computes (reference counterpart: the checkpoint load, depth_pro.py:134-149).
* Frame-failure attribution in the frame loop: a frame whose forward fails (fault injection) is
  reported and NOT written; its neighbours are written.
"""

import os
import socket

import numpy as np
import pytest
import torch

os.environ.setdefault("DEPTH_PRO_SYNTHETIC", "1")  # no checkpoint offline: synthetic weights

pytestmark = pytest.mark.gpu


def frame(seed, h=1536, w=1536):
    return np.random.default_rng(seed=seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def rel_l1(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).mean() / np.abs(b).mean())


def test_config5_frame_loop_4k_pointcloud(tmp_path, cuda, golden_dir, record):
    """Two 3840x2160 frames through the drop-in loop with --raw and --pointcloud:
    depth (read back from the PLY's z, every pixel valid) vs the reference's 4K infer at
    rel-L1 < 1e-3; the PLY equals depth_to_3d(loop depth, loop f_px) bit for bit with the
    frame's colours; the --raw PNG is exactly the reference's uint16 encoding of that depth."""
    from PIL import Image

    import generate_depth_maps as G
    from depth_pro import pointcloud as PC
    from oracle import depth_pro_oracle as O

    g = np.load(f"{golden_dir}/golden_infer_4k.npz")
    H, W, seed = int(g["H"]), int(g["W"]), int(g["frame_seed"])
    src = tmp_path / "frames"
    src.mkdir()
    imgs = {0: frame(seed, H, W), 1: frame(seed + 1, H, W)}
    for k, img in imgs.items():
        Image.fromarray(img).save(src / f"output_{k:04d}.png")
    out = tmp_path / "out"
    n = G.batch_generate_depth_maps(str(src), str(out), pattern="output_*.png", colored=False, pointcloud=True)
    assert n == 2
    model, transform = G._model(cuda, False)
    for k, img in imgs.items():
        pts, cols = PC.read_ply(str(out / f"output_{k:04d}_points.ply"))
        assert pts.shape == (H * W, 3)                          # every depth finite and > 0
        depth = pts[:, 2].reshape(H, W).astype(np.float32)      # z = depth, row-major pixel order
        with torch.no_grad():
            pred = model.infer(transform(img))
        d_ref = pred["depth"].cpu().numpy()
        assert np.array_equal(depth, d_ref)                     # the loop's depth is the engine's
        ref, valid = O.depth_to_3d(depth, float(pred["focallength_px"]), W, H)
        assert np.array_equal(pts, ref) and np.array_equal(cols, img[valid])
        raw = np.asarray(Image.open(out / f"output_{k:04d}_depth.png")).astype(np.uint16)
        assert np.array_equal(raw, G.raw_depth_u16(depth))
        if k == 0:
            e_d = rel_l1(depth[::16, ::16], g["depth_sub16"])
            e_f = abs(float(pred["focallength_px"]) - float(g["f_px"])) / float(g["f_px"])
            print(f"\nconfig 5 loop, 4K frame {seed}: depth rel-L1 {e_d:.3e}, f_px rel {e_f:.2e}")
            record("config5_loop_4k_depth_rel_l1", e_d)
            record("config5_loop_4k_fpx_rel", e_f)
            assert e_d < 1e-3 and e_f < 1e-3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_worker(rank, world, port, outdir):
    """One rank of config 4 on cuda:0 (gloo carries the broadcast: two ranks cannot share a GPU
    under RCCL)."""
    import torch.distributed as dist

    import depth_pro
    from depth_pro import distributed as D

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DEPTH_PRO_SYNTHETIC="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        cfg = depth_pro.depth_pro.run_config()
        model, transform = D.create_model_and_transforms_shared(cfg, torch.device("cuda"), torch.float32)
        model.use_hip_graph(True)
        with torch.no_grad():
            pred = model.infer(transform(frame(0)))
        model.last_status().check()
        np.save(os.path.join(outdir, f"depth{rank}.npy"), pred["depth"].cpu().numpy())
        np.save(os.path.join(outdir, f"fpx{rank}.npy"), pred["focallength_px"].cpu().numpy())
        with open(os.path.join(outdir, f"kind{rank}.txt"), "w") as f:
            f.write("from_packed" if model._packed_device is not None else "local")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_config4_nonroot_rank_builds_from_broadcast(tmp_path, golden_dir, record):
    """Rank 1's model comes from rank 0's broadcast packed weights (DepthPro.from_packed, device
    given as a bare 'cuda') and computes frame 0 bit for bit like rank 0's locally packed model;
    both match the reference's frame-0 forward within the parity target."""
    import torch.multiprocessing as mp

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(600)
        assert p.exitcode == 0
    assert (tmp_path / "kind0.txt").read_text() == "local"
    assert (tmp_path / "kind1.txt").read_text() == "from_packed"
    d0, d1 = np.load(tmp_path / "depth0.npy"), np.load(tmp_path / "depth1.npy")
    assert np.array_equal(d0, d1)
    assert np.array_equal(np.load(tmp_path / "fpx0.npy"), np.load(tmp_path / "fpx1.npy"))
    g = np.load(f"{golden_dir}/golden_forward_frame0.npz")
    W = 1536.0
    f_ref = 0.5 * W / np.tan(0.5 * np.deg2rad(float(g["fov_deg"][0])))
    d_ref = 1.0 / np.clip(g["canonical_sub8"].astype(np.float64) * (W / f_ref), 1e-4, 1e4)
    e = rel_l1(d1[::8, ::8], d_ref)
    print(f"\nconfig 4 rank 1 (from_packed) frame 0 depth rel-L1 {e:.3e}")
    record("config4_rank1_depth_rel_l1", e)
    assert e < 1e-3


def _nccl_worker(port, outdir):
    """World-1 process group over the nccl backend (RCCL) on cuda:0: every collective the frame-
    parallel paths use runs through RCCL once (bench.py, distributed.py, generate_depth_maps)."""
    import torch.distributed as dist

    import depth_pro
    from depth_pro import distributed as D
    from depth_pro.depth_pro import DepthPro

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DEPTH_PRO_SYNTHETIC="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    res = {}
    try:
        assert dist.get_backend() == "nccl"
        cfg = depth_pro.depth_pro.run_config()
        # create_model_and_transforms_shared: broadcast_object_list + the one-blob weight broadcast
        model, transform = D.create_model_and_transforms_shared(cfg, torch.device("cuda"), torch.float32)
        # the non-root path: an engine built on the RCCL-broadcast blob (DepthPro.from_packed)
        received = D.broadcast_packed(model.engine().P, dev, src=0)
        other = DepthPro.from_packed(received, dev, model.compute_dtype, use_fov_head=model.use_fov_head)
        x = transform(frame(0))
        with torch.no_grad():
            d_local = model.infer(x)["depth"].clone()
            d_recv = other.infer(x)["depth"].clone()
        model.last_status().check()
        other.last_status().check()
        res["equal"] = bool(torch.equal(d_local, d_recv))
        # the per-step depth gather: gather_frames (async handle) and the raw RCCL gather under it
        bufs, work = D.gather_frames(d_recv, dst=0, async_op=True)
        if work is not None:
            work.wait()
        gl = [torch.empty_like(d_recv)]
        w2 = dist.gather(d_recv, gather_list=gl, dst=0, async_op=True)
        w2.wait()
        torch.cuda.synchronize()
        res["gather_equal"] = bool(torch.equal(bufs[0], d_local) and torch.equal(gl[0], d_local))
        # bench.py's max-over-ranks timing
        t = torch.tensor([1.25], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        res["allreduce"] = float(t.item())
        dist.barrier()
    finally:
        dist.destroy_process_group()
    import json
    with open(os.path.join(outdir, "nccl.json"), "w") as f:
        json.dump(res, f)


def test_config4_collectives_over_rccl(tmp_path):
    """the RCCL (nccl-backend) code of the frame-parallel path executes on
    the GPU box: weight broadcast, engine from the broadcast blob bit-identical to the local one,
    the depth gather and the max-over-ranks all-reduce (world 1: one GPU per box)."""
    import json

    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), str(tmp_path)))
    p.start()
    p.join(600)
    assert p.exitcode == 0
    res = json.loads((tmp_path / "nccl.json").read_text())
    assert res == {"equal": True, "gather_equal": True, "allreduce": 1.25}, res


@pytest.mark.parametrize("sync_after", [False, True])
def test_frame_loop_drops_exactly_the_failed_frame(tmp_path, cuda, sync_after):
    """Fault injection on frame 1 of 3 (a stream-K hand-off that gives up at once): the loop
    reports frame 1, writes nothing for it, and writes frames 0 and 2 (whose own forwards were
    healthy: the failed forward's workspace check cleared the error word and the flags).
    sync_after: the GPU has finished frame 1 before frame 2 is submitted, so frame 2's infer finds
    frame 1's bad status final -- the loop's claim leaves it to frame 1's writer."""
    from PIL import Image

    import depth_pro
    import generate_depth_maps as G
    from depth_pro import _lib

    src = tmp_path / "frames"
    src.mkdir()
    for k in range(3):
        Image.fromarray(frame(30 + k, 270, 480)).save(src / f"output_{k:04d}.png")
    model, transform = depth_pro.create_model_and_transforms(depth_pro.depth_pro.run_config(), device=cuda)
    model.use_hip_graph(False)                  # the injected flag is read per launch
    lib = _lib.load()

    class Faulty:
        def __init__(self, m):
            self.m, self.n = m, 0

        def infer(self, x, f_px=None):
            lib.dp_gemm_debug_flags(64 if self.n == 1 else 0)
            try:
                return self.m.infer(x, f_px=f_px)
            finally:
                lib.dp_gemm_debug_flags(0)
                if sync_after and self.n == 1:
                    torch.cuda.synchronize()
                self.n += 1

        def last_status(self):
            return self.m.last_status()

    out = tmp_path / "out"
    n = G.batch_generate_depth_maps(str(src), str(out), pattern="output_*.png", pointcloud=True,
                                    model=(Faulty(model), transform))
    assert n == 2
    assert sorted(os.listdir(out)) == ["output_0000_depth.png", "output_0000_points.ply",
                                       "output_0002_depth.png", "output_0002_points.ply"]


@pytest.mark.parametrize("factor", [0.5, 0.6, 1.5])
def test_frame_loop_downscale_factor(tmp_path, cuda, factor):
    """--downscale_factor (reference generate_depth_maps.py:95-110): the loop resizes on the GPU
    (dp_resize_u8_cv) exactly as the cv2.resize restatement does (oracle/cv_resize_oracle.py:
    INTER_AREA below 1, INTER_LINEAR above; parity vs a cv2 binary unpinned), and the written PNG
    is the colour map of the model's depth for that resized frame."""
    from PIL import Image

    import generate_depth_maps as G
    from oracle import cv_resize_oracle as CV

    src = tmp_path / "frames"
    src.mkdir()
    img = frame(40, 250, 330)
    Image.fromarray(img).save(src / "output_0000.png")
    out = tmp_path / "out"
    assert G.batch_generate_depth_maps(str(src), str(out), pattern="output_*.png", downscale_factor=factor) == 1
    small = CV.cv2_resize_u8(img, factor)
    model, transform = G._model(cuda, False)
    with torch.no_grad():
        depth = model.infer(transform(small))["depth"].cpu().numpy()
    png = np.asarray(Image.open(out / "output_0000_depth.png"))
    assert png.shape == small.shape
    assert np.array_equal(png, G.colorize_depth(depth))


def test_stressed_weights_mixed_precision_margin(cuda, golden_dir, record):
    """Parity outside the benign synthetic distribution (LayerScale x5 and outlier residual
    channels, depth_pro.weights.stressed_state_dict; reference forward: golden_stress_frame0.npz)
    in the default mixed mode (bf16 ViTs, f16 decoder): every output finite (no f16 overflow in
    the decoder; the frame's FrameStatus is healthy) and the measured error printed and bounded.
    Bound: 1e-3 on depth like the benign set -- if this fails, the f16 decoder is where the margin
    ends."""
    import depth_pro
    from depth_pro.depth_pro import DepthPro, Transform, _compute_dtype
    from depth_pro.weights import stressed_state_dict

    g = np.load(f"{golden_dir}/golden_stress_frame0.npz")
    m = DepthPro(use_fov_head=True, compute_dtype=_compute_dtype(torch.float32))
    m.load_state_dict(stressed_state_dict(0), strict=True)
    m = m.to(cuda).eval()
    t = Transform(cuda, torch.float32)
    with torch.no_grad():
        pred = m.infer(t(frame(0)))
        canonical, fov = m.forward(t(frame(0)).unsqueeze(0))
    m.last_status().check()
    depth = pred["depth"].cpu().numpy()
    assert np.isfinite(depth).all() and np.isfinite(float(pred["focallength_px"]))
    c = canonical[0, 0, ::8, ::8].float().cpu().numpy()
    e_c = rel_l1(c, g["canonical_sub8"])
    W = 1536.0
    f_ref = 0.5 * W / np.tan(0.5 * np.deg2rad(float(g["fov_deg"][0])))
    d_ref = 1.0 / np.clip(g["canonical_sub8"].astype(np.float64) * (W / f_ref), 1e-4, 1e4)
    e_d = rel_l1(depth[::8, ::8], d_ref)
    e_f = abs(fov.item() - float(g["fov_deg"][0])) / abs(float(g["fov_deg"][0]))
    print(f"\nstressed weights (mixed): canonical rel-L1 {e_c:.3e}  depth rel-L1 {e_d:.3e}  fov rel {e_f:.2e}; "
          f"reference residual |max| {g['residual_absmax']}, decoder features |max| {float(g['features_absmax']):.1f}")
    record("stress_mixed_canonical_rel_l1", e_c)
    record("stress_mixed_depth_rel_l1", e_d)
    record("stress_mixed_fov_rel", e_f)
    assert e_d < 1e-3 and e_f < 1e-3
