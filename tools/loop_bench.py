#!/usr/bin/env python3
"""Throughput of the drop-in video loop (generate_depth_maps.batch_generate_depth_maps) as a user
runs it: PNG frames on disk -> decode -> GPU (one HIP graph per frame) -> PNG (+ PLY) on disk.
BASELINE configs 3 (1536^2 stream) and 5 (4K frames with the FOV head and --pointcloud), 1 GPU.

    python tools/loop_bench.py --frames 64 --size 1536x1536
    python tools/loop_bench.py --frames 16 --size 3840x2160 --pointcloud

Frames are synthetic (uniform random RGB, as bench.py: the worst case for PNG decode / encode);
weights synthetic.  Reports end-to-end frames/s of the loop and each stage alone on the same host
(decode in the loop's pool, GPU infer on resident frames, PNG encode of the GPU-made image,
PLY write), one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ml-depth-pro-video_amd"))
os.environ.setdefault("DEPTH_PRO_SYNTHETIC", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--size", default="1536x1536", help="WxH of the input frames")
    ap.add_argument("--pointcloud", action="store_true")
    ap.add_argument("--raw", action="store_true")
    ap.add_argument("--workers", type=int, default=None,
                    help="decode and encode threads each (default: the loop's own defaults)")
    ap.add_argument("--dir", default=None, help="scratch directory (default: a temp dir, removed)")
    ap.add_argument("--ply-copy", action="store_true",
                    help="A/B: the round-4 PLY writer (body copied to bytes with the GIL held before the write)")
    args = ap.parse_args()
    W, H = (int(v) for v in args.size.split("x"))

    from PIL import Image

    import depth_pro
    import generate_depth_maps as G
    from depth_pro import pointcloud as PC

    if args.ply_copy:
        def write_ply_copy(path, points, colors=None):
            pts = np.ascontiguousarray(np.asarray(points, dtype="<f8").reshape(-1, 3))
            rec = np.empty(pts.shape[0], dtype=[("p", "<f8", 3), ("c", "u1", 3)])
            rec["p"], rec["c"] = pts, colors
            hdr = ("ply\nformat binary_little_endian 1.0\nelement vertex %d\nproperty double x\nproperty double y\n"
                   "property double z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n"
                   % pts.shape[0])
            with open(path, "wb") as f:
                f.write(hdr.encode("ascii"))
                f.write(rec.tobytes())
            return path
        PC.write_ply = write_ply_copy

    root = args.dir or tempfile.mkdtemp(prefix="loop_bench_")
    src, dst = os.path.join(root, "frames"), os.path.join(root, "out")
    os.makedirs(src, exist_ok=True)
    t = time.time()
    rng = np.random.default_rng(0)
    for k in range(args.frames):
        Image.fromarray(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).save(
            os.path.join(src, f"output_{k:04d}.png"), compress_level=1)
    t_gen = time.time() - t

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t = time.time()
    model = G._model(dev, False)
    m, transform = model
    torch.cuda.synchronize()
    t_setup = time.time() - t
    kw = dict(colored=not args.raw, pointcloud=args.pointcloud, model=model)
    if args.workers:
        kw.update(decode_workers=args.workers, encode_workers=args.workers)
    import inspect
    dflt = inspect.signature(G.batch_generate_depth_maps).parameters
    n_dec = kw.get("decode_workers", dflt["decode_workers"].default)
    n_enc = kw.get("encode_workers") or max(4, min(8, len(os.sched_getaffinity(0)) // 2))
    # warm-up pass over 2 frames (first launches, allocator, thread pools), then the timed loop
    warm = os.path.join(root, "warm")
    os.makedirs(warm, exist_ok=True)
    for k in range(2):
        shutil.copy(os.path.join(src, f"output_{k:04d}.png"), warm)
    G.batch_generate_depth_maps(warm, os.path.join(root, "warm_out"), **kw)
    torch.cuda.synchronize()
    t = time.time()
    n_ok = G.batch_generate_depth_maps(src, dst, **kw)
    torch.cuda.synchronize()
    t_loop = time.time() - t

    paths = sorted(os.path.join(src, f) for f in os.listdir(src))
    # stage: decode alone (the loop's decoder: depth_pro.load_rgb in a pool)
    t = time.time()
    with ThreadPoolExecutor(n_dec) as ex:
        imgs = list(ex.map(lambda p: G._load(p, 1.0)[0], paths))
    t_dec = time.time() - t
    # stage: GPU alone (transform + infer on host frames already decoded; includes the u8 upload)
    n_gpu = min(len(imgs), 16)
    for img in imgs[:2]:
        with torch.no_grad():
            m.infer(transform(img))
    torch.cuda.synchronize()
    t = time.time()
    depths = []
    for img in imgs[:n_gpu]:
        with torch.no_grad():
            depths.append(m.infer(transform(img))["depth"])
    torch.cuda.synchronize()
    t_gpu = (time.time() - t) / n_gpu
    # stage: image content on the GPU + PNG encode in the writer pool
    hosts = [G._image_async(d, not args.raw, "turbo") for d in depths]
    torch.cuda.synchronize()
    t = time.time()
    with ThreadPoolExecutor(n_enc) as ex:
        list(ex.map(lambda ih: G._write_png(os.path.join(root, f"enc_{ih[0]}.png"), G._host_image(ih[1])),
                    enumerate(hosts)))
    t_enc = (time.time() - t) / len(hosts)
    t_ply = None
    if args.pointcloud:
        img_dev = (imgs[0] if torch.is_tensor(imgs[0]) else torch.from_numpy(imgs[0])).to(dev)
        f = m.infer(transform(imgs[0]))["focallength_px"]
        xyz, _, cols, count = PC.depth_to_points_async(depths[0], f, W, H, rgb=img_dev)
        torch.cuda.synchronize()
        n = int(count)
        a, c = xyz[:n].cpu().numpy(), cols[:n].cpu().numpy()
        t = time.time()
        PC.write_ply(os.path.join(root, "one.ply"), a, c)
        t_ply = time.time() - t
    out = {
        "what": "generate_depth_maps.batch_generate_depth_maps end to end, 1 GPU",
        "frames": args.frames, "size": [W, H], "pointcloud": args.pointcloud, "raw": args.raw,
        "ply_writer": "bytes copy" if args.ply_copy else "zero-copy",
        "decode_workers": n_dec, "encode_workers": n_enc, "frames_ok": n_ok,
        "loop_fps": round(args.frames / t_loop, 2),
        "stage_fps": {"decode_png_pool": round(len(paths) / t_dec, 2),
                      "gpu_infer_incl_upload": round(1.0 / t_gpu, 2),
                      "encode_png_pool": round(1.0 / t_enc, 2) if t_enc else None},
        "stage_ms_per_frame": {"decode_png_pool": round(1000 * t_dec / len(paths), 2),
                               "gpu_infer_incl_upload": round(1000 * t_gpu, 2),
                               "encode_png_pool": round(1000 * t_enc, 2),
                               "ply_write_1_thread": round(1000 * t_ply, 1) if t_ply else None},
        "host_cpus": len(os.sched_getaffinity(0)), "setup_s": round(t_setup, 1), "gen_s": round(t_gen, 1),
        "data": "synthetic uniform-random RGB PNG frames (compress_level=1), synthetic weights",
    }
    print(json.dumps(out), flush=True)
    if args.dir is None:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
