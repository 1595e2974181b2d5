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
    ap.add_argument("--trace", action="store_true",
                    help="time where the loop's submitting thread spends the timed run (waits vs work)")
    ap.add_argument("--switch-ms", type=float, default=None,
                    help="A/B: sys.setswitchinterval for the run (the GIL hand-off to the submitting thread)")
    ap.add_argument("--png-copy", action="store_true",
                    help="A/B: the PNG writer that copied the filtered image and the compressed stream "
                         "into new bytes objects (GIL held) before one write")
    ap.add_argument("--ply-host", action="store_true",
                    help="A/B: PLY vertex records interleaved by the writer thread on the host (numpy) "
                         "instead of on the GPU")
    args = ap.parse_args()
    W, H = (int(v) for v in args.size.split("x"))

    from PIL import Image

    import depth_pro
    import generate_depth_maps as G
    from depth_pro import pointcloud as PC

    if args.png_copy:
        def write_png_copy(path, arr):
            import struct
            import zlib
            arr = np.ascontiguousarray(arr)
            if arr.dtype == np.uint16:
                depth, ctype, rows = 16, 0, arr.astype(">u2").view(np.uint8).reshape(arr.shape[0], -1)
            else:
                depth, ctype, rows = 8, 2, arr.reshape(arr.shape[0], -1)
            raw = np.empty((arr.shape[0], rows.shape[1] + 1), np.uint8)
            raw[:, 0] = 0
            raw[:, 1:] = rows

            def chunk(tag, data):
                return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)
            ihdr = struct.pack(">IIBBBBB", arr.shape[1], arr.shape[0], depth, ctype, 0, 0, 0)
            with open(path, "wb") as f:
                f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", zlib.compress(raw.tobytes(), 1))
                        + chunk(b"IEND", b""))
        G._write_png = write_png_copy

    if args.ply_host:
        def points_host_interleave(depth, f_px, image):
            h, w = depth.shape
            rgb = image.to(depth.device, non_blocking=True) if torch.is_tensor(image) else \
                torch.from_numpy(np.ascontiguousarray(image)).to(depth.device, non_blocking=True)
            xyz, _, cols, count = PC.depth_to_points_async(depth, f_px, w, h, rgb=rgb)
            out = []
            for t in (xyz, cols, count):
                hb = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                hb.copy_(t, non_blocking=True)
                out.append(hb)
            return tuple(out)

        def records_on_host(pc):
            xyz, cols, cnt = pc
            n = int(cnt)
            rec = np.empty(n, dtype=[("p", "<f8", 3), ("c", "u1", 3)])
            rec["p"], rec["c"] = xyz[:n].numpy(), cols[:n].numpy()
            return rec.view(np.uint8).reshape(n, PC.PLY_RECORD)
        G._points, G._points_host = points_host_interleave, records_on_host

    if args.switch_ms is not None:
        import sys
        sys.setswitchinterval(args.switch_ms / 1000.0)

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
    main_t = {}
    if args.trace:
        import concurrent.futures as cf
        import threading
        main_id = threading.get_ident()
        orig_result, orig_infer, orig_img = cf.Future.result, m.infer, G._image_async

        def timed(key, fn):
            def w(*a, **k):
                if threading.get_ident() != main_id:
                    return fn(*a, **k)
                t0 = time.perf_counter()
                try:
                    return fn(*a, **k)
                finally:
                    main_t[key] = main_t.get(key, 0.0) + time.perf_counter() - t0
            return w
        cf.Future.result = timed("future_waits", orig_result)
        m.infer = timed("infer_call", orig_infer)
        G._image_async = timed("image_async", orig_img)
    t = time.time()
    n_ok = G.batch_generate_depth_maps(src, dst, **kw)
    torch.cuda.synchronize()
    t_loop = time.time() - t
    if args.trace:
        cf.Future.result, m.infer, G._image_async = orig_result, orig_infer, orig_img

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
        rec = PC.ply_records_async(xyz, cols)[:n].cpu().numpy()
        t = time.time()
        if args.ply_host:
            PC.write_ply(os.path.join(root, "one.ply"), a, c)
        else:
            PC.write_ply_records(os.path.join(root, "one.ply"), rec)
        t_ply = time.time() - t
    out = {
        "what": "generate_depth_maps.batch_generate_depth_maps end to end, 1 GPU",
        "frames": args.frames, "size": [W, H], "pointcloud": args.pointcloud, "raw": args.raw,
        "ply_records": "host (numpy)" if args.ply_host else "GPU",
        "png_writer": "bytes copies" if args.png_copy else "zero-copy parts",
        "switch_ms": args.switch_ms,
        "main_thread_ms_per_frame": {k: round(1000 * v / args.frames, 2) for k, v in main_t.items()} or None,
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
