#!/usr/bin/env python3
"""Drop-in for the reference `generate_depth_maps.py` frame loop, on the MI355X engine.

Same CLI, same functions (`colorize_depth`, `generate_depth_map`,
`batch_generate_depth_maps`), same output names (`{base}_depth.png`) and formats
(turbo-coloured 8-bit RGB PNG over the per-frame depth range, or `--raw`
16-bit grey) as `generate_depth_maps.py:15-251` of the reference.

What changes is the loop: the model is created and packed ONCE
(the reference rebuilds it for every frame, `:76-80`), the forward replays one
HIP graph, frames are decoded by a thread pool ahead of the GPU, only the
uint8 frame crosses PCIe (7 MB at 1536^2 instead of 28 MB fp32), and PNG
encoding runs in writer threads behind the GPU.  Under `torchrun` (one process
per GPU) only rank 0 reads and packs the checkpoint and RCCL-broadcasts the
packed weights; the frame list is sharded k -> rank k mod N and every rank
writes its own frames (`--resume`: rank 0 decides which frames are still
missing, one broadcast before anything is written).  cv2 is not required: PNGs are written with Pillow (pixel-identical
content; the reference's cv2 encoder may choose different zlib settings).
"""

from __future__ import annotations

import argparse
import glob
import os
import queue
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import depth_pro  # noqa: E402  (this package's drop-in)
from depth_pro import distributed as D  # noqa: E402
from depth_pro import pointcloud as PC  # noqa: E402


def colorize_depth(depth, min_depth=None, max_depth=None, cmap="turbo"):
    """Colorize a depth map (reference generate_depth_maps.py:15-44)."""
    import matplotlib.pyplot as plt

    if min_depth is None:
        min_depth = np.nanmin(depth)
    if max_depth is None:
        max_depth = np.nanmax(depth)
    depth_norm = (depth - min_depth) / (max_depth - min_depth)
    depth_norm = np.clip(depth_norm, 0, 1)
    mapper = plt.get_cmap(cmap)
    colored_depth = mapper(depth_norm)[:, :, :3]
    return (colored_depth * 255).astype(np.uint8)


def raw_depth_u16(depth_np: np.ndarray) -> np.ndarray:
    """--raw encoding (reference :135-143)."""
    min_depth = np.nanmin(depth_np)
    max_depth = np.nanmax(depth_np)
    return ((depth_np - min_depth) / (max_depth - min_depth) * 65535).astype(np.uint16)


def _png_parts(arr: np.ndarray, level: int = 1) -> list:
    """The PNG file of an 8-bit RGB (H, W, 3) or 16-bit greyscale (H, W) image as a list of byte
    pieces: filter type 0 on every row and one zlib stream (level 1) -- the same pixels as any PNG
    writer (the reference's cv2.imwrite included), ~3x faster than PIL's adaptive filtering.
    zlib (compress, crc32) runs without the GIL and nothing here copies the image or the
    compressed stream with the GIL held, so the loop's writer threads scale."""
    import struct
    import zlib

    if arr.dtype == np.uint16 and arr.ndim == 2:
        depth, ctype, rows = 16, 0, arr.astype(">u2").view(np.uint8).reshape(arr.shape[0], -1)
    elif arr.dtype == np.uint8 and arr.ndim == 3 and arr.shape[2] == 3:
        depth, ctype, rows = 8, 2, arr.reshape(arr.shape[0], -1)
    else:
        raise ValueError(f"_png_bytes: unsupported image {arr.dtype} {arr.shape}")
    h, w = arr.shape[0], arr.shape[1]
    raw = np.empty((h, rows.shape[1] + 1), np.uint8)
    raw[:, 0] = 0
    raw[:, 1:] = rows

    def chunk(tag: bytes, data) -> list:
        crc = zlib.crc32(data, zlib.crc32(tag)) & 0xFFFFFFFF
        return [struct.pack(">I", len(data)), tag, data, struct.pack(">I", crc)]

    ihdr = struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0)
    idat = zlib.compress(memoryview(raw).cast("B"), level)
    return [b"\x89PNG\r\n\x1a\n", *chunk(b"IHDR", ihdr), *chunk(b"IDAT", idat), *chunk(b"IEND", b"")]


def _png_bytes(arr: np.ndarray, level: int = 1) -> bytes:
    """PNG file bytes of an 8-bit RGB (H, W, 3) or 16-bit greyscale (H, W) image (`_png_parts`)."""
    return b"".join(_png_parts(arr, level))


def _write_png(path: str, arr: np.ndarray) -> None:
    with open(path, "wb") as f:
        for part in _png_parts(np.ascontiguousarray(arr)):
            f.write(part)


_MODEL = {}


def _dist() -> Tuple[int, int]:
    """(world, rank).  Under torchrun (WORLD_SIZE > 1) the process group is created here if the
    caller has not: RCCL ("nccl") on the ROCm device, gloo otherwise."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 1, 0
    if not dist.is_initialized():
        if torch.cuda.is_available():
            dev = _device()
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    return dist.get_world_size(), dist.get_rank()


def _model(device: torch.device, half_precision: bool):
    """One model per (device, precision) per process (the reference reloads it per frame, :76-80).
    In a process group only rank 0 reads and packs the checkpoint; the others receive the packed
    weights over RCCL (distributed.create_model_and_transforms_shared)."""
    key = (str(device), bool(half_precision))
    if key not in _MODEL:
        precision = torch.float16 if half_precision else torch.float32
        cfg = depth_pro.depth_pro.run_config()       # DEPTH_PRO_SYNTHETIC=1: synthetic weights if no checkpoint
        world, _ = _dist()
        if world > 1:
            model, transform = D.create_model_and_transforms_shared(cfg, device, precision)
        else:
            model, transform = depth_pro.create_model_and_transforms(cfg, device=device, precision=precision)
        model.eval()
        model.use_hip_graph(True)
        _MODEL[key] = (model, transform)
    return _MODEL[key]


def _device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    raise RuntimeError("the MI355X Depth Pro engine needs a ROCm GPU")


def _load(image_path: str, downscale_factor: float):
    """Decode (host thread): the frame and its EXIF focal length, scaled by --downscale_factor as
    the reference does (:108-110); the resize itself runs on the GPU (`_downscale`)."""
    image, _, f_px = depth_pro.load_rgb(image_path)
    if downscale_factor != 1.0 and downscale_factor > 0 and f_px is not None:
        f_px = f_px * downscale_factor
    if torch.cuda.is_available():
        # into pinned host memory here, in the decode thread: the upload is then an asynchronous
        # copy on the frame's stream, so the main thread queues frame i+1 while frame i computes
        # (a pageable upload blocks the host until the GPU has finished every earlier frame)
        image = torch.from_numpy(np.ascontiguousarray(image)).pin_memory()
    return image, f_px


def _downscale(image: np.ndarray, downscale_factor: float, device: torch.device):
    """The reference's cv2.resize (:95-107: new size int(H * f) x int(W * f), INTER_AREA for f < 1,
    INTER_LINEAR otherwise) on the GPU (dp_resize_u8_cv): uint8 upload, uint8 frame on the device.
    Without a factor the host frame is returned as is (the transform uploads it)."""
    if downscale_factor == 1.0 or downscale_factor <= 0:
        return image
    from depth_pro import ops

    h, w = image.shape[:2]
    src = image if torch.is_tensor(image) else torch.from_numpy(np.ascontiguousarray(image))
    src = src.to(device, non_blocking=True)
    return ops.resize_u8_cv(src, int(h * downscale_factor), int(w * downscale_factor), area=downscale_factor < 1.0)


def _encode(depth_np: np.ndarray, output_path: str, colored: bool, cmap: str) -> str:
    if colored:
        _write_png(output_path, colorize_depth(depth_np, cmap=cmap))
    else:
        _write_png(output_path, raw_depth_u16(depth_np))
    return output_path


def _image_async(depth: torch.Tensor, colored: bool, cmap: str) -> torch.Tensor:
    """The PNG content of a device depth map, made on the GPU (dp_depth_to_image: colorize_depth /
    --raw, byte-identical) and queued into pinned host memory on the current stream (no host
    sync): the writer thread only PNG-encodes it after the frame's event."""
    from depth_pro import ops

    img = ops.depth_to_image(depth.contiguous(), colored=colored, cmap=cmap)
    host = torch.empty(img.shape, dtype=img.dtype, pin_memory=True)
    host.copy_(img, non_blocking=True)
    return host


def _host_image(host: torch.Tensor) -> np.ndarray:
    a = host.numpy()
    return a.view(np.uint16) if a.dtype == np.int16 else a


def generate_depth_map(image_path, output_path=None, downscale_factor=1.0, half_precision=False, colored=True,
                       cmap="turbo"):
    """One frame (reference :46-151); returns the output path or None on error."""
    try:
        if output_path is None:
            base_name = os.path.splitext(os.path.basename(image_path))[0]
            output_path = f"{base_name}_depth.png"
        model, transform = _model(_device(), half_precision)
        image, f_px = _load(image_path, downscale_factor)
        image = _downscale(image, downscale_factor, _device())
        with torch.no_grad():
            depth = model.infer(transform(image), f_px=f_px)["depth"]
        model.last_status().check()
        if depth.is_cuda:
            host = _image_async(depth, colored, cmap)
            torch.cuda.current_stream(depth.device).synchronize()
            _write_png(output_path, _host_image(host))
            return output_path
        return _encode(depth.detach().cpu().numpy(), output_path, colored, cmap)
    except Exception as e:  # reference :147-151: report and skip the frame
        print(f"Error generating depth map for {image_path}: {str(e)}")
        import traceback

        traceback.print_exc()
        return None


def output_name(image_path: str) -> str:
    """`{base}_depth.png` (reference :187-188)."""
    return f"{os.path.splitext(os.path.basename(image_path))[0]}_depth.png"


def plan_frames(image_paths, output_dir: str, world: int, rank: int, resume: bool) -> List[int]:
    """Indices of the frames this rank processes: the frames still to do (all of them, or with
    `resume` those whose output file is missing -- decided by rank 0 alone and broadcast before
    any rank writes, so every rank shards the same list), dealt round-robin over the ranks."""
    todo = list(range(len(image_paths)))
    if resume:
        if rank == 0:
            todo = [k for k in todo if not os.path.exists(os.path.join(output_dir, output_name(image_paths[k])))]
        if world > 1:
            box = [todo]
            dist.broadcast_object_list(box, src=0)
            todo = box[0]
    return [todo[i] for i in D.shard_frames(len(todo), rank, world)]


def batch_generate_depth_maps(input_dir, output_dir, pattern="*.png", downscale_factor=1.0, half_precision=False,
                              colored=True, cmap="turbo", decode_workers=4, encode_workers=None, pointcloud=False,
                              resume=False, model=None):
    """Directory loop (reference :153-206), pipelined decode -> GPU -> encode, frame-sharded across ranks.

    Every rank writes its own frames' files; each frame has exactly one owner.  resume=True skips
    frames whose `{base}_depth.png` already exists (checkpoint/resume row).
    pointcloud=True also writes `{base}_points.ply` per frame: the reference's depth_to_3d
    back-projection with the frame's focal length (EXIF, or the FOV head's) and RGB colours
    (the reference's ground-plane normalisation is out of scope).
    `model`: an already-built (model, transform) pair (tests); default: `_model`.
    Returns the number of frames this rank wrote.
    """
    os.makedirs(output_dir, exist_ok=True)
    image_paths = sorted(glob.glob(os.path.join(input_dir, pattern)))
    if not image_paths:
        print(f"No images found matching pattern {os.path.join(input_dir, pattern)}")
        return 0
    world, rank = _dist()
    mine = plan_frames(image_paths, output_dir, world, rank, resume)
    print(f"[rank {rank}/{world}] Found {len(image_paths)} images, processing {len(mine)}")
    if model is None:
        model = _model(_device(), half_precision)
    model, transform = model
    if encode_workers is None:   # PNG (+ PLY) writing is the host side's long pole: zlib drops the GIL
        encode_workers = max(4, min(8, len(os.sched_getaffinity(0)) // 2))

    successful = 0
    t0 = time.time()
    # frames queued to the writers but not written yet (each holds pinned host copies of its
    # depth map and, with --pointcloud, its points): at most this many, so host memory stays
    # bounded when PNG / PLY writing falls behind the GPU
    max_inflight = 2 * encode_workers

    def collect(f):
        nonlocal successful
        try:
            if f is not None and f.result() is not None:
                successful += 1
        except Exception as e:  # a bad frame or a write failure skips that frame, like the reference
            print(f"Error writing a depth map: {e}")

    with ThreadPoolExecutor(decode_workers) as dec, ThreadPoolExecutor(encode_workers) as enc:
        futs = {k: dec.submit(_load, image_paths[k], downscale_factor) for k in mine[: 2 * decode_workers]}
        nxt = 2 * decode_workers
        pending = []
        for n, k in enumerate(mine):
            base_name = os.path.splitext(os.path.basename(image_paths[k]))[0]
            output_path = os.path.join(output_dir, output_name(image_paths[k]))
            while len(pending) >= max_inflight:
                collect(pending.pop(0))
            try:
                image, f_px = futs.pop(k).result()
                if nxt < len(mine):
                    futs[mine[nxt]] = dec.submit(_load, image_paths[mine[nxt]], downscale_factor)
                    nxt += 1
                if downscale_factor != 1.0 and downscale_factor > 0:
                    image = _downscale(image, downscale_factor, getattr(transform, "device", None) or _device())
                with torch.no_grad():
                    pred = model.infer(transform(image), f_px=f_px)
                    depth = pred["depth"]
                # this frame's health (engine.FrameStatus: a timed-out stream-K hand-off, NaN / inf
                # output), checked by the writer after the frame's event, before any file is written;
                # claimed, so the next infer's sweep of finished frames leaves it to that writer (a
                # bad frame is dropped once, by its writer, never the next frame in its place)
                status = model.last_status() if hasattr(model, "last_status") else None
                if status is not None and hasattr(status, "claim"):
                    status.claim()
                pc = None
                gpu_img = False
                if depth.is_cuda:
                    # the PNG content (colour / raw) made on the GPU, and every device->host copy,
                    # queued behind the frame on this stream; a writer thread waits on its event
                    host = _image_async(depth, colored, cmap)
                    gpu_img = True
                    if pointcloud:
                        pc = _points(depth, pred["focallength_px"], image)
                    ev = torch.cuda.Event()
                    ev.record()
                else:
                    host, ev = depth, None

                def _finish(host=host, ev=ev, path=output_path, pc=pc, base=base_name, status=status,
                            gpu_img=gpu_img):
                    if ev is not None:
                        ev.synchronize()
                    if status is not None:
                        status.check()          # raises: this frame is dropped, nothing written
                    if pc is not None:
                        PC.write_ply_records(os.path.join(output_dir, f"{base}_points.ply"), _points_host(pc))
                    if gpu_img:
                        _write_png(path, _host_image(host))
                        return path
                    return _encode(host.numpy(), path, colored, cmap)

                pending.append(enc.submit(_finish))
            except Exception as e:
                print(f"Error generating depth map for {image_paths[k]}: {str(e)}")
                pending.append(None)
            print(f"[{n + 1}/{len(mine)}] Processing {base_name}")
        for f in pending:
            collect(f)
    dt = time.time() - t0
    print(f"Processing complete: {successful}/{len(mine)} images successfully processed "
          f"({len(mine) / max(dt, 1e-9):.2f} frames/s on rank {rank})")
    return successful


def _points(depth: torch.Tensor, f_px, image):
    """Queue the frame's point cloud on the GPU (depth_to_3d, img_to_normalized_pointcloud.py:819-856),
    interleaved into PLY vertex records there, and their copy into a pinned host buffer, on the
    current stream, without a host synchronisation: the full-size record buffer + the point count
    (the writer slices it after the frame's event and writes it as it is)."""
    h, w = depth.shape
    rgb = image.to(depth.device, non_blocking=True) if torch.is_tensor(image) else \
        torch.from_numpy(np.ascontiguousarray(image)).to(depth.device, non_blocking=True)
    xyz, _, cols, count = PC.depth_to_points_async(depth, f_px, w, h, rgb=rgb)
    out = []
    for t in (PC.ply_records_async(xyz, cols), count):
        hbuf = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        hbuf.copy_(t, non_blocking=True)
        out.append(hbuf)
    return tuple(out)


def _points_host(pc):
    """Writer-thread side (after the frame's event): exactly the valid points' records."""
    rec, n_host = pc
    return rec[:int(n_host)].numpy()


def main():
    parser = argparse.ArgumentParser(description="Generate depth maps from input images")
    parser.add_argument("--input_dir", type=str, default="./TEMP/FRAMES", help="Directory containing input images")
    parser.add_argument("--output_dir", type=str, default="./TMP/DEPTH", help="Directory to save output depth maps")
    parser.add_argument("--pattern", type=str, default="*.png", help="Glob pattern to match input images")
    parser.add_argument("--downscale_factor", type=float, default=1.0,
                        help="Downscale input images for faster processing")
    parser.add_argument("--half_precision", action="store_true", help="Use float16 for faster computation")
    parser.add_argument("--raw", action="store_true", help="Save raw depth maps (grayscale) instead of colored ones")
    parser.add_argument("--pointcloud", action="store_true",
                        help="Also write {frame}_points.ply (depth_to_3d back-projection with RGB colours)")
    parser.add_argument("--resume", action="store_true",
                        help="Skip frames whose {frame}_depth.png already exists in --output_dir")
    parser.add_argument("--colormap", type=str, default="turbo",
                        choices=["turbo", "viridis", "plasma", "inferno", "magma", "cividis", "jet"],
                        help="Colormap for depth visualization")
    args = parser.parse_args()
    batch_generate_depth_maps(input_dir=args.input_dir, output_dir=args.output_dir, pattern=args.pattern,
                              downscale_factor=args.downscale_factor, half_precision=args.half_precision,
                              colored=not args.raw, cmap=args.colormap, pointcloud=args.pointcloud,
                              resume=args.resume)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
