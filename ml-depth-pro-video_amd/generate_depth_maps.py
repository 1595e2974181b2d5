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
encoding runs in writer threads behind the GPU.  Under `torchrun` the frame
list is sharded k -> rank k mod N (one process per GPU); every rank writes its
own frames.  cv2 is not required: PNGs are written with Pillow (pixel-identical
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
from typing import Optional

import numpy as np
import torch

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


def _write_png(path: str, arr: np.ndarray) -> None:
    from PIL import Image

    if arr.dtype == np.uint16:
        Image.fromarray(np.ascontiguousarray(arr)).save(path)          # 16-bit greyscale (I;16)
    else:
        Image.fromarray(np.ascontiguousarray(arr)).save(path, compress_level=1)


def _resize_u8(image: np.ndarray, factor: float) -> np.ndarray:
    """Host stand-in for cv2.resize(INTER_AREA if factor < 1 else INTER_LINEAR) (reference :95-110)."""
    from PIL import Image

    h, w = image.shape[:2]
    nh, nw = int(h * factor), int(w * factor)
    resample = Image.BOX if factor < 1.0 else Image.BILINEAR
    return np.asarray(Image.fromarray(image).resize((nw, nh), resample=resample))


_MODEL = {}


def _model(device: torch.device, half_precision: bool):
    """One model per (device, precision) per process (the reference reloads per frame)."""
    key = (str(device), bool(half_precision))
    if key not in _MODEL:
        precision = torch.float16 if half_precision else torch.float32
        cfg = depth_pro.DEFAULT_MONODEPTH_CONFIG_DICT
        if not os.path.exists(cfg.checkpoint_uri or "") and os.environ.get("DEPTH_PRO_SYNTHETIC", "0") == "1":
            from depth_pro.depth_pro import DepthProConfig

            print(f"checkpoint {cfg.checkpoint_uri} not found: using synthetic weights (DEPTH_PRO_SYNTHETIC=1)")
            cfg = DepthProConfig(patch_encoder_preset="dinov2l16_384", image_encoder_preset="dinov2l16_384",
                                 checkpoint_uri=None, decoder_features=256, use_fov_head=True,
                                 fov_encoder_preset="dinov2l16_384")
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
    image, _, f_px = depth_pro.load_rgb(image_path)
    if downscale_factor != 1.0 and downscale_factor > 0:
        image = _resize_u8(image, downscale_factor)
        if f_px is not None:
            f_px = f_px * downscale_factor
    return image, f_px


def _encode(depth_np: np.ndarray, output_path: str, colored: bool, cmap: str) -> str:
    if colored:
        _write_png(output_path, colorize_depth(depth_np, cmap=cmap))
    else:
        _write_png(output_path, raw_depth_u16(depth_np))
    return output_path


def generate_depth_map(image_path, output_path=None, downscale_factor=1.0, half_precision=False, colored=True,
                       cmap="turbo"):
    """One frame (reference :46-151); returns the output path or None on error."""
    try:
        if output_path is None:
            base_name = os.path.splitext(os.path.basename(image_path))[0]
            output_path = f"{base_name}_depth.png"
        model, transform = _model(_device(), half_precision)
        image, f_px = _load(image_path, downscale_factor)
        with torch.no_grad():
            depth = model.infer(transform(image), f_px=f_px)["depth"]
        return _encode(depth.detach().cpu().numpy(), output_path, colored, cmap)
    except Exception as e:  # reference :147-151: report and skip the frame
        print(f"Error generating depth map for {image_path}: {str(e)}")
        import traceback

        traceback.print_exc()
        return None


def _points(depth: torch.Tensor, f_px, image: np.ndarray, device: torch.device):
    """Camera-space point cloud of one frame on the GPU (depth_to_3d, img_to_normalized_pointcloud.py:819-856)."""
    h, w = depth.shape
    rgb = torch.from_numpy(np.ascontiguousarray(image)).to(device, non_blocking=True)
    pts, _, cols = PC.depth_to_3d(depth, f_px, w, h, rgb=rgb)
    host_p = torch.empty(pts.shape, dtype=pts.dtype, pin_memory=True)
    host_c = torch.empty(cols.shape, dtype=cols.dtype, pin_memory=True)
    host_p.copy_(pts, non_blocking=True)
    host_c.copy_(cols, non_blocking=True)
    return host_p, host_c


def batch_generate_depth_maps(input_dir, output_dir, pattern="*.png", downscale_factor=1.0, half_precision=False,
                              colored=True, cmap="turbo", decode_workers=4, encode_workers=4, pointcloud=False):
    """Directory loop (reference :153-206), pipelined decode -> GPU -> encode, frame-sharded across ranks.

    pointcloud=True also writes `{base}_points.ply` per frame: the reference's depth_to_3d
    back-projection with the frame's focal length (EXIF, or the FOV head's) and RGB colours
    (the reference's ground-plane normalisation is out of scope)."""
    os.makedirs(output_dir, exist_ok=True)
    image_paths = sorted(glob.glob(os.path.join(input_dir, pattern)))
    if not image_paths:
        print(f"No images found matching pattern {os.path.join(input_dir, pattern)}")
        return 0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    mine = D.shard_frames(len(image_paths), rank, world)
    print(f"[rank {rank}/{world}] Found {len(image_paths)} images, processing {len(mine)}")
    device = _device()
    model, transform = _model(device, half_precision)

    successful = 0
    t0 = time.time()
    with ThreadPoolExecutor(decode_workers) as dec, ThreadPoolExecutor(encode_workers) as enc:
        futs = {k: dec.submit(_load, image_paths[k], downscale_factor) for k in mine[: 2 * decode_workers]}
        nxt = 2 * decode_workers
        pending = []
        for n, k in enumerate(mine):
            base_name = os.path.splitext(os.path.basename(image_paths[k]))[0]
            output_path = os.path.join(output_dir, f"{base_name}_depth.png")
            try:
                image, f_px = futs.pop(k).result()
                if nxt < len(mine):
                    futs[mine[nxt]] = dec.submit(_load, image_paths[mine[nxt]], downscale_factor)
                    nxt += 1
                with torch.no_grad():
                    pred = model.infer(transform(image), f_px=f_px)
                    depth = pred["depth"]
                host = torch.empty(depth.shape, dtype=depth.dtype, pin_memory=True)
                host.copy_(depth, non_blocking=True)
                pc = _points(depth, pred["focallength_px"], image, device) if pointcloud else None
                ev = torch.cuda.Event()
                ev.record()

                def _finish(host=host, ev=ev, path=output_path, pc=pc, base=base_name):
                    ev.synchronize()
                    if pc is not None:
                        PC.write_ply(os.path.join(output_dir, f"{base}_points.ply"), pc[0].numpy(), pc[1].numpy())
                    return _encode(host.numpy(), path, colored, cmap)

                pending.append(enc.submit(_finish))
            except Exception as e:
                print(f"Error generating depth map for {image_paths[k]}: {str(e)}")
                pending.append(None)
            print(f"[{n + 1}/{len(mine)}] Processing {base_name}")
        for f in pending:
            if f is not None and f.result() is not None:
                successful += 1
    dt = time.time() - t0
    print(f"Processing complete: {successful}/{len(mine)} images successfully processed "
          f"({len(mine) / max(dt, 1e-9):.2f} frames/s on rank {rank})")
    return successful


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
    parser.add_argument("--colormap", type=str, default="turbo",
                        choices=["turbo", "viridis", "plasma", "inferno", "magma", "cividis", "jet"],
                        help="Colormap for depth visualization")
    args = parser.parse_args()
    batch_generate_depth_maps(input_dir=args.input_dir, output_dir=args.output_dir, pattern=args.pattern,
                              downscale_factor=args.downscale_factor, half_precision=args.half_precision,
                              colored=not args.raw, cmap=args.colormap, pointcloud=args.pointcloud)


if __name__ == "__main__":
    main()
