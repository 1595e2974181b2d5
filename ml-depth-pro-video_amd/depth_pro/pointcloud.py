"""Point-cloud write-out of a depth frame (BASELINE config 5).

Reference: `depth_to_3d` (img_to_normalized_pointcloud.py:819-856) followed by the
Open3D PLY write (`o3d.io.write_point_cloud`, :1318).  The back-projection and the
row-major compaction of the valid pixels run in `dp_depth_to_points` (HIP, fp64 as
numpy computes it); the PLY writer is this package's own (no Open3D): binary
little-endian, `double x y z` + `uchar red green blue`, the vertex layout Open3D writes.
The reference's ground-plane normalisation / RANSAC / floor plans are out of scope.
"""

from __future__ import annotations

import ctypes
from typing import Optional, Tuple, Union

import numpy as np
import torch

from . import _lib
from ._lib import check


def depth_to_3d(depth_in: torch.Tensor, focallength_px: Union[float, torch.Tensor], width: int, height: int,
                rgb: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
    """Same arguments and point order as the reference `depth_to_3d`, on the GPU.

    depth_in: (height, width) fp32 device tensor (`model.infer(...)["depth"]`);
    focallength_px: a float, or the device scalar `infer` returns (read on the device);
    rgb: optional (height, width, 3) uint8 device tensor -> colours of the valid points.
    Returns (points (N, 3) fp64, valid_mask (height, width) bool, colors (N, 3) uint8 or None).
    Reads the point count back (one synchronisation); `depth_to_points_async` does not.
    """
    xyz, valid, cols, count = depth_to_points_async(depth_in, focallength_px, width, height, rgb)
    n = int(count.item())
    return xyz[:n], valid, (None if cols is None else cols[:n])


def depth_to_points_async(depth_in: torch.Tensor, focallength_px: Union[float, torch.Tensor], width: int,
                          height: int, rgb: Optional[torch.Tensor] = None):
    """`depth_to_3d` without the read-back: (points buffer (H*W, 3) fp64, valid mask, colours buffer
    or None, device int32 point count).  The first `count` rows of the buffers are the result;
    nothing is synchronised, so a frame loop can queue it behind `infer` and read it later."""
    if depth_in.device.type != "cuda":
        raise _lib.DPError("depth_to_3d runs on the ROCm device (dp_depth_to_points)")
    d = depth_in.detach().to(torch.float32).contiguous()
    if tuple(d.shape) != (height, width):
        raise ValueError(f"depth shape {tuple(d.shape)} != (height, width) = {(height, width)}")
    dev = d.device
    rows = torch.empty(height + 1, dtype=torch.int32, device=dev)
    xyz = torch.empty(height * width, 3, dtype=torch.float64, device=dev)
    cols = None
    if rgb is not None:
        rgb = rgb.contiguous()
        if rgb.dtype != torch.uint8 or tuple(rgb.shape) != (height, width, 3):
            raise ValueError("rgb must be uint8 (height, width, 3)")
        cols = torch.empty(height * width, 3, dtype=torch.uint8, device=dev)
    if torch.is_tensor(focallength_px):
        f_dev = focallength_px.detach().to(device=dev, dtype=torch.float32).reshape(1).contiguous()
        use_given, f_host, f_ptr = 0, 0.0, f_dev.data_ptr()
    else:
        f_dev, use_given, f_host, f_ptr = None, 1, float(focallength_px), None
    stream = torch.cuda.current_stream(dev).cuda_stream
    check(_lib.load().dp_depth_to_points(d.data_ptr(), height, width, f_ptr, f_host, use_given,
                                         None if rgb is None else rgb.data_ptr(), rows.data_ptr(), xyz.data_ptr(),
                                         None if cols is None else cols.data_ptr(), stream), "dp_depth_to_points")
    valid = (d == d) & (d > 0)
    return xyz, valid, cols, rows[height]


PLY_RECORD = 27   # bytes per vertex: double x, y, z + uchar red, green, blue


def ply_records_async(xyz: torch.Tensor, cols: torch.Tensor) -> torch.Tensor:
    """The PLY vertex records of `depth_to_points_async`'s buffers, interleaved on the device
    ((H*W, 27) uint8: the 24 bytes of x, y, z then r, g, b -- the layout `write_ply` writes), so
    that the frame loop's writer only writes bytes.  Queued on the current stream, no sync."""
    n = xyz.shape[0]
    rec = torch.empty(n, PLY_RECORD, dtype=torch.uint8, device=xyz.device)
    rec[:, :24].copy_(xyz.view(torch.uint8).view(n, 24))
    rec[:, 24:].copy_(cols.view(n, 3))
    return rec


def _ply_header(n: int, colored: bool) -> bytes:
    props = ["property double x", "property double y", "property double z"]
    if colored:
        props += ["property uchar red", "property uchar green", "property uchar blue"]
    return ("\n".join(["ply", "format binary_little_endian 1.0", f"element vertex {n}", *props, "end_header"])
            + "\n").encode("ascii")


def write_ply_records(path: str, records: np.ndarray) -> str:
    """`write_ply` for vertex records already in file layout ((n, 27) uint8, `ply_records_async`)."""
    rec = np.ascontiguousarray(records, dtype=np.uint8).reshape(-1, PLY_RECORD)
    if not path.endswith(".ply"):
        path = path + ".ply"
    with open(path, "wb") as f:
        f.write(_ply_header(rec.shape[0], True))
        f.write(memoryview(rec).cast("B"))
    return path


def write_ply(path: str, points: np.ndarray, colors: Optional[np.ndarray] = None) -> str:
    """Binary little-endian PLY: double x, y, z (+ uchar red, green, blue)."""
    pts = np.ascontiguousarray(np.asarray(points, dtype="<f8").reshape(-1, 3))
    n = pts.shape[0]
    if colors is not None:
        col = np.ascontiguousarray(np.asarray(colors, dtype=np.uint8).reshape(-1, 3))
        if col.shape[0] != n:
            raise ValueError("points and colors differ in length")
        body = np.empty(n, dtype=[("p", "<f8", 3), ("c", "u1", 3)])   # the 27-byte vertex records
        body["p"], body["c"] = pts, col
    else:
        body = pts
    if not path.endswith(".ply"):
        path = path + ".ply"
    with open(path, "wb") as f:
        f.write(_ply_header(n, colors is not None))
        # straight from the array's buffer: no bytes copy of the ~224 MB body (4K frame) made with
        # the GIL held, which serialised the loop's writer threads
        f.write(memoryview(body).cast("B"))
    return path


def read_ply(path: str) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    """Reader for the files `write_ply` produces (tests, tools)."""
    with open(path, "rb") as f:
        data = f.read()
    end = data.index(b"end_header\n") + len(b"end_header\n")
    lines = data[:end].decode("ascii").splitlines()
    n = int(next(l for l in lines if l.startswith("element vertex")).split()[-1])
    has_c = any("red" in l for l in lines)
    if has_c:
        rec = np.frombuffer(data[end:], dtype=[("p", "<f8", 3), ("c", "u1", 3)], count=n)
        return rec["p"].copy(), rec["c"].copy()
    return np.frombuffer(data[end:], dtype="<f8", count=3 * n).reshape(n, 3).copy(), None
