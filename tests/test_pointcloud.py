"""Point-cloud write-out: dp_depth_to_points vs the reference depth_to_3d.

The reference function (img_to_normalized_pointcloud.py:819-856) lives in a module that
imports open3d / cv2 at the top, so the oracle restates it (oracle.depth_pro_oracle.depth_to_3d,
same numpy expression); the GPU result must equal it bit for bit (fp64, same op order,
same row-major point order).  Both are pinned to the reference function itself:
tests/golden/golden_pointcloud.npz holds its outputs (lifted out of the reference module
with `ast` by make_golden_frameloop.py).  The PLY writer is checked by a round trip.
"""

import numpy as np
import pytest
import torch

from oracle import depth_pro_oracle as O
from depth_pro import pointcloud as PC


def depth_frame(h, w, seed=0):
    g = np.random.default_rng(seed)
    d = (g.random((h, w)) * 20).astype(np.float32)
    d[g.random((h, w)) < 0.01] = np.nan
    d[g.random((h, w)) < 0.01] = 0.0
    d[g.random((h, w)) < 0.01] = -3.0
    d[0, :] = np.nan                      # an empty row
    return d


def test_oracle_depth_to_3d_known_values():
    d = np.array([[1.0, np.nan], [0.0, 4.0]], dtype=np.float32)
    pts, valid = O.depth_to_3d(d, 2.0, 2, 2)
    assert valid.tolist() == [[True, False], [False, True]]
    # (u, v) = (0, 0): x = -(0 - 1) * 1 / 2 = 0.5, y = 0.5; (1, 1): x = -(1 - 1) * 4 / 2 = 0
    np.testing.assert_array_equal(pts, [[0.5, 0.5, 1.0], [0.0, 0.0, 4.0]])


def _golden_cases(golden_dir):
    g = np.load(f"{golden_dir}/golden_pointcloud.npz")
    for i in range(int(g["n_cases"])):
        yield g[f"case{i}_depth"], float(g[f"case{i}_f"]), g[f"case{i}_points"], g[f"case{i}_valid"]


def test_oracle_depth_to_3d_matches_reference_function(golden_dir):
    for d, f, pts_ref, valid_ref in _golden_cases(golden_dir):
        h, w = d.shape
        pts, valid = O.depth_to_3d(d, f, w, h)
        assert np.array_equal(valid, valid_ref)
        assert pts.dtype == pts_ref.dtype and np.array_equal(pts, pts_ref)


@pytest.mark.gpu
def test_depth_to_points_matches_reference_function(cuda, golden_dir):
    for d, f, pts_ref, valid_ref in _golden_cases(golden_dir):
        h, w = d.shape
        pts, vmask, _ = PC.depth_to_3d(torch.from_numpy(d).to(cuda), f, w, h)
        assert np.array_equal(vmask.cpu().numpy(), valid_ref)
        assert np.array_equal(pts.cpu().numpy(), pts_ref)        # bit-exact fp64


def test_ply_round_trip(tmp_path):
    pts = np.random.default_rng(1).standard_normal((1000, 3))
    cols = np.random.default_rng(2).integers(0, 256, (1000, 3), dtype=np.uint8)
    path = PC.write_ply(str(tmp_path / "a"), pts, cols)
    assert path.endswith(".ply")
    p2, c2 = PC.read_ply(path)
    assert np.array_equal(p2, pts) and np.array_equal(c2, cols)
    head = open(path, "rb").read(200)
    assert head.startswith(b"ply\nformat binary_little_endian 1.0\nelement vertex 1000\nproperty double x\n")
    p3, c3 = PC.read_ply(PC.write_ply(str(tmp_path / "b.ply"), pts))
    assert np.array_equal(p3, pts) and c3 is None


def test_ply_records_layout(tmp_path):
    """The record interleave (x, y, z as 24 little-endian bytes, then r, g, b) and its writer give
    `write_ply`'s file bytes; the frame loop runs the same torch ops on the device (GPU test below)."""
    g = np.random.default_rng(5)
    pts = g.standard_normal((777, 3))
    cols = g.integers(0, 256, (777, 3), dtype=np.uint8)
    rec = PC.ply_records_async(torch.from_numpy(pts), torch.from_numpy(cols))
    assert rec.shape == (777, PC.PLY_RECORD) and rec.dtype == torch.uint8
    a = PC.write_ply_records(str(tmp_path / "r"), rec.numpy())
    b = PC.write_ply(str(tmp_path / "w"), pts, cols)
    assert open(a, "rb").read() == open(b, "rb").read()
    p2, c2 = PC.read_ply(a)
    assert np.array_equal(p2, pts) and np.array_equal(c2, cols)


@pytest.mark.gpu
@pytest.mark.parametrize("h,w", [(2160, 3840), (37, 300)])
def test_ply_records_on_device_write_the_same_file(cuda, tmp_path, h, w):
    """The frame loop's PLY path (vertex records interleaved on the GPU, written as they are) gives
    the same file bytes as `write_ply` of the host points and colours."""
    d = depth_frame(h, w, seed=7)
    rgb = np.random.default_rng(4).integers(0, 256, (h, w, 3), dtype=np.uint8)
    xyz, _, cols, count = PC.depth_to_points_async(torch.from_numpy(d).to(cuda), 987.25, w, h,
                                                   rgb=torch.from_numpy(rgb).to(cuda))
    rec = PC.ply_records_async(xyz, cols)
    n = int(count)
    a = PC.write_ply_records(str(tmp_path / "gpu"), rec[:n].cpu().numpy())
    b = PC.write_ply(str(tmp_path / "host"), xyz[:n].cpu().numpy(), cols[:n].cpu().numpy())
    assert open(a, "rb").read() == open(b, "rb").read()


@pytest.mark.gpu
@pytest.mark.parametrize("h,w", [(2160, 3840), (1536, 1536), (37, 300), (1, 1)])
def test_depth_to_points_bit_exact(cuda, h, w):
    d = depth_frame(h, w, seed=h + w)
    rgb = np.random.default_rng(3).integers(0, 256, (h, w, 3), dtype=np.uint8)
    f = np.float32(1234.5678)
    ref, valid = O.depth_to_3d(d, f.item(), w, h)
    dt, rt = torch.from_numpy(d).to(cuda), torch.from_numpy(rgb).to(cuda)
    for fp in (f.item(), torch.tensor(f, device=cuda)):      # given float, or infer's device f_px
        pts, vmask, cols = PC.depth_to_3d(dt, fp, w, h, rgb=rt)
        got = pts.cpu().numpy()
        assert got.shape == ref.shape
        assert np.array_equal(got, ref)                      # bit-exact fp64, same point order
        assert np.array_equal(vmask.cpu().numpy(), valid)
        assert np.array_equal(cols.cpu().numpy(), rgb[valid])
