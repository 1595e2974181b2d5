"""Golden vectors for the frame-loop writers and the point-cloud back-projection, from the
REFERENCE's own `colorize_depth` and `depth_to_3d`.

Run in the build container only:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_frameloop.py

`generate_depth_maps.py` of the reference imports cv2/open3d at module level
(absent here), so the single function `colorize_depth` (generate_depth_maps.py:15-44)
is lifted out of the reference file with `ast` and executed with numpy and
matplotlib -- the reference's own code, on synthetic depth maps.  The `--raw`
path is inline code in the reference (:135-143, no function to call); its
expected output is pinned by restating those two lines here.

`depth_to_3d` (img_to_normalized_pointcloud.py:819-856) is lifted the same way: that module
imports open3d / cv2 / sklearn at the top (absent here), the function itself needs only numpy.
It runs on synthetic depth maps with NaN / zero / negative pixels and an empty row, with the
focal length as a Python float, as its call site passes it (`focallength_px.item()`, :1221).
Output: golden_pointcloud.npz.
"""

import ast
import os

import matplotlib
import numpy as np

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/generate_depth_maps.py"
REF_PC = "/root/reference/img_to_normalized_pointcloud.py"


def lift(path, name, ns):
    """The reference function `name` from `path`, compiled alone into namespace `ns`."""
    tree = ast.parse(open(path).read())
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == name)
    exec(compile(ast.Module(body=[fn], type_ignores=[]), path, "exec"), ns)
    return ns[name]


def reference_colorize():
    return lift(REF, "colorize_depth", {"np": np, "plt": plt})


def pointcloud_fixtures():
    depth_to_3d = lift(REF_PC, "depth_to_3d", {"np": np})
    out = {}
    for i, (h, w, f) in enumerate([(37, 53, 1234.5678), (64, 48, 97.25), (1, 1, 3.0), (270, 480, 1663.8462)]):
        g = np.random.default_rng(100 + i)
        d = (g.random((h, w)) * 20).astype(np.float32)
        if h > 1:
            d[g.random((h, w)) < 0.02] = np.nan
            d[g.random((h, w)) < 0.02] = 0.0
            d[g.random((h, w)) < 0.02] = -3.0
            d[1, :] = np.nan                      # an empty row
        f = float(np.float32(f))                  # an fp32 FOV-head focal length, passed as .item()
        pts, valid = depth_to_3d(d, f, w, h)
        out[f"case{i}_depth"], out[f"case{i}_f"] = d, np.array(f)
        out[f"case{i}_points"], out[f"case{i}_valid"] = pts, valid
    out["n_cases"] = np.array(4)
    np.savez_compressed(os.path.join(HERE, "golden_pointcloud.npz"), **out)
    print("wrote golden_pointcloud.npz", {k: v.shape for k, v in out.items() if k.endswith("points")})


def main():
    colorize = reference_colorize()
    rng = np.random.default_rng(5)
    depth = (rng.random((48, 64)) * 9.0 + 0.5).astype(np.float32)
    depth[3, 4] = np.nan  # nanmin / nanmax path
    out = {"depth": depth}
    for cmap in ("turbo", "viridis", "jet"):
        out[f"color_{cmap}"] = colorize(depth, cmap=cmap)
    d = np.nan_to_num(depth, nan=1.0)
    mn, mx = np.nanmin(d), np.nanmax(d)
    out["raw_u16"] = ((d - mn) / (mx - mn) * 65535).astype(np.uint16)
    np.savez_compressed(os.path.join(HERE, "golden_frameloop.npz"), **out)
    print("wrote golden_frameloop.npz", {k: v.shape for k, v in out.items()})
    pointcloud_fixtures()


if __name__ == "__main__":
    main()
