"""Golden vectors for the frame-loop writers, from the REFERENCE's own `colorize_depth`.

Run in the build container only:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_frameloop.py

`generate_depth_maps.py` of the reference imports cv2/open3d at module level
(absent here), so the single function `colorize_depth` (generate_depth_maps.py:15-44)
is lifted out of the reference file with `ast` and executed with numpy and
matplotlib -- the reference's own code, on synthetic depth maps.  The `--raw`
path is inline code in the reference (:135-143, no function to call); its
expected output is pinned by restating those two lines here.
"""

import ast
import os

import matplotlib
import numpy as np

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/generate_depth_maps.py"


def reference_colorize():
    tree = ast.parse(open(REF).read())
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "colorize_depth")
    mod = ast.Module(body=[fn], type_ignores=[])
    ns = {"np": np, "plt": plt}
    exec(compile(mod, REF, "exec"), ns)
    return ns["colorize_depth"]


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


if __name__ == "__main__":
    main()
