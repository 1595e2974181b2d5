"""depth_pro.load_rgb vs the reference's own load_rgb (utils.py:47-112).

Fixtures (tests/golden/make_golden.py --io / the main run): golden_load_rgb.npz holds small
synthetic images (EXIF orientations 1/3/6/8/5, 35 mm focal-length tags incl. 0, grey,
palette and RGBA PNGs) as file bytes together with what the reference returned for them;
golden_example_jpg.npz holds the reference's load_rgb of data/example.jpg (BASELINE config 1;
the image itself is committed as tests/golden/data/example.jpg).
"""

import json
import os

import numpy as np
import pytest

from depth_pro import load_rgb
from depth_pro.utils import fpx_from_f35


def _cases(golden_dir):
    g = np.load(f"{golden_dir}/golden_load_rgb.npz")
    for i in range(int(g["n_files"])):
        yield (str(g[f"file{i}_name"]), g[f"file{i}_bytes"].tobytes(), g[f"file{i}_img"],
               float(g[f"file{i}_fpx"]), bool(g[f"file{i}_icc"]))


def test_load_rgb_matches_reference_on_every_branch(golden_dir, tmp_path):
    n = 0
    for name, data, img_ref, fpx_ref, icc_ref in _cases(golden_dir):
        path = tmp_path / name
        path.write_bytes(data)
        img, icc, fpx = load_rgb(path)
        assert img.dtype == np.uint8 and img.shape == img_ref.shape, name
        assert np.array_equal(img, img_ref), name
        if np.isnan(fpx_ref):
            assert fpx is None, name
        else:
            assert fpx == fpx_ref, (name, fpx, fpx_ref)
        assert (icc is not None) == icc_ref, name
        n += 1
    assert n == 9


def test_load_rgb_example_jpg(golden_dir):
    g = np.load(f"{golden_dir}/golden_example_jpg.npz")
    meta = json.load(open(f"{golden_dir}/golden_meta.json"))["example_jpg"]
    img, icc, fpx = load_rgb(os.path.join(golden_dir, "data", "example.jpg"))
    assert list(img.shape) == meta["shape"] and tuple(img.shape) == tuple(g["shape"])
    assert int(img.astype(np.int64).sum()) == meta["u8_sum"]
    assert np.array_equal(img[::16, ::16], g["img_sub16"])
    assert fpx is None and meta["f_px_exif"] is None     # no 35 mm focal tag: FOV head supplies f_px
    assert icc is not None


def test_fpx_from_f35():
    # a 36 x 24 image at f = 50 mm-equivalent has f_px = 50 * diag / film diag = 50 px-per-mm * ...
    assert fpx_from_f35(36, 24, 50) == pytest.approx(50.0)
    assert fpx_from_f35(3024, 2268, 26) == pytest.approx(26 * np.hypot(3024, 2268) / np.hypot(36, 24))
