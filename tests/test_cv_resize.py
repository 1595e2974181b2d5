"""--downscale_factor: cv2.resize (INTER_AREA for factor < 1, INTER_LINEAR otherwise) as the
reference calls it (generate_depth_maps.py:95-110), on the GPU (dp_resize_u8_cv).

cv2 is not importable here and the reference holds no resized fixture: the oracle
(oracle/cv_resize_oracle.py, OpenCV 4.x's published rules) is pinned by the known-answer
cases below, derived by hand from those rules -- parity UNPINNED vs a cv2 binary."""

import numpy as np
import pytest

from oracle import cv_resize_oracle as CV


def test_area_integer_cells_simd_and_scalar_rounding():
    # 2 x 2 cell summing to 10: the SIMD form (sum + 2) >> 2 = 3 where the row has >= 16 output
    # pixels; narrower rows take the scalar form, round_half_even(10 * 0.25) = 2
    wide = np.repeat(np.tile(np.array([[1, 2], [3, 4]], np.uint8), (1, 32))[:, :, None], 3, axis=2)   # 2 x 64
    assert (CV.resize_area(wide, 1, 32) == 3).all()
    small = np.stack([np.array([[1, 2], [3, 4]], np.uint8)] * 3, -1)
    small = np.tile(small, (2, 2, 1))                                          # 4 x 4 x 3
    assert (CV.resize_area(small, 2, 2) == 2).all()
    # 3 x 3 cells: round_half_even(sum / 9) (float product with 1/9)
    img = np.full((3, 3, 3), 7, np.uint8)
    img[0, 0] = 11                                # sum 67 -> 7.444 -> 7
    assert (CV.resize_area(img, 1, 1) == 7).all()


def test_area_fractional_cells():
    # 3 x 3 -> 2 x 2 (scale 1.5): output (0, 0) weights rows / cols {0: 2/3, 1: 1/3}
    g = np.array([[0, 30, 60], [90, 120, 150], [180, 210, 240]], np.uint8)
    img = np.stack([g, g, g], -1)
    out = CV.resize_area(img, 2, 2)
    # (2/3)[(2/3) 0 + (1/3) 30] + (1/3)[(2/3) 90 + (1/3) 120] = 40; by symmetry (1,1) = 200
    assert out[0, 0, 0] == 40 and out[1, 1, 0] == 200
    # (0, 1): rows {0: 2/3, 1: 1/3}, cols {1: 1/3, 2: 2/3} -> (2/3) 50 + (1/3) 140 = 80
    assert out[0, 1, 0] == 80
    # the reference's call: int(3 * 0.67) = 2
    assert np.array_equal(CV.cv2_resize_u8(img, 0.67), out)


def test_linear_upscale_fixed_point():
    # 2 x 2 -> 4 x 4: x weights (2048, 0) (1536, 512) (512, 1536) (2048, 0) from the half-pixel
    # centres with the border clamp; row 0 reads source row 0 twice (weights 512 / 1536 kept)
    g = np.array([[0, 100], [200, 40]], np.uint8)
    img = np.stack([g, g, g], -1)
    out = CV.resize_linear(img, 4, 4)
    assert out[0, 0, 0] == 0 and out[0, 3, 0] == 100
    assert out[0, 1, 0] == 25                    # SIMD form: (25 + 75 + 2) >> 2
    # (1, 1): rows 0 / 1 at 0.75 / 0.25, cols 0 / 1 at 0.75 / 0.25:
    # 0.75 (0.75 * 0 + 0.25 * 100) + 0.25 (0.75 * 200 + 0.25 * 40) = 58.75; SIMD form:
    # h0 = 51200, h1 = 327680 -> (3200 * 1536 >> 16) + (20480 * 512 >> 16) = 75 + 160 -> (235 + 2) >> 2 = 59;
    # element (1, 3, 0) is in the scalar row tail (bytes 8..11 of a 12-byte row)
    assert out[1, 1, 0] == 59
    assert out[1, 3, 0] == 85                    # 0.75 * 100 + 0.25 * 40 = 85
    assert np.array_equal(CV.cv2_resize_u8(img, 2.0), out)


def _frames():
    rng = np.random.default_rng(3)
    return {(h, w): rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in
            ((64, 96), (101, 77), (45, 160), (20, 18))}


@pytest.mark.gpu
@pytest.mark.parametrize("factor", [0.5, 0.25, 1 / 3, 0.6, 0.37, 1.5, 2.0, 1.27])
def test_gpu_cv_resize_matches_oracle(cuda, factor):
    import torch

    from depth_pro import ops

    for (h, w), img in _frames().items():
        oh, ow = int(h * factor), int(w * factor)
        if oh < 1 or ow < 1:
            continue
        ref = CV.cv2_resize_u8(img, factor)
        got = ops.resize_u8_cv(torch.from_numpy(img).to(cuda), oh, ow, area=factor < 1.0).cpu().numpy()
        assert got.shape == ref.shape
        bad = np.argwhere(got != ref)
        assert bad.size == 0, (factor, (h, w), bad[:5], got[tuple(bad[0])], ref[tuple(bad[0])])
