"""numpy restatement of OpenCV's cv::resize for 8-bit 3-channel images -- TEST INFRASTRUCTURE ONLY.

The reference downscales frames with `cv2.resize(image, (new_w, new_h), interpolation=cv2.INTER_AREA
if downscale_factor < 1.0 else cv2.INTER_LINEAR)` (generate_depth_maps.py:95-110), with
new_h = int(H * factor), new_w = int(W * factor).  OpenCV is a third-party dependency
(`opencv-python>=4.5.0`, reference 3d_effects_requirements.txt:15; not installed here), so its
published algorithm (imgproc/src/resize.cpp, OpenCV 4.x) is restated below and the product's HIP
kernel (`dp_resize_u8_cv`) is checked against this file.  PARITY UNPINNED vs a cv2 binary: no cv2 is
importable here and the reference holds no resized fixture; the known-answer cases in
tests/test_cv_resize.py are derived by hand from the formulas.

INTER_LINEAR (resizeGeneric_, fixed point, INTER_RESIZE_COEF_BITS = 11):
  fx = (float)((dx + 0.5) * scale_x - 0.5); sx = floor(fx); fx -= sx; sx < 0 -> (sx, fx) = (0, 0);
  sx >= W - 1 -> (sx, fx) = (W - 1, 0); ax = (round(2048 (1 - fx)), round(2048 fx)) (float products,
  round half to even, short); rows likewise (fy, sy; rows clamped to [0, H - 1], weights kept);
  horizontal pass h = S[sx] ax0 + S[sx + 1] ax1 (int);
  vertical pass, SIMD form (VResizeLinearVec_32s8u: all but the row tail):
      d = sat_u8((mulhi(h0 >> 4, by0) + mulhi(h1 >> 4, by1) + 2) >> 2),  mulhi(a, b) = (a b) >> 16
  and for the row tail (the last 1..8 bytes the 16-byte SIMD loops leave, SSE width) the scalar
  form d = sat_u8((h0 by0 + h1 by1 + 2^21) >> 22).
INTER_AREA, integer scale (resizeAreaFast_): 2 x 2 cells -> (a + b + c + d + 2) >> 2 (SIMD form,
  ResizeAreaFastVec_SIMD_8u; its scalar row tail: round_half_even(sum * 0.25f)); other integer
  scales -> round_half_even(sum * (1.f / area)).
INTER_AREA, other scales (resizeArea_ with computeResizeAreaTab): per axis, the source cells
  overlapping [d * scale, (d + 1) * scale) with weights overlap / cellWidth (float), summed in
  table order in float (horizontal per source row, then rows weighted in order), then
  round_half_even.
"""

from __future__ import annotations

import math

import numpy as np

COEF = 2048          # INTER_RESIZE_COEF_SCALE
SIMD_BYTES = 16      # vector width the row-tail rule assumes (SSE baseline)
DBL_EPSILON = np.finfo(np.float64).eps


def _f32(x):
    return np.float32(x)


def _round_even(x) -> np.ndarray:
    return np.rint(np.asarray(x, dtype=np.float32)).astype(np.int64)   # cvRound: round half to even


def _scales(h: int, w: int, oh: int, ow: int):
    """cv::resize: inv_scale = dsize / ssize (double), scale = 1 / inv_scale."""
    return 1.0 / (oh / h), 1.0 / (ow / w)


def _linear_taps(d: int, scale: float, n: int, clamp_index: bool):
    """(index0, index1, w0, w1) per output position of one axis (resizeGeneric_ tables)."""
    i0 = np.empty(d, np.int64)
    w = np.empty((d, 2), np.int64)
    for k in range(d):
        f = _f32((k + 0.5) * scale - 0.5)
        s = int(math.floor(f))
        f = _f32(f - _f32(s))
        if clamp_index:
            if s < 0:
                f, s = _f32(0.0), 0
            if s >= n - 1:
                f, s = _f32(0.0), n - 1
        i0[k] = s
        w[k, 0] = int(np.rint(_f32(_f32(1.0) - f) * _f32(COEF)))
        w[k, 1] = int(np.rint(f * _f32(COEF)))
    return i0, w


def _tail_mask(width: int) -> np.ndarray:
    """Elements of a row of `width` bytes that the scalar tail of a 16-byte SIMD loop pair
    (one loop of 16 bytes while x <= width - 16, then 8-lane int16 blocks while x < width - 8)
    handles."""
    x = (width // SIMD_BYTES) * SIMD_BYTES if width >= SIMD_BYTES else 0
    half = SIMD_BYTES // 2
    while x < width - half:
        x += half
    m = np.zeros(width, bool)
    m[x:] = True
    return m


def resize_linear(img: np.ndarray, oh: int, ow: int) -> np.ndarray:
    h, w, c = img.shape
    sy_, sx_ = _scales(h, w, oh, ow)
    x0, ax = _linear_taps(ow, sx_, w, True)
    y0, by = _linear_taps(oh, sy_, h, False)
    x1 = np.minimum(x0 + 1, w - 1)
    s = img.astype(np.int64)
    hor = s[:, x0, :] * ax[None, :, 0, None] + s[:, x1, :] * ax[None, :, 1, None]   # [h][ow][c]
    r0 = np.clip(y0, 0, h - 1)
    r1 = np.clip(y0 + 1, 0, h - 1)
    h0, h1 = hor[r0], hor[r1]                      # [oh][ow][c]
    b0, b1 = by[:, 0, None, None], by[:, 1, None, None]
    simd = ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2
    scal = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22
    tail = _tail_mask(ow * c).reshape(ow, c)[None]
    return np.clip(np.where(tail, scal, simd), 0, 255).astype(np.uint8)


def _area_tab(ssize: int, dsize: int, scale: float):
    """computeResizeAreaTab: per output index, [(source index, alpha float32)] in table order."""
    tab = []
    for dx in range(dsize):
        fsx1 = dx * scale
        fsx2 = fsx1 + scale
        cell = min(scale, ssize - fsx1)
        sx1, sx2 = math.ceil(fsx1), math.floor(fsx2)
        sx2 = min(sx2, ssize - 1)
        sx1 = min(sx1, sx2)
        row = []
        if sx1 - fsx1 > 1e-3:
            row.append((sx1 - 1, _f32((sx1 - fsx1) / cell)))
        for sx in range(sx1, sx2):
            row.append((sx, _f32(1.0 / cell)))
        if fsx2 - sx2 > 1e-3:
            row.append((sx2, _f32(min(min(fsx2 - sx2, 1.0), cell) / cell)))
        tab.append(row)
    return tab


def resize_area(img: np.ndarray, oh: int, ow: int) -> np.ndarray:
    h, w, c = img.shape
    sy_, sx_ = _scales(h, w, oh, ow)
    isx, isy = int(round(sx_)), int(round(sy_))
    if abs(sx_ - isx) < DBL_EPSILON and abs(sy_ - isy) < DBL_EPSILON:
        # resizeAreaFast_: the output fits whole cells (new size = int(size * factor))
        s = img[:oh * isy, :ow * isx].astype(np.int64).reshape(oh, isy, ow, isx, c).sum(axis=(1, 3))
        if isx == 2 and isy == 2:
            simd = (s + 2) >> 2
            scal = _round_even(s.astype(np.float32) * _f32(0.25))
            # the SIMD loop takes whole 3 x 16-pixel groups of the row
            n_simd = (ow // SIMD_BYTES) * SIMD_BYTES if ow * c >= 3 * SIMD_BYTES else 0
            tail = np.zeros((ow, c), bool)
            tail[n_simd:] = True
            out = np.where(tail[None], scal, simd)
        else:
            out = _round_even(s.astype(np.float32) * _f32(1.0 / (isx * isy)))
        return np.clip(out, 0, 255).astype(np.uint8)
    xt, yt = _area_tab(w, ow, sx_), _area_tab(h, oh, sy_)
    src = img.astype(np.float32)
    out = np.empty((oh, ow, c), np.float32)
    for dy in range(oh):
        acc = np.zeros((ow, c), np.float32)
        for (sy, beta) in yt[dy]:
            buf = np.zeros((ow, c), np.float32)
            for dx in range(ow):
                b = np.zeros(c, np.float32)
                for (sx, alpha) in xt[dx]:
                    b = (b + src[sy, sx] * alpha).astype(np.float32)
                buf[dx] = b
            acc = (acc + (beta * buf).astype(np.float32)).astype(np.float32)
        out[dy] = acc
    return np.clip(_round_even(out), 0, 255).astype(np.uint8)


def cv2_resize_u8(img: np.ndarray, factor: float) -> np.ndarray:
    """The reference's downscale call: new size int(H * factor) x int(W * factor), INTER_AREA
    for factor < 1, INTER_LINEAR otherwise (generate_depth_maps.py:95-110)."""
    h, w = img.shape[:2]
    oh, ow = int(h * factor), int(w * factor)
    return resize_area(img, oh, ow) if factor < 1.0 else resize_linear(img, oh, ow)
