"""Host-side image loading for the drop-in API (reference `src/depth_pro/utils.py`).

`load_rgb(path, auto_rotate=True, remove_alpha=True) -> (uint8 HxWx3, icc_profile, f_px | None)`
behaves as the reference's (`utils.py:47-112`, pinned byte-for-byte by
tests/golden/golden_load_rgb.npz and golden_example_jpg.npz):

* decode with PIL (HEIC through the optional `pillow_heif`);
* upright the image from the EXIF Orientation tag -- only 3, 6 and 8 are acted on,
  anything else but 1 is logged and ignored;
* grey / single-channel images become 3 identical channels, a 4th (alpha) channel is
  dropped;
* the focal length in pixels comes from the first 35 mm-equivalent focal-length tag
  present (three spellings are looked up, as the reference does); absent or <= 0
  means "unknown" (None), and the FOV head estimates it downstream.

The tag table is built once: TIFF IFD0 names override Exif sub-IFD names, which is
the reference's dict-merge order (`utils.py:30-39`).
"""

from __future__ import annotations

import logging
from pathlib import Path
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np
from PIL import ExifTags, Image, TiffTags

LOGGER = logging.getLogger(__name__)

EXIF_SUB_IFD = 0x8769
# Orientation tag value -> the PIL transpose that uprights the image (utils.py:78-87)
UPRIGHT = {3: Image.ROTATE_180, 6: Image.ROTATE_270, 8: Image.ROTATE_90}
# looked up in this order; the first one present wins, even if its value is 0 (utils.py:100-105)
FOCAL_35MM_TAGS = ("FocalLengthIn35mmFilm", "FocalLenIn35mmFilm", "FocalLengthIn35mmFormat")
FILM_DIAGONAL_MM = float(np.sqrt(36.0**2 + 24.0**2))


def _named(tags, namer) -> Dict[str, Any]:
    out = {}
    for code, value in tags.items():
        name = namer(code)
        if name is not None:
            out[name] = value
    return out


def extract_exif(img_pil: Image.Image) -> Dict[str, Any]:
    """Tag name -> value over the Exif sub-IFD and IFD0 (IFD0 wins on a name clash)."""
    ifd0 = img_pil.getexif()
    table = _named(ifd0.get_ifd(EXIF_SUB_IFD), ExifTags.TAGS.get)
    table.update(_named(ifd0, lambda c: TiffTags.TAGS_V2[c].name if c in TiffTags.TAGS_V2 else None))
    return table


def fpx_from_f35(width: float, height: float, f_mm: float = 50) -> float:
    """35 mm-equivalent focal length [mm] -> pixels: scale by image diagonal / film diagonal."""
    return f_mm * np.sqrt(width**2.0 + height**2.0) / FILM_DIAGONAL_MM


def _open(path: Path) -> Image.Image:
    if path.suffix.lower() != ".heic":
        return Image.open(path)
    try:
        import pillow_heif
    except ImportError as e:  # the reference imports it unconditionally
        raise ImportError("loading .heic needs pillow_heif") from e
    return pillow_heif.open_heif(path, convert_hdr_to_8bit=True).to_pillow()


def _focal_35mm(tags: Dict[str, Any]) -> Optional[float]:
    for name in FOCAL_35MM_TAGS:
        if name in tags:
            return tags[name]
    return None


def load_rgb(path: Union[Path, str], auto_rotate: bool = True, remove_alpha: bool = True
             ) -> Tuple[np.ndarray, List[bytes], Optional[float]]:
    """Load an image as uint8 HxWx3 (+ ICC profile, + focal length in pixels or None)."""
    img_pil = _open(Path(path))
    tags = extract_exif(img_pil)
    icc_profile = img_pil.info.get("icc_profile", None)

    if auto_rotate:
        orientation = tags.get("Orientation", 1)
        if orientation in UPRIGHT:
            img_pil = img_pil.transpose(UPRIGHT[orientation])
        elif orientation != 1:
            LOGGER.warning(f"Ignoring image orientation {orientation}.")

    img = np.array(img_pil)
    if img.ndim == 2 or img.shape[2] == 1:
        img = np.repeat(img.reshape(img.shape[0], img.shape[1], 1), 3, axis=2)
    if remove_alpha:
        img = img[:, :, :3]

    f35 = _focal_35mm(tags)
    f_px = fpx_from_f35(img.shape[1], img.shape[0], f35) if f35 is not None and f35 > 0 else None
    return img, icc_profile, f_px
