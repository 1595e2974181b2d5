"""Image loading (reference `src/depth_pro/utils.py:16-112`).

`load_rgb(path) -> (uint8 HxWx3, icc_profile, f_px | None)`: PIL decode, EXIF
orientation (3/6/8), grey -> RGB, alpha dropped, and the focal length in
pixels from the 35 mm-equivalent EXIF focal length when present.  HEIC needs
`pillow_heif`, which is optional here (an ImportError names it when absent).
"""

from __future__ import annotations

import logging
from pathlib import Path
from typing import Any, Dict, List, Tuple, Union

import numpy as np
from PIL import ExifTags, Image, TiffTags

LOGGER = logging.getLogger(__name__)


def extract_exif(img_pil: Image.Image) -> Dict[str, Any]:
    """EXIF (IFD 0x8769) and TIFF tags as one name -> value dict (utils.py:16-39)."""
    img_exif = img_pil.getexif().get_ifd(0x8769)
    exif_dict = {ExifTags.TAGS[k]: v for k, v in img_exif.items() if k in ExifTags.TAGS}
    tiff_tags = img_pil.getexif()
    tiff_dict = {TiffTags.TAGS_V2[k].name: v for k, v in tiff_tags.items() if k in TiffTags.TAGS_V2}
    return {**exif_dict, **tiff_dict}


def fpx_from_f35(width: float, height: float, f_mm: float = 50) -> float:
    """35 mm-equivalent focal length [mm] -> pixels (utils.py:42-44)."""
    return f_mm * np.sqrt(width**2.0 + height**2.0) / np.sqrt(36**2 + 24**2)


def load_rgb(path: Union[Path, str], auto_rotate: bool = True, remove_alpha: bool = True
             ) -> Tuple[np.ndarray, List[bytes], float]:
    path = Path(path)
    if path.suffix.lower() in [".heic"]:
        try:
            import pillow_heif
        except ImportError as e:  # the reference imports it unconditionally
            raise ImportError("loading .heic needs pillow_heif") from e
        img_pil = pillow_heif.open_heif(path, convert_hdr_to_8bit=True).to_pillow()
    else:
        img_pil = Image.open(path)

    img_exif = extract_exif(img_pil)
    icc_profile = img_pil.info.get("icc_profile", None)

    if auto_rotate:
        orientation = img_exif.get("Orientation", 1)
        if orientation == 3:
            img_pil = img_pil.transpose(Image.ROTATE_180)
        elif orientation == 6:
            img_pil = img_pil.transpose(Image.ROTATE_270)
        elif orientation == 8:
            img_pil = img_pil.transpose(Image.ROTATE_90)
        elif orientation != 1:
            LOGGER.warning(f"Ignoring image orientation {orientation}.")

    img = np.array(img_pil)
    if img.ndim < 3 or img.shape[2] == 1:
        img = np.dstack((img, img, img))
    if remove_alpha:
        img = img[:, :, :3]

    f_35mm = img_exif.get("FocalLengthIn35mmFilm",
                          img_exif.get("FocalLenIn35mmFilm", img_exif.get("FocalLengthIn35mmFormat", None)))
    if f_35mm is not None and f_35mm > 0:
        f_px = fpx_from_f35(img.shape[1], img.shape[0], f_35mm)
    else:
        f_px = None
    return img, icc_profile, f_px
