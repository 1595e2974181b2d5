#!/usr/bin/env python3
"""`depth-pro-run`: Depth Pro on one image or a directory tree (reference `cli/run.py:33-150`).

Same flags (-i/--image-path, -o/--output-path, --skip-display, -v/--verbose), same model
precision (the reference builds the model with precision=torch.half: f16 throughout on the
MI355X engine), same outputs per image: `<out>/<relative dir>/<stem>.npz` holding `depth`
(np.savez_compressed) and `<stem>.jpg`, the turbo colour map of inverse depth clipped to
[0.1 m, 250 m] (JPEG quality 90).  Unreadable files are logged and skipped, as in the
reference.  The model runs its forward as one replayed HIP graph (the shapes are static).

Without ./checkpoints/depth_pro.pt, DEPTH_PRO_SYNTHETIC=1 substitutes the synthetic weight
set (depth_pro.weights); otherwise a missing checkpoint raises like the reference.
"""

from __future__ import annotations

import argparse
import logging
from pathlib import Path
from typing import Iterable, Tuple

import numpy as np
import PIL.Image
import torch

from ..depth_pro import create_model_and_transforms, run_config
from ..utils import load_rgb

LOGGER = logging.getLogger(__name__)
VIZ_NEAR_M, VIZ_FAR_M = 0.1, 250.0


def get_torch_device() -> torch.device:
    """The ROCm device (reference :23-30 falls back to mps/cpu; this engine has no host path)."""
    if torch.cuda.is_available():
        return torch.device("cuda:0")
    raise RuntimeError("depth-pro-run on the MI355X engine needs a ROCm GPU")


def inverse_depth_view(depth: np.ndarray) -> np.ndarray:
    """Inverse depth normalised over its range clipped to [1/250 m, 1/0.1 m] (reference :78-85)."""
    inv = 1 / depth
    hi = min(inv.max(), 1 / VIZ_NEAR_M)
    lo = max(1 / VIZ_FAR_M, inv.min())
    return (inv - lo) / (hi - lo)


def turbo_u8(x: np.ndarray) -> np.ndarray:
    from matplotlib import pyplot as plt

    return (plt.get_cmap("turbo")(x)[..., :3] * 255).astype(np.uint8)


def _inputs(image_path: Path) -> Tuple[Iterable[Path], Path]:
    if image_path.is_dir():
        return image_path.glob("**/*"), image_path
    return [image_path], image_path.parent


def run(args) -> int:
    """Predict every image; returns how many were written (or displayed)."""
    if args.verbose:
        logging.basicConfig(level=logging.INFO)
    model, transform = create_model_and_transforms(run_config(), device=get_torch_device(), precision=torch.half)
    model.eval()
    model.use_hip_graph(True)

    paths, root = _inputs(Path(args.image_path))
    show = not args.skip_display
    if show:
        from matplotlib import pyplot as plt

        plt.ion()
        fig = plt.figure()
        ax_rgb, ax_disp = fig.add_subplot(121), fig.add_subplot(122)
    done = 0
    for image_path in paths:
        try:
            LOGGER.info(f"Loading image {image_path} ...")
            image, _, f_px = load_rgb(image_path)
        except Exception as e:  # directories, non-images: skipped (reference :60-65)
            LOGGER.error(str(e))
            continue
        pred = model.infer(transform(image), f_px=f_px)
        depth = pred["depth"].detach().cpu().numpy().squeeze()
        try:
            model.last_status().check()     # this frame's health, before anything is written
        except Exception as e:
            LOGGER.error(f"{image_path}: {e}")
            continue
        if f_px is not None:
            LOGGER.debug(f"Focal length (from exif): {f_px:0.2f}")
        elif pred["focallength_px"] is not None:
            LOGGER.info(f"Estimated focal length: {pred['focallength_px'].detach().cpu().item()}")
        view = inverse_depth_view(depth)
        if args.output_path is not None:
            stem = Path(args.output_path) / image_path.relative_to(root).parent / image_path.stem
            stem.parent.mkdir(parents=True, exist_ok=True)
            LOGGER.info(f"Saving depth map to: {stem}")
            np.savez_compressed(stem, depth=depth)
            PIL.Image.fromarray(turbo_u8(view)).save(str(stem) + ".jpg", format="JPEG", quality=90)
        if show:
            ax_rgb.imshow(image)
            ax_disp.imshow(view, cmap="turbo")
            fig.canvas.draw()
            fig.canvas.flush_events()
        done += 1
    LOGGER.info("Done predicting depth!")
    if show:
        plt.show(block=True)
    return done


def main(argv=None) -> None:
    """`depth-pro-run` (reference :120-150).  Returns None like the reference's main, so the console
    script (`sys.exit(run_main())`) exits 0 on success; `run` returns the image count."""
    parser = argparse.ArgumentParser(description="Inference scripts of DepthPro with PyTorch models.")
    parser.add_argument("-i", "--image-path", type=Path, default="./data/example.jpg", help="Path to input image.")
    parser.add_argument("-o", "--output-path", type=Path, help="Path to store output files.")
    parser.add_argument("--skip-display", action="store_true", help="Skip matplotlib display.")
    parser.add_argument("-v", "--verbose", action="store_true", help="Show verbose output.")
    run(parser.parse_args(argv))


if __name__ == "__main__":
    main()
