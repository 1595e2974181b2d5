"""depth_pro.cli (`depth-pro-run`, reference src/depth_pro/cli/run.py:33-150)."""

import io
import os

import numpy as np
import pytest

os.environ.setdefault("DEPTH_PRO_SYNTHETIC", "1")  # no checkpoint offline: synthetic weights


def test_entry_point_table():
    """pyproject.toml:15-16 of the reference: depth-pro-run = "depth_pro.cli:run_main"."""
    from depth_pro.cli import run_main
    from depth_pro.cli.run import main

    assert run_main is main
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = open(os.path.join(here, "ml-depth-pro-video_amd", "pyproject.toml")).read()
    assert 'depth-pro-run = "depth_pro.cli:run_main"' in text


def test_inverse_depth_view_matches_reference_formula():
    """cli/run.py:78-85: 1/depth normalised over [max(1/250, min), min(max, 1/0.1)]."""
    from depth_pro.cli.run import inverse_depth_view

    d = np.random.default_rng(0).random((40, 50)).astype(np.float32) * 300 + 0.05
    inv = 1 / d
    hi, lo = min(inv.max(), 1 / 0.1), max(1 / 250, inv.min())
    assert np.array_equal(inverse_depth_view(d), (inv - lo) / (hi - lo))


@pytest.mark.gpu
def test_depth_pro_run_on_a_directory(tmp_path, cuda):
    import torch
    from PIL import Image

    from depth_pro.cli.run import main, inverse_depth_view, turbo_u8

    src = tmp_path / "in"
    (src / "sub").mkdir(parents=True)
    rng = np.random.default_rng(9)
    imgs = {"a": rng.integers(0, 256, (300, 400, 3), dtype=np.uint8),
            "sub/b": rng.integers(0, 256, (256, 192, 3), dtype=np.uint8)}
    for k, v in imgs.items():
        Image.fromarray(v).save(src / f"{k}.png")
    (src / "notes.txt").write_text("not an image")       # logged and skipped, as in the reference
    out = tmp_path / "out"
    assert main(["-i", str(src), "-o", str(out), "--skip-display"]) is None    # exit status 0, like the reference
    import depth_pro

    model, transform = depth_pro.create_model_and_transforms(
        depth_pro.depth_pro.run_config(), device=cuda, precision=torch.half)
    for k, v in imgs.items():
        depth = np.load(out / f"{k}.npz")["depth"]
        assert depth.shape == v.shape[:2] and depth.dtype == np.float32
        ref = model.infer(transform(v))["depth"].cpu().numpy()
        assert np.array_equal(depth, ref)                    # same f16 engine, same frame
        jpg = Image.open(out / f"{k}.jpg")
        assert jpg.size == (v.shape[1], v.shape[0]) and jpg.mode == "RGB"
        # the reference's encoding of the same colour map (cli/run.py:97-106), through the same libjpeg
        buf = io.BytesIO()
        Image.fromarray(turbo_u8(inverse_depth_view(depth))).save(buf, format="JPEG", quality=90)
        assert np.array_equal(np.asarray(jpg), np.asarray(Image.open(buf)))


def test_console_script_exit_status(tmp_path):
    """The console script runs `sys.exit(run_main())`: a successful run must exit 0 (main returns
    None), whatever the number of images; `run` keeps the count for callers."""
    import subprocess
    import sys

    from depth_pro.cli import run as R

    calls = []
    orig = R.run
    try:
        R.run = lambda args: calls.append(args) or 2
        assert R.main(["-i", str(tmp_path), "--skip-display"]) is None
    finally:
        R.run = orig
    assert len(calls) == 1 and calls[0].skip_display
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = os.path.join(here, "ml-depth-pro-video_amd")
    code = ("import sys; from depth_pro.cli import run as R; R.run = lambda a: 3; "
            "from depth_pro.cli import run_main; sys.exit(run_main(['--skip-display']))")
    r = subprocess.run([sys.executable, "-c", code], cwd=pkg, env={**os.environ, "PYTHONPATH": pkg})
    assert r.returncode == 0
