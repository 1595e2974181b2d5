"""Depth Pro CLI (reference `src/depth_pro/cli/__init__.py`): the `depth-pro-run` entry point
(`pyproject.toml:15-16`: depth-pro-run = "depth_pro.cli:run_main")."""

from .run import main as run_main  # noqa: F401
