"""Deterministic synthetic Depth Pro weights.

`depth_pro.pt` (`get_pretrained_models.sh:8`) cannot be downloaded offline, so
benches, parity tests and golden fixtures all run on a synthetic state dict
whose every tensor is a pure function of (seed, key, shape): a CPU
`torch.Generator` seeded from crc32(key) ^ seed draws it, so the same tensor
comes out in this container and on any GPU box.

Scales are chosen so the network stays in its working range:
fan-in scaled Gaussian weights, LayerScale gammas around 0.1, a positive
depth-head tail (canonical inverse depth > 0, so `infer`'s clamp at
`depth_pro.py:293` does not saturate) and an FOV head centred at 60 deg.
"""

from __future__ import annotations

import zlib
from collections import OrderedDict
from typing import Dict

import torch

from .spec import param_spec


def _gen(seed: int, key: str) -> torch.Generator:
    g = torch.Generator(device="cpu")
    g.manual_seed((zlib.crc32(key.encode()) ^ (seed * 0x9E3779B1)) & 0x7FFFFFFFFFFF)
    return g


def synthetic_tensor(key: str, shape, seed: int = 0) -> torch.Tensor:
    g = _gen(seed, key)
    n = lambda: torch.randn(shape, generator=g, dtype=torch.float32)  # noqa: E731
    leaf = key.rsplit(".", 1)[-1]
    if key.endswith("cls_token"):
        return 0.02 * n()
    if key.endswith("pos_embed"):
        return 0.02 * n()
    if leaf == "gamma":  # LayerScale
        return 0.1 + 0.02 * n()
    if ".norm" in key and leaf in ("weight", "bias"):  # LayerNorm
        return (1.0 + 0.1 * n()) if leaf == "weight" else 0.02 * n()
    if key == "head.4.weight":
        return n().abs() * (1.0 / 32.0) + 0.01
    if key == "head.4.bias":
        return torch.full(shape, 0.5)
    if key == "fov.head.4.bias":
        return torch.full(shape, 60.0)
    if key == "fov.head.4.weight":
        return n() * (4.0 / (32 * 36) ** 0.5)
    if leaf == "bias":
        return 0.02 * n()
    if leaf == "weight":
        if len(shape) == 2:  # Linear [out, in]
            fan_in = shape[1]
        elif ".upsample" in key and ".0." not in key or "deconv" in key or key in (
            "head.1.weight",
        ):  # ConvTranspose2d [in, out, kh, kw]: each output sums `in` inputs
            fan_in = shape[0]
        else:  # Conv2d [out, in, kh, kw]
            fan_in = shape[1] * shape[2] * shape[3]
        return n() * (1.0 / fan_in) ** 0.5
    raise KeyError(f"no synthetic rule for {key}")


def synthetic_state_dict(seed: int = 0, use_fov_head: bool = True) -> Dict[str, torch.Tensor]:
    """The full synthetic fp32 state dict (1,119 keys, 951,991,330 params)."""
    sd: Dict[str, torch.Tensor] = OrderedDict()
    for key, shape in param_spec(use_fov_head).items():
        sd[key] = synthetic_tensor(key, shape, seed)
    return sd


# Stress set (parity margin outside the benign synthetic distribution): real
# DINOv2 checkpoints carry LayerScale gammas well above 0.1 and a few residual-stream channels
# with very large activations.  Same tensors as `synthetic_state_dict`, except every LayerScale
# gamma x STRESS_LS, and in every ViT block the fc2 bias of STRESS_CHANNELS raised by
# STRESS_BIAS (the outliers then grow block by block through the residual stream).
STRESS_LS = 5.0
STRESS_CHANNELS = (7, 300, 901)
STRESS_BIAS = 20.0


def stressed_state_dict(seed: int = 0, use_fov_head: bool = True) -> Dict[str, torch.Tensor]:
    sd = synthetic_state_dict(seed, use_fov_head)
    for k, v in sd.items():
        if k.endswith(".gamma"):
            sd[k] = v * STRESS_LS
        elif k.endswith("mlp.fc2.bias"):
            v = v.clone()
            v[list(STRESS_CHANNELS)] += STRESS_BIAS
            sd[k] = v
    return sd
