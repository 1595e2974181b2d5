"""CPU fp32 restatement of the Depth Pro hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity oracle.  Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import it; the product package
(`ml-depth-pro-video_amd/depth_pro`) never does, and it must fail loudly when
its HIP library is missing instead of falling back to this file.

It restates, as plain functional PyTorch on fp32 CPU tensors, what the
reference computes for `DepthPro.infer` (`src/depth_pro/depth_pro.py:243-298`):

* the timm `vit_large_patch14_dinov2` forward_features the reference binds
  (`network/vit_factory.py:97-110`, `network/vit.py:13-35`) -- third-party
  timm (unpinned, `pyproject.toml:9`, absent here); its published algorithm is
  restated in `vit_forward` and cross-checked against `transformers`'
  independent Dinov2Layer in `tests/golden/make_golden.py`;
* `DepthProEncoder.forward` (`network/encoder.py:151-332`);
* `MultiresConvDecoder.forward` + `FeatureFusionBlock2d` (`network/decoder.py:74-206`);
* the depth head (`depth_pro.py:182-207`) and `FOVNetwork.forward` (`network/fov.py:56-82`);
* the `infer` prologue/epilogue (`depth_pro.py:268-298`).

Parity pin: `tests/golden/golden_*.npz`, produced by running the reference's own
modules (imported from /root/reference in the survey container, with a timm
stand-in) on the synthetic weights of `depth_pro.weights`; see
`tests/golden/make_golden.py` and `tests/test_oracle_golden.py`.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

EMBED = 1024
HEADS = 16
GRID = 24
LN_EPS = 1e-6
IMG = 1536


# ----------------------------------------------------------------------------- ViT
def vit_block(sd: Dict[str, torch.Tensor], p: str, x: torch.Tensor) -> torch.Tensor:
    """timm `Block.forward`: x += ls1(attn(norm1 x)); x += ls2(mlp(norm2 x))."""
    B, N, C = x.shape
    h = F.layer_norm(x, (C,), sd[p + "norm1.weight"], sd[p + "norm1.bias"], LN_EPS)
    qkv = F.linear(h, sd[p + "attn.qkv.weight"], sd[p + "attn.qkv.bias"])
    qkv = qkv.reshape(B, N, 3, HEADS, C // HEADS).permute(2, 0, 3, 1, 4)
    q, k, v = qkv.unbind(0)
    a = F.scaled_dot_product_attention(q, k, v)  # scale = head_dim ** -0.5
    a = a.transpose(1, 2).reshape(B, N, C)
    a = F.linear(a, sd[p + "attn.proj.weight"], sd[p + "attn.proj.bias"])
    x = x + sd[p + "ls1.gamma"] * a
    h = F.layer_norm(x, (C,), sd[p + "norm2.weight"], sd[p + "norm2.bias"], LN_EPS)
    h = F.linear(h, sd[p + "mlp.fc1.weight"], sd[p + "mlp.fc1.bias"])
    h = F.gelu(h)  # exact erf GELU (timm default act_layer nn.GELU)
    h = F.linear(h, sd[p + "mlp.fc2.weight"], sd[p + "mlp.fc2.bias"])
    return x + sd[p + "ls2.gamma"] * h


def vit_embed(sd: Dict[str, torch.Tensor], p: str, img: torch.Tensor) -> torch.Tensor:
    """patch_embed (k16 s16 conv, NHWC) + cls prefix + pos_embed (timm `_pos_embed`)."""
    B = img.shape[0]
    t = F.conv2d(img, sd[p + "patch_embed.proj.weight"], sd[p + "patch_embed.proj.bias"], stride=16)
    t = t.flatten(2).transpose(1, 2)  # (B, 576, C)
    cls = sd[p + "cls_token"].expand(B, -1, -1)
    return torch.cat((cls, t), dim=1) + sd[p + "pos_embed"]


def vit_forward(
    sd: Dict[str, torch.Tensor], p: str, img: torch.Tensor, hooks: Sequence[int] = ()
) -> Tuple[torch.Tensor, Dict[int, torch.Tensor]]:
    """forward_features (vit.py:33) returning final-norm tokens and hooked block outputs."""
    x = vit_embed(sd, p, img)
    saved = {}
    for i in range(24):
        x = vit_block(sd, f"{p}blocks.{i}.", x)
        if i in hooks:
            saved[i] = x
    x = F.layer_norm(x, (EMBED,), sd[p + "norm.weight"], sd[p + "norm.bias"], LN_EPS)
    return x, saved


# ------------------------------------------------------------------------- encoder
def pyramid(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """encoder.py:151-168 (bilinear, align_corners=False, scale_factor path)."""
    x1 = F.interpolate(x, scale_factor=0.5, mode="bilinear", align_corners=False)
    x2 = F.interpolate(x, scale_factor=0.25, mode="bilinear", align_corners=False)
    return x, x1, x2


def split(x: torch.Tensor, overlap_ratio: float) -> torch.Tensor:
    """encoder.py:170-188: 384^2 windows, row-major (j outer, i inner)."""
    size = 384
    stride = int(size * (1 - overlap_ratio))
    steps = int(math.ceil((x.shape[-1] - size) / stride)) + 1
    out = []
    for j in range(steps):
        for i in range(steps):
            out.append(x[..., j * stride:j * stride + size, i * stride:i * stride + size])
    return torch.cat(out, dim=0)


def merge(x: torch.Tensor, batch: int, padding: int) -> torch.Tensor:
    """encoder.py:190-217: stitch steps x steps NCHW windows, cropping `padding`."""
    steps = int(math.sqrt(x.shape[0] // batch))
    rows = []
    idx = 0
    for j in range(steps):
        cols = []
        for i in range(steps):
            o = x[batch * idx: batch * (idx + 1)]
            y0 = padding if j != 0 else 0
            y1 = o.shape[-2] - (padding if j != steps - 1 else 0)
            x0 = padding if i != 0 else 0
            x1 = o.shape[-1] - (padding if i != steps - 1 else 0)
            cols.append(o[..., y0:y1, x0:x1])
            idx += 1
        rows.append(torch.cat(cols, dim=-1))
    return torch.cat(rows, dim=-2)


def tokens_to_nchw(t: torch.Tensor) -> torch.Tensor:
    """encoder.py:219-231 reshape_feature: drop cls, (B,576,C) -> (B,C,24,24)."""
    b, _, c = t.shape
    return t[:, 1:, :].reshape(b, GRID, GRID, c).permute(0, 3, 1, 2)


def project_upsample(sd, p: str, x: torch.Tensor, n_up: int) -> torch.Tensor:
    """encoder.py:60-88: 1x1 conv (no bias) then n_up k2s2 ConvTranspose (no bias)."""
    x = F.conv2d(x, sd[p + "0.weight"])
    for i in range(1, n_up + 1):
        x = F.conv_transpose2d(x, sd[p + f"{i}.weight"], stride=2)
    return x


def encoder_forward(sd, x: torch.Tensor) -> List[torch.Tensor]:
    """DepthProEncoder.forward (encoder.py:233-332)."""
    B = x.shape[0]
    x0, x1, x2 = pyramid(x)
    p0 = split(x0, 0.25)
    p1 = split(x1, 0.5)
    patches = torch.cat((p0, p1, x2), dim=0)
    enc, hooks = vit_forward(sd, "encoder.patch_encoder.", patches, hooks=(5, 11))
    enc = tokens_to_nchw(enc)
    lat0 = merge(tokens_to_nchw(hooks[5])[: B * 25], B, 3)
    lat1 = merge(tokens_to_nchw(hooks[11])[: B * 25], B, 3)
    e0, e1, e2 = torch.split(enc, [len(p0), len(p1), len(x2)], dim=0)
    f0 = merge(e0, B, 3)
    f1 = merge(e1, B, 6)
    f2 = e2
    g, _ = vit_forward(sd, "encoder.image_encoder.", x2)
    g = tokens_to_nchw(g)
    lat0 = project_upsample(sd, "encoder.upsample_latent0.", lat0, 3)
    lat1 = project_upsample(sd, "encoder.upsample_latent1.", lat1, 2)
    f0 = project_upsample(sd, "encoder.upsample0.", f0, 1)
    f1 = project_upsample(sd, "encoder.upsample1.", f1, 1)
    f2 = project_upsample(sd, "encoder.upsample2.", f2, 1)
    g = F.conv_transpose2d(g, sd["encoder.upsample_lowres.weight"], sd["encoder.upsample_lowres.bias"], stride=2)
    g = F.conv2d(torch.cat((f2, g), dim=1), sd["encoder.fuse_lowres.weight"], sd["encoder.fuse_lowres.bias"])
    return [lat0, lat1, f0, f1, g]


# ------------------------------------------------------------------------- decoder
def residual_block(sd, p: str, x: torch.Tensor) -> torch.Tensor:
    """decoder.py:96-118,186-206: x + conv(relu(conv(relu(x)))) (3x3, bias)."""
    h = F.conv2d(F.relu(x), sd[p + "residual.1.weight"], sd[p + "residual.1.bias"], padding=1)
    h = F.conv2d(F.relu(h), sd[p + "residual.3.weight"], sd[p + "residual.3.bias"], padding=1)
    return x + h


def fusion_block(sd, i: int, x0: torch.Tensor, x1: Optional[torch.Tensor]) -> torch.Tensor:
    """FeatureFusionBlock2d.forward (decoder.py:169-184)."""
    p = f"decoder.fusions.{i}."
    x = x0
    if x1 is not None:
        x = x + residual_block(sd, p + "resnet1.", x1)
    x = residual_block(sd, p + "resnet2.", x)
    if i != 0:
        x = F.conv_transpose2d(x, sd[p + "deconv.weight"], stride=2)
    return F.conv2d(x, sd[p + "out_conv.weight"], sd[p + "out_conv.bias"])


def decoder_forward(sd, enc: List[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
    """MultiresConvDecoder.forward (decoder.py:74-93)."""
    feats = F.conv2d(enc[4], sd["decoder.convs.4.weight"], padding=1)
    low = feats
    feats = fusion_block(sd, 4, feats, None)
    for i in range(3, -1, -1):
        fi = enc[i] if i == 0 else F.conv2d(enc[i], sd[f"decoder.convs.{i}.weight"], padding=1)
        feats = fusion_block(sd, i, feats, fi)
    return feats, low


def head_forward(sd, feats: torch.Tensor) -> torch.Tensor:
    """depth_pro.py:182-207."""
    x = F.conv2d(feats, sd["head.0.weight"], sd["head.0.bias"], padding=1)
    x = F.conv_transpose2d(x, sd["head.1.weight"], sd["head.1.bias"], stride=2)
    x = F.relu(F.conv2d(x, sd["head.2.weight"], sd["head.2.bias"], padding=1))
    return F.relu(F.conv2d(x, sd["head.4.weight"], sd["head.4.bias"]))


def fov_forward(sd, x: torch.Tensor, low: torch.Tensor) -> torch.Tensor:
    """FOVNetwork.forward (fov.py:56-82) with the fov encoder present."""
    x = F.interpolate(x, scale_factor=0.25, mode="bilinear", align_corners=False)
    t, _ = vit_forward(sd, "fov.encoder.0.", x)
    t = F.linear(t, sd["fov.encoder.1.weight"], sd["fov.encoder.1.bias"])
    t = t[:, 1:].permute(0, 2, 1)
    d = F.relu(F.conv2d(low, sd["fov.downsample.0.weight"], sd["fov.downsample.0.bias"], stride=2, padding=1))
    x = t.reshape_as(d) + d
    x = F.relu(F.conv2d(x, sd["fov.head.0.weight"], sd["fov.head.0.bias"], stride=2, padding=1))
    x = F.relu(F.conv2d(x, sd["fov.head.2.weight"], sd["fov.head.2.bias"], stride=2, padding=1))
    return F.conv2d(x, sd["fov.head.4.weight"], sd["fov.head.4.bias"])


def forward(sd, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """DepthPro.forward (depth_pro.py:218-241)."""
    assert x.shape[-2] == IMG and x.shape[-1] == IMG
    enc = encoder_forward(sd, x)
    feats, low = decoder_forward(sd, enc)
    canonical = head_forward(sd, feats)
    fov_deg = fov_forward(sd, x, low)
    return canonical, fov_deg


def infer(sd, x: torch.Tensor, f_px=None) -> Dict[str, torch.Tensor]:
    """DepthPro.infer (depth_pro.py:243-298), bilinear interpolation mode."""
    if x.dim() == 3:
        x = x.unsqueeze(0)
    _, _, H, W = x.shape
    resize = H != IMG or W != IMG
    if resize:
        x = F.interpolate(x, size=(IMG, IMG), mode="bilinear", align_corners=False)
    canonical, fov_deg = forward(sd, x)
    if f_px is None:
        f_px = 0.5 * W / torch.tan(0.5 * torch.deg2rad(fov_deg.to(torch.float)))
    inv = canonical * (W / f_px)
    f_px = f_px.squeeze()
    if resize:
        inv = F.interpolate(inv, size=(H, W), mode="bilinear", align_corners=False)
    depth = 1.0 / torch.clamp(inv, min=1e-4, max=1e4)
    return {"depth": depth.squeeze(), "focallength_px": f_px}


def transform(img_u8) -> torch.Tensor:
    """depth_pro.py:125-132 Compose: ToTensor, Normalize(.5,.5), fp32."""
    t = torch.from_numpy(img_u8).permute(2, 0, 1).contiguous().to(torch.float32).div(255.0)
    return (t - 0.5) / 0.5


# --------------------------------------------------------------- point cloud
def depth_to_3d(depth_in, focallength_px, width, height):
    """Reference `depth_to_3d` (img_to_normalized_pointcloud.py:819-856), restated in numpy
    (that module imports open3d / cv2 at the top, so it cannot be imported here).
    Returns (points_3d (N, 3) float64, valid_mask (height, width) bool)."""
    import numpy as np

    depth_np = np.asarray(depth_in)
    y_indices, x_indices = np.indices((height, width))
    cx = width / 2
    cy = height / 2
    valid_mask = ~np.isnan(depth_np) & (depth_np > 0)
    z = depth_np[valid_mask].flatten()
    x = -1 * (x_indices[valid_mask] - cx) * z / focallength_px
    y = -1 * (y_indices[valid_mask] - cy) * z / focallength_px
    return np.column_stack((x, y, z)), valid_mask
