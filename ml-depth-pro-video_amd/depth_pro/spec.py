"""Parameter inventory of the Depth Pro network (names and shapes).

The names are exactly the 1,119 state-dict keys that the reference model
(`src/depth_pro/depth_pro.py:72-151`, assembled from
`network/encoder.py:14-130`, `network/decoder.py:16-206`, `network/fov.py:11-54`
and the timm `vit_large_patch14_dinov2` backbone built by
`network/vit_factory.py:68-124`) exposes, so that a `depth_pro.pt`
checkpoint loads with `strict=True` (`depth_pro.py:134-149`).

Shapes are the post-resize shapes the checkpoint stores: patch-embed 16x16
(`vit.py:70-123`) and a 24x24+1 position table (`vit.py:51-67`).
"""

from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Tuple

# ViT-L/16 at 384^2 (VIT_CONFIG_DICT["dinov2l16_384"], vit_factory.py:53-65)
EMBED_DIM = 1024
DEPTH = 24
HEADS = 16
HEAD_DIM = 64
MLP_DIM = 4096
PATCH = 16
VIT_IMG = 384
GRID = VIT_IMG // PATCH            # 24
TOKENS = GRID * GRID + 1           # 577 (cls + 24x24)
HOOK_BLOCK_IDS = (5, 11, 17, 23)   # encoder_feature_layer_ids
DIMS_ENCODER = (256, 512, 1024, 1024)
DECODER_FEATURES = 256
IMG_SIZE = VIT_IMG * 4             # 1536 (encoder.py:146-149)
LN_EPS = 1e-6


def vit_spec(prefix: str) -> "OrderedDict[str, Tuple[int, ...]]":
    """timm VisionTransformer (dinov2, no reg tokens) parameter names."""
    s: "OrderedDict[str, Tuple[int, ...]]" = OrderedDict()
    d = EMBED_DIM
    s[f"{prefix}cls_token"] = (1, 1, d)
    s[f"{prefix}pos_embed"] = (1, TOKENS, d)
    s[f"{prefix}patch_embed.proj.weight"] = (d, 3, PATCH, PATCH)
    s[f"{prefix}patch_embed.proj.bias"] = (d,)
    for i in range(DEPTH):
        b = f"{prefix}blocks.{i}."
        s[b + "norm1.weight"] = (d,)
        s[b + "norm1.bias"] = (d,)
        s[b + "attn.qkv.weight"] = (3 * d, d)
        s[b + "attn.qkv.bias"] = (3 * d,)
        s[b + "attn.proj.weight"] = (d, d)
        s[b + "attn.proj.bias"] = (d,)
        s[b + "ls1.gamma"] = (d,)
        s[b + "norm2.weight"] = (d,)
        s[b + "norm2.bias"] = (d,)
        s[b + "mlp.fc1.weight"] = (MLP_DIM, d)
        s[b + "mlp.fc1.bias"] = (MLP_DIM,)
        s[b + "mlp.fc2.weight"] = (d, MLP_DIM)
        s[b + "mlp.fc2.bias"] = (d,)
        s[b + "ls2.gamma"] = (d,)
    s[f"{prefix}norm.weight"] = (d,)
    s[f"{prefix}norm.bias"] = (d,)
    return s


def param_spec(use_fov_head: bool = True) -> "OrderedDict[str, Tuple[int, ...]]":
    """All state-dict keys of `DepthPro` in registration order."""
    s: "OrderedDict[str, Tuple[int, ...]]" = OrderedDict()
    d = EMBED_DIM
    f = DECODER_FEATURES
    de = DIMS_ENCODER
    s.update(vit_spec("encoder.patch_encoder."))
    s.update(vit_spec("encoder.image_encoder."))
    # encoder.py:60-130 project/upsample blocks
    s["encoder.upsample_latent0.0.weight"] = (de[0], d, 1, 1)
    for i in range(1, 4):
        s[f"encoder.upsample_latent0.{i}.weight"] = (de[0] if i == 1 else f, f, 2, 2)
    s["encoder.upsample_latent1.0.weight"] = (de[0], d, 1, 1)
    for i in range(1, 3):
        s[f"encoder.upsample_latent1.{i}.weight"] = (de[0], de[0], 2, 2)
    for name, dim in (("upsample0", de[1]), ("upsample1", de[2]), ("upsample2", de[3])):
        s[f"encoder.{name}.0.weight"] = (dim, d, 1, 1)
        s[f"encoder.{name}.1.weight"] = (dim, dim, 2, 2)
    s["encoder.upsample_lowres.weight"] = (d, de[3], 2, 2)
    s["encoder.upsample_lowres.bias"] = (de[3],)
    s["encoder.fuse_lowres.weight"] = (de[3], 2 * de[3], 1, 1)
    s["encoder.fuse_lowres.bias"] = (de[3],)
    # decoder.py:16-93
    dec_dims = (f,) + de
    for i in range(1, 5):
        s[f"decoder.convs.{i}.weight"] = (f, dec_dims[i], 3, 3)
    for i in range(5):
        p = f"decoder.fusions.{i}."
        for r in ("resnet1", "resnet2"):
            for j in (1, 3):
                s[p + f"{r}.residual.{j}.weight"] = (f, f, 3, 3)
                s[p + f"{r}.residual.{j}.bias"] = (f,)
        if i != 0:
            s[p + "deconv.weight"] = (f, f, 2, 2)
        s[p + "out_conv.weight"] = (f, f, 1, 1)
        s[p + "out_conv.bias"] = (f,)
    # depth_pro.py:182-207 head
    s["head.0.weight"] = (f // 2, f, 3, 3)
    s["head.0.bias"] = (f // 2,)
    s["head.1.weight"] = (f // 2, f // 2, 2, 2)
    s["head.1.bias"] = (f // 2,)
    s["head.2.weight"] = (32, f // 2, 3, 3)
    s["head.2.bias"] = (32,)
    s["head.4.weight"] = (1, 32, 1, 1)
    s["head.4.bias"] = (1,)
    if use_fov_head:
        # fov.py:28-54
        s.update(vit_spec("fov.encoder.0."))
        s["fov.encoder.1.weight"] = (f // 2, d)
        s["fov.encoder.1.bias"] = (f // 2,)
        s["fov.downsample.0.weight"] = (f // 2, f, 3, 3)
        s["fov.downsample.0.bias"] = (f // 2,)
        s["fov.head.0.weight"] = (f // 4, f // 2, 3, 3)
        s["fov.head.0.bias"] = (f // 4,)
        s["fov.head.2.weight"] = (f // 8, f // 4, 3, 3)
        s["fov.head.2.bias"] = (f // 8,)
        s["fov.head.4.weight"] = (1, f // 8, 6, 6)
        s["fov.head.4.bias"] = (1,)
    return s


def num_params(spec: Dict[str, Tuple[int, ...]]) -> int:
    n = 0
    for shape in spec.values():
        c = 1
        for x in shape:
            c *= x
        n += c
    return n
