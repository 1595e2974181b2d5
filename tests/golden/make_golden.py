"""Generate the golden fixtures by running the REFERENCE Depth Pro modules.

Run in the survey/build container only (it needs /root/reference, which does
not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py            # all fixtures
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py --stages   # golden_stages_frame0.npz only
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py --io       # load_rgb + 4K infer fixtures
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py --stress   # golden_stress_frame0.npz (stressed weights)

What it does
------------
The reference package `depth_pro` (/root/reference/src) is imported as-is.  Its
third-party imports that are absent from this image are replaced by stand-ins
written here (none of them is reference code):

* `torchvision.transforms` -- the five transform classes `depth_pro.py:12-18`
  imports, restated from torchvision's published semantics;
* `pillow_heif` -- `register_heif_opener` no-op (`utils.py:8-12`);
* `timm` -- `create_model("vit_large_patch14_dinov2", dynamic_img_size=True)`
  returning a timm-compatible VisionTransformer (same module tree and
  parameter names: `vit_factory.py:97-99` binds it), and
  `timm.layers.resample_abs_pos_embed` (`vit.py:5`).  Its Block is
  cross-checked here against `transformers`' independent `Dinov2Layer`.

Everything else -- `create_model_and_transforms`, `DepthProEncoder` (pyramid,
split, hooks, merge, upsample/fuse), `MultiresConvDecoder`, the head,
`FOVNetwork`, `DepthPro.infer`, `load_rgb` -- is the reference's own code.
The synthetic weights come from `depth_pro.weights.synthetic_state_dict(0)`
(this repo) and are loaded into the reference model with `strict=True`.

Outputs: tests/golden/golden_*.npz (small: sub-sampled maps + statistics).
"""

from __future__ import annotations

import json
import math
import os
import sys
import time
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SRC = "/root/reference/src"
REF_DATA = "/root/reference/data"


# ---------------------------------------------------------------- stand-ins
def install_torchvision_stub():
    tv = types.ModuleType("torchvision")
    tr = types.ModuleType("torchvision.transforms")

    class Compose:
        def __init__(self, ts):
            self.transforms = ts

        def __call__(self, x):
            for t in self.transforms:
                x = t(x)
            return x

    class ToTensor:
        def __call__(self, pic):
            a = np.asarray(pic)
            if a.ndim == 2:
                a = a[:, :, None]
            t = torch.from_numpy(a.transpose((2, 0, 1))).contiguous()
            return t.to(torch.float32).div(255) if t.dtype == torch.uint8 else t

    class Lambda:
        def __init__(self, f):
            self.f = f

        def __call__(self, x):
            return self.f(x)

    class Normalize:
        def __init__(self, mean, std):
            self.mean, self.std = mean, std

        def __call__(self, t):
            m = torch.as_tensor(self.mean, dtype=t.dtype).view(-1, 1, 1)
            s = torch.as_tensor(self.std, dtype=t.dtype).view(-1, 1, 1)
            return (t - m) / s

    class ConvertImageDtype:
        def __init__(self, dtype):
            self.dtype = dtype

        def __call__(self, t):
            return t.to(self.dtype)

    for c in (Compose, ToTensor, Lambda, Normalize, ConvertImageDtype):
        setattr(tr, c.__name__, c)
    tv.transforms = tr
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.transforms"] = tr


def install_heif_stub():
    ph = types.ModuleType("pillow_heif")
    ph.register_heif_opener = lambda: None

    def open_heif(*a, **k):
        raise RuntimeError("HEIF not supported in the fixture container")

    ph.open_heif = open_heif
    sys.modules["pillow_heif"] = ph


class _LayerScale(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.gamma = nn.Parameter(1e-5 * torch.ones(d))

    def forward(self, x):
        return x * self.gamma


class _Attention(nn.Module):
    def __init__(self, d, heads):
        super().__init__()
        self.num_heads = heads
        self.qkv = nn.Linear(d, 3 * d, bias=True)
        self.proj = nn.Linear(d, d)

    def forward(self, x):
        B, N, C = x.shape
        qkv = self.qkv(x).reshape(B, N, 3, self.num_heads, C // self.num_heads).permute(2, 0, 3, 1, 4)
        q, k, v = qkv.unbind(0)
        x = F.scaled_dot_product_attention(q, k, v)
        return self.proj(x.transpose(1, 2).reshape(B, N, C))


class _Mlp(nn.Module):
    def __init__(self, d, h):
        super().__init__()
        self.fc1 = nn.Linear(d, h)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(h, d)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))


class _Block(nn.Module):
    def __init__(self, d, heads):
        super().__init__()
        self.norm1 = nn.LayerNorm(d, eps=1e-6)
        self.attn = _Attention(d, heads)
        self.ls1 = _LayerScale(d)
        self.norm2 = nn.LayerNorm(d, eps=1e-6)
        self.mlp = _Mlp(d, 4 * d)
        self.ls2 = _LayerScale(d)

    def forward(self, x):
        x = x + self.ls1(self.attn(self.norm1(x)))
        return x + self.ls2(self.mlp(self.norm2(x)))


class _PatchEmbed(nn.Module):
    def __init__(self, img, patch, d):
        super().__init__()
        self.img_size = (img, img)
        self.patch_size = (patch, patch)
        self.grid_size = (img // patch, img // patch)
        self.proj = nn.Conv2d(3, d, kernel_size=patch, stride=patch)

    def forward(self, x):
        return self.proj(x).permute(0, 2, 3, 1)  # NHWC (dynamic_img_size)


def resample_abs_pos_embed(posemb, new_size, num_prefix_tokens=1, **kw):
    n_old = posemb.shape[1] - num_prefix_tokens
    old = int(math.sqrt(n_old))
    if old == new_size[0] and old == new_size[1]:
        return posemb
    prefix, grid = posemb[:, :num_prefix_tokens], posemb[:, num_prefix_tokens:]
    grid = grid.reshape(1, old, old, -1).permute(0, 3, 1, 2)
    grid = F.interpolate(grid, size=new_size, mode="bicubic", antialias=True, align_corners=False)
    grid = grid.permute(0, 2, 3, 1).reshape(1, -1, posemb.shape[-1])
    return torch.cat([prefix, grid], dim=1)


class TimmViTStandIn(nn.Module):
    """timm VisionTransformer('vit_large_patch14_dinov2', dynamic_img_size=True)."""

    def __init__(self):
        super().__init__()
        d = 1024
        self.embed_dim = d
        self.num_prefix_tokens = 1
        self.no_embed_class = False
        self.patch_embed = _PatchEmbed(518, 14, d)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, d))
        self.pos_embed = nn.Parameter(torch.zeros(1, 1 + 37 * 37, d))
        self.blocks = nn.Sequential(*[_Block(d, 16) for _ in range(24)])
        self.norm = nn.LayerNorm(d, eps=1e-6)
        self.grad_checkpointing = False

    def set_grad_checkpointing(self, enable=True):
        self.grad_checkpointing = enable

    def _pos_embed(self, x):
        B, H, W, C = x.shape
        pos = resample_abs_pos_embed(self.pos_embed, (H, W), num_prefix_tokens=1)
        x = x.reshape(B, -1, C)
        x = torch.cat([self.cls_token.expand(B, -1, -1), x], dim=1)
        return x + pos

    def forward_features(self, x):
        x = self.patch_embed(x)
        x = self._pos_embed(x)
        for blk in self.blocks:
            x = blk(x)
        return self.norm(x)

    def forward(self, x):
        return self.forward_features(x)


def install_timm_stub():
    timm = types.ModuleType("timm")
    layers = types.ModuleType("timm.layers")

    def create_model(name, pretrained=False, dynamic_img_size=False, **kw):
        assert name == "vit_large_patch14_dinov2" and not pretrained
        return TimmViTStandIn()

    timm.create_model = create_model
    layers.resample_abs_pos_embed = resample_abs_pos_embed
    timm.layers = layers
    sys.modules["timm"] = timm
    sys.modules["timm.layers"] = layers


def import_reference():
    install_torchvision_stub()
    install_heif_stub()
    install_timm_stub()
    sys.path.insert(0, REF_SRC)
    import depth_pro as ref  # noqa: the REFERENCE package

    assert os.path.realpath(ref.__file__).startswith(REF_SRC), ref.__file__
    return ref


# ---------------------------------------------------------------- helpers
def frame(seed: int, h: int = 1536, w: int = 1536) -> np.ndarray:
    """SURVEY 8d synthetic frame k."""
    return np.random.default_rng(seed=seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def stats(t: torch.Tensor) -> np.ndarray:
    t = t.detach().double()
    return np.array([t.mean().item(), t.std().item(), t.abs().mean().item(), t.min().item(), t.max().item()])


def sub(t: torch.Tensor, s: int) -> np.ndarray:
    return t[..., ::s, ::s].detach().float().numpy().copy()


def stages(model, transform, t0):
    """Per-stage intermediates of the reference forward on synthetic frame 0, for localising
    a precision error stage by stage (tests/test_gpu_model.py::test_stage_parity).

    Forward hooks on the reference modules (no reference code changed): the three ViT outputs
    (final-norm tokens), the five encodings, the decoder's low-res projection, every fusion
    block's output and the canonical inverse depth -- each sub-sampled to a small grid.
    """
    caps = {}

    def keep(name):
        def hook(mod, inp, out):
            caps[name] = (out[0] if isinstance(out, tuple) else out).detach()
        return hook

    enc = model.encoder
    hs = [enc.patch_encoder.register_forward_hook(keep("vit_patch")),
          enc.image_encoder.register_forward_hook(keep("vit_image")),
          model.fov.encoder[0].register_forward_hook(keep("vit_fov")),
          model.decoder.convs[4].register_forward_hook(keep("lowres"))]
    for i in range(5):
        hs.append(model.decoder.fusions[i].register_forward_hook(keep(f"fusion{i}")))
    enc_fwd = enc.forward

    def enc_capture(x):
        out = enc_fwd(x)
        for i, o in enumerate(out):
            caps[f"enc{i}"] = o.detach()
        return out

    enc.forward = enc_capture
    with torch.no_grad():
        canonical, fov_deg = model.forward(transform(frame(0)).unsqueeze(0))
    enc.forward = enc_fwd
    for h in hs:
        h.remove()
    out = {"frame_seed": 0, "fov_deg": fov_deg.numpy().reshape(-1)}
    # ViT tokens [n, 577, 1024]: every 16th token of windows 0, 12, 34 (patch) / the image, every 4th channel
    out["vit_patch"] = caps["vit_patch"][[0, 12, 34], ::16, ::4].numpy().copy()
    out["vit_image"] = caps["vit_image"][0, ::16, ::4].numpy().copy()
    out["vit_fov"] = caps["vit_fov"][0, ::16, ::4].numpy().copy()
    # NCHW maps, sub-sampled to <= 24 x 24 spatially, every 4th channel
    for k, t in caps.items():
        if k.startswith("vit"):
            continue
        s = max(1, t.shape[-1] // 24)
        out[k] = t[0, ::4, ::s, ::s].numpy().copy()
    out["canonical_sub8"] = sub(canonical[0, 0], 8)
    np.savez_compressed(os.path.join(HERE, "golden_stages_frame0.npz"), **out)
    print(f"[golden] stages done ({time.time()-t0:.1f}s): " + ", ".join(f"{k}{list(np.shape(v))}" for k, v in out.items()))


def io_images():
    """Small synthetic images covering every branch of the reference load_rgb (utils.py:47-112):
    EXIF orientations 1/3/6/8 and an ignored one (5), the three 35 mm focal-length tag names
    (only the first is in PIL's EXIF table), a zero focal length, grey / palette / RGBA inputs."""
    import io as _io

    from PIL import Image

    rng = np.random.default_rng(21)
    out = {}

    def jpeg(name, orient=None, f35=None, size=(48, 64)):
        im = Image.fromarray(rng.integers(0, 256, size + (3,), dtype=np.uint8))
        ex = Image.Exif()
        if orient is not None:
            ex[0x0112] = orient
        if f35 is not None:
            ex.get_ifd(0x8769)[0xA405] = f35
        b = _io.BytesIO()
        im.save(b, "JPEG", exif=ex, quality=95)
        out[name] = b.getvalue()

    def png(name, arr, mode=None):
        b = _io.BytesIO()
        Image.fromarray(arr, mode=mode).save(b, "PNG") if mode else Image.fromarray(arr).save(b, "PNG")
        out[name] = b.getvalue()

    jpeg("o1_f28.jpg", 1, 28)
    jpeg("o3_f50.jpg", 3, 50, (40, 56))
    jpeg("o6_f24.jpg", 6, 24)
    jpeg("o8_nofocal.jpg", 8)
    jpeg("o5_ignored.jpg", 5, 35)
    jpeg("f0.jpg", None, 0)
    png("grey.png", rng.integers(0, 256, (37, 53), dtype=np.uint8))
    png("rgba.png", rng.integers(0, 256, (30, 40, 4), dtype=np.uint8))
    pal = Image.fromarray(rng.integers(0, 256, (20, 24, 3), dtype=np.uint8)).convert("P", palette=Image.ADAPTIVE)
    b = _io.BytesIO()
    pal.save(b, "PNG")
    out["palette.png"] = b.getvalue()
    return out


def io_fixtures(ref, model, transform, t0):
    """Fixtures for the host-side input path and config 5:

    * golden_load_rgb.npz -- the reference load_rgb on io_images() (file bytes + its outputs);
    * golden_infer_4k.npz -- the reference infer on a synthetic 3840x2160 frame (config 5's
      resize path: 4K -> 1536^2 -> depth resized back), f_px from the FOV head.
    """
    import tempfile

    imgs = io_images()
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for i, (name, data) in enumerate(sorted(imgs.items())):
            path = os.path.join(d, name)
            with open(path, "wb") as f:
                f.write(data)
            img, icc, fpx = ref.load_rgb(path)
            out[f"file{i}_name"] = np.array(name)
            out[f"file{i}_bytes"] = np.frombuffer(data, dtype=np.uint8).copy()
            out[f"file{i}_img"] = img
            out[f"file{i}_fpx"] = np.array(np.nan if fpx is None else float(fpx))
            out[f"file{i}_icc"] = np.array(icc is not None)
    out["n_files"] = np.array(len(imgs))
    np.savez_compressed(os.path.join(HERE, "golden_load_rgb.npz"), **out)
    print(f"[golden] load_rgb fixtures: {len(imgs)} files ({time.time()-t0:.1f}s)")

    img4k = frame(5, 2160, 3840)
    with torch.no_grad():
        p = model.infer(transform(img4k), f_px=None)
    np.savez_compressed(os.path.join(HERE, "golden_infer_4k.npz"), frame_seed=5, H=2160, W=3840,
                        depth_sub16=sub(p["depth"], 16), depth_stats=stats(p["depth"]),
                        f_px=np.array(float(p["focallength_px"])))
    print(f"[golden] infer 4K done ({time.time()-t0:.1f}s): f_px={float(p['focallength_px']):.3f}")


def stress_fixture(model, transform, t0):
    """golden_stress_frame0.npz: the reference forward on frame 0 with the STRESSED synthetic
    weights (depth_pro.weights.stressed_state_dict: LayerScale x5, outlier residual channels)."""
    from depth_pro_amd_spec import stressed_state_dict  # noqa: see shim below

    model.load_state_dict(stressed_state_dict(0), strict=True)
    caps = {}
    dec_fwd = model.decoder.forward

    def dec_capture(e):
        f, lo = dec_fwd(e)
        caps["enc_absmax"] = np.array([float(t.abs().max()) for t in e])
        caps["features_absmax"], caps["lowres_absmax"] = float(f.abs().max()), float(lo.abs().max())
        return f, lo

    model.decoder.forward = dec_capture
    hooks, peaks = [], {}
    for name in ("patch_encoder", "image_encoder"):
        vit = getattr(model.encoder, name)
        hooks.append(vit.blocks[23].register_forward_hook(
            lambda m, i, o, name=name: peaks.__setitem__(name, float(o.abs().max()))))
    x = transform(frame(0)).unsqueeze(0)
    with torch.no_grad():
        canonical, fov_deg = model.forward(x)
    for h in hooks:
        h.remove()
    model.decoder.forward = dec_fwd
    print(f"[golden] stress forward done ({time.time()-t0:.1f}s): fov={fov_deg.item():.4f} residual peaks {peaks} "
          f"encodings |max| {caps['enc_absmax']} features |max| {caps['features_absmax']:.1f}")
    np.savez_compressed(
        os.path.join(HERE, "golden_stress_frame0.npz"), frame_seed=0, fov_deg=fov_deg.numpy().reshape(-1),
        canonical_sub8=sub(canonical[0, 0], 8), canonical_stats=stats(canonical),
        residual_absmax=np.array([peaks["patch_encoder"], peaks["image_encoder"]]),
        enc_absmax=caps["enc_absmax"], features_absmax=np.array(caps["features_absmax"]),
        lowres_absmax=np.array(caps["lowres_absmax"]))


def main():
    t0 = time.time()
    torch.set_num_threads(len(os.sched_getaffinity(0)))
    try:  # before the torchvision stub goes in (transformers probes torchvision.__spec__)
        from transformers import Dinov2Config
        from transformers.models.dinov2.modeling_dinov2 import Dinov2Layer
    except ImportError:  # pragma: no cover
        Dinov2Config = Dinov2Layer = None
    ref = import_reference()
    from depth_pro.depth_pro import DepthProConfig  # reference module

    from depth_pro_amd_spec import param_spec, synthetic_state_dict  # noqa: see shim below

    cfg = DepthProConfig(
        patch_encoder_preset="dinov2l16_384",
        image_encoder_preset="dinov2l16_384",
        checkpoint_uri=None,
        decoder_features=256,
        use_fov_head=True,
        fov_encoder_preset="dinov2l16_384",
    )
    model, transform = ref.create_model_and_transforms(cfg, device=torch.device("cpu"), precision=torch.float32)
    model.eval()
    ref_sd = model.state_dict()
    spec = param_spec()
    assert list(ref_sd.keys()) == list(spec.keys()), "state-dict key order/name mismatch"
    for k, shp in spec.items():
        assert tuple(ref_sd[k].shape) == tuple(shp), (k, ref_sd[k].shape, shp)
    print(f"[golden] reference model built: {len(ref_sd)} keys, "
          f"{sum(v.numel() for v in ref_sd.values())} params ({time.time()-t0:.1f}s)")
    if "--stress" in sys.argv:
        return stress_fixture(model, transform, t0)
    sd = synthetic_state_dict(0)
    model.load_state_dict(sd, strict=True)
    print(f"[golden] synthetic weights loaded ({time.time()-t0:.1f}s)")
    if "--stages" in sys.argv:
        return stages(model, transform, t0)
    if "--io" in sys.argv:
        return io_fixtures(ref, model, transform, t0)
    meta = {"keys": len(ref_sd), "params": int(sum(v.numel() for v in ref_sd.values())),
            "torch": torch.__version__}

    # -- KAT 1: ViT block (patch_encoder.blocks[0]) + transformers Dinov2Layer cross-check
    g = torch.Generator().manual_seed(1234)
    xb = torch.randn(1, 577, 1024, generator=g)
    blk = model.encoder.patch_encoder.blocks[0]
    with torch.no_grad():
        yb = blk(xb)
    if Dinov2Layer is not None:
        hc = Dinov2Config(hidden_size=1024, num_attention_heads=16, intermediate_size=4096,
                          layer_norm_eps=1e-6, qkv_bias=True, layerscale_value=1.0,
                          hidden_act="gelu", attn_implementation="eager")
        hl = Dinov2Layer(hc).eval()
        p = "encoder.patch_encoder.blocks.0."
        with torch.no_grad():
            hl.norm1.weight.copy_(sd[p + "norm1.weight"]); hl.norm1.bias.copy_(sd[p + "norm1.bias"])
            qw, kw, vw = sd[p + "attn.qkv.weight"].chunk(3, 0)
            qb, kb, vb = sd[p + "attn.qkv.bias"].chunk(3, 0)
            a = hl.attention.attention
            a.query.weight.copy_(qw); a.key.weight.copy_(kw); a.value.weight.copy_(vw)
            a.query.bias.copy_(qb); a.key.bias.copy_(kb); a.value.bias.copy_(vb)
            hl.attention.output.dense.weight.copy_(sd[p + "attn.proj.weight"])
            hl.attention.output.dense.bias.copy_(sd[p + "attn.proj.bias"])
            hl.layer_scale1.lambda1.copy_(sd[p + "ls1.gamma"])
            hl.norm2.weight.copy_(sd[p + "norm2.weight"]); hl.norm2.bias.copy_(sd[p + "norm2.bias"])
            hl.mlp.fc1.weight.copy_(sd[p + "mlp.fc1.weight"]); hl.mlp.fc1.bias.copy_(sd[p + "mlp.fc1.bias"])
            hl.mlp.fc2.weight.copy_(sd[p + "mlp.fc2.weight"]); hl.mlp.fc2.bias.copy_(sd[p + "mlp.fc2.bias"])
            hl.layer_scale2.lambda1.copy_(sd[p + "ls2.gamma"])
            yh = hl(xb)
            if isinstance(yh, tuple):
                yh = yh[0]
        meta["dinov2_block_maxabs_vs_transformers"] = float((yh - yb).abs().max())
        print(f"[golden] timm stand-in Block vs transformers Dinov2Layer: max|d| = "
              f"{meta['dinov2_block_maxabs_vs_transformers']:.3e}")
        assert meta["dinov2_block_maxabs_vs_transformers"] < 1e-4
    else:  # pragma: no cover
        meta["dinov2_block_maxabs_vs_transformers"] = None
    np.savez_compressed(os.path.join(HERE, "golden_vit_block.npz"),
                        seed=1234, out_rows=yb[0, :64].numpy(), out_stats=stats(yb))

    # -- KAT 2: decoder fusion block 1 (with deconv) at 8x8, and the depth head at 16x16
    g = torch.Generator().manual_seed(99)
    x0 = torch.randn(1, 256, 8, 8, generator=g)
    x1 = torch.randn(1, 256, 8, 8, generator=g)
    hin = torch.randn(1, 256, 16, 16, generator=g)
    with torch.no_grad():
        fo = model.decoder.fusions[1](x0, x1)
        ho = model.head(hin)
        lo = torch.randn(1, 256, 48, 48, generator=g)
        # FOV head tail (downsample + head) on a random lowres map with zero encoder tokens
        d = model.fov.downsample(lo)
        fh = model.fov.head(d)
    np.savez_compressed(os.path.join(HERE, "golden_blocks.npz"), seed=99,
                        fusion1=fo.numpy(), head=ho.numpy(), fov_tail=fh.numpy())

    # -- KAT 3: pyramid / split / merge index semantics on a small exact image
    with torch.no_grad():
        xs = torch.randn(1, 3, 1536, 1536, generator=torch.Generator().manual_seed(7))
        x0_, x1_, x2_ = model.encoder._create_pyramid(xs)
        s0 = model.encoder.split(x0_, 0.25)
        s1 = model.encoder.split(x1_, 0.5)
        ids = torch.arange(35 * 24 * 24, dtype=torch.float64).reshape(35, 1, 24, 24)
        m0 = model.encoder.merge(ids[:25], 1, 3)
        m1 = model.encoder.merge(ids[25:34], 1, 6)
    np.savez_compressed(os.path.join(HERE, "golden_pyramid.npz"), seed=7,
                        x1_stats=stats(x1_), x2=sub(x2_, 8), x1=sub(x1_, 16),
                        s0_shape=np.array(s0.shape), s1_shape=np.array(s1.shape),
                        s0_sum=np.array([s0.double().sum().item(), (s0.double() ** 2).sum().item()]),
                        s1_sum=np.array([s1.double().sum().item(), (s1.double() ** 2).sum().item()]),
                        merge0=m0[0, 0].numpy().astype(np.int32), merge1=m1[0, 0].numpy().astype(np.int32))
    print(f"[golden] KATs done ({time.time()-t0:.1f}s)")

    # -- full forward, synthetic frame 0 (config 2/3 input), captured intermediates
    caps = {}
    enc_fwd = model.encoder.forward

    def enc_capture(x):
        out = enc_fwd(x)
        caps["encodings"] = [o.detach() for o in out]
        return out

    model.encoder.forward = enc_capture
    dec_fwd = model.decoder.forward

    def dec_capture(e):
        f, lo = dec_fwd(e)
        caps["features"], caps["lowres"] = f.detach(), lo.detach()
        return f, lo

    model.decoder.forward = dec_capture
    img0 = frame(0)
    x = transform(img0).unsqueeze(0)
    with torch.no_grad():
        canonical, fov_deg = model.forward(x)
    enc_stats = np.stack([stats(e) for e in caps["encodings"]])
    print(f"[golden] forward frame0 done ({time.time()-t0:.1f}s): fov={fov_deg.item():.4f} "
          f"canon mean={canonical.mean().item():.5f} min={canonical.min().item():.5f}")
    np.savez_compressed(
        os.path.join(HERE, "golden_forward_frame0.npz"),
        frame_seed=0, fov_deg=fov_deg.numpy().reshape(-1),
        canonical_sub8=sub(canonical[0, 0], 8), canonical_stats=stats(canonical),
        enc_stats=enc_stats, enc4_sub=sub(caps["encodings"][4][0], 4),
        enc3_sub=sub(caps["encodings"][3][0], 8),
        features_stats=stats(caps["features"]), lowres_stats=stats(caps["lowres"]),
        lowres_sub=sub(caps["lowres"][0], 4),
    )
    model.encoder.forward = enc_fwd
    model.decoder.forward = dec_fwd

    # -- infer on a non-square frame (resize path), f_px None and f_px given (np.float64)
    img1 = frame(1, 1080, 1920)
    x = transform(img1)
    with torch.no_grad():
        p0 = model.infer(x, f_px=None)
        p1 = model.infer(x, f_px=np.float64(1400.0))
    np.savez_compressed(
        os.path.join(HERE, "golden_infer_frame1.npz"), frame_seed=1, H=1080, W=1920,
        depth_sub8=sub(p0["depth"], 8), depth_stats=stats(p0["depth"]),
        f_px=np.array(float(p0["focallength_px"])),
        depth_given_sub8=sub(p1["depth"], 8), depth_given_stats=stats(p1["depth"]),
        f_px_given=np.array(float(p1["focallength_px"])),
    )
    print(f"[golden] infer frame1 done ({time.time()-t0:.1f}s): f_px={float(p0['focallength_px']):.3f}")

    # -- config 1: data/example.jpg through the reference load_rgb + transform + infer
    img, icc, fpx = ref.load_rgb(os.path.join(REF_DATA, "example.jpg"))
    meta["example_jpg"] = {"shape": list(img.shape), "f_px_exif": fpx,
                           "u8_sum": int(img.astype(np.int64).sum())}
    with torch.no_grad():
        pe = model.infer(transform(img), f_px=fpx)
    np.savez_compressed(
        os.path.join(HERE, "golden_example_jpg.npz"), shape=np.array(img.shape),
        depth_sub16=sub(pe["depth"], 16), depth_stats=stats(pe["depth"]),
        f_px=np.array(float(pe["focallength_px"])), img_sub16=img[::16, ::16].copy(),
    )
    print(f"[golden] example.jpg done ({time.time()-t0:.1f}s): f_px={float(pe['focallength_px']):.3f}")
    with open(os.path.join(HERE, "golden_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    # `depth_pro` names the REFERENCE package inside this script, so this repo's
    # spec/weights modules are loaded under a private alias.
    import importlib

    pkg_dir = os.path.join(REPO, "ml-depth-pro-video_amd", "depth_pro")
    pkg = types.ModuleType("_dpamd")
    pkg.__path__ = [pkg_dir]
    sys.modules["_dpamd"] = pkg
    shim = types.ModuleType("depth_pro_amd_spec")
    shim.param_spec = importlib.import_module("_dpamd.spec").param_spec
    shim.synthetic_state_dict = importlib.import_module("_dpamd.weights").synthetic_state_dict
    shim.stressed_state_dict = importlib.import_module("_dpamd.weights").stressed_state_dict
    sys.modules["depth_pro_amd_spec"] = shim
    main()
