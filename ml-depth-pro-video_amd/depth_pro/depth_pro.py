"""Drop-in `depth_pro` model API backed by the MI355X engine.

Mirrors the reference module `src/depth_pro/depth_pro.py`:
  DepthProConfig / DEFAULT_MONODEPTH_CONFIG_DICT   (:26-46)
  create_model_and_transforms(config, device, precision) -> (DepthPro, transform)   (:72-151)
  DepthPro.img_size (:213-216), DepthPro.forward (:218-241), DepthPro.infer (:243-298)

Same names, argument meanings, state-dict keys (1,119, strict loading) and
error behaviour (KeyError for an unknown preset or bad checkpoint keys,
AssertionError for a non-1536^2 `forward` input).  Differences, by design:
  * the arithmetic runs in libdp_mi355x.so HIP kernels on a ROCm device (bf16
    ViTs + f16 decoder/heads by default, f16 throughout for precision=torch.half,
    DEPTH_PRO_COMPUTE_DTYPE=bf16|fp16|mixed to override); a CPU device or a
    missing library raises instead of computing anything on the host;
  * with `checkpoint_uri=None` the weights are the deterministic synthetic set
    of `depth_pro.weights` (the reference leaves PyTorch's random init);
  * the fp32 parameters stay in host memory: `model.to(device)` / `.cuda()` only pick
    the device the engine runs on, and the engine packs its 16-bit GEMM-ready weight
    set straight from the host tensors (no fp32 copy of the 952 M parameters in HBM);
  * a bad frame (timed-out stream-K hand-off, NaN / inf output) is reported without
    stalling the stream: `last_status().check()` for the last call, and every later
    `infer` / `forward` call raises DPError for an earlier bad frame nobody checked.
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Mapping, Optional, Tuple, Union

import numpy as np
import torch
from torch import nn

from . import ops
from ._lib import DP_BF16, DP_F16, DPError, load
from .engine import BatchStatus, Engine, pack_weights
from .spec import IMG_SIZE, param_spec
from .weights import synthetic_state_dict

ViTPreset = str
VIT_PRESETS = ("dinov2l16_384",)


@dataclass
class DepthProConfig:
    """Configuration for DepthPro (reference depth_pro.py:26-37)."""

    patch_encoder_preset: ViTPreset
    image_encoder_preset: ViTPreset
    decoder_features: int

    checkpoint_uri: Optional[str] = None
    fov_encoder_preset: Optional[ViTPreset] = None
    use_fov_head: bool = True


DEFAULT_MONODEPTH_CONFIG_DICT = DepthProConfig(
    patch_encoder_preset="dinov2l16_384",
    image_encoder_preset="dinov2l16_384",
    checkpoint_uri="./checkpoints/depth_pro.pt",
    decoder_features=256,
    use_fov_head=True,
    fov_encoder_preset="dinov2l16_384",
)


def run_config(config: DepthProConfig = DEFAULT_MONODEPTH_CONFIG_DICT) -> DepthProConfig:
    """The config the frame loops use: `config`, unless its checkpoint file is missing and
    DEPTH_PRO_SYNTHETIC=1 asks for the deterministic synthetic weights instead (tests and
    benchmarks without the 1.9 GB checkpoint).  Without that opt-in a missing checkpoint fails
    in torch.load, as in the reference."""
    if config.checkpoint_uri and not os.path.exists(config.checkpoint_uri) and \
            os.environ.get("DEPTH_PRO_SYNTHETIC", "0") == "1":
        print(f"checkpoint {config.checkpoint_uri} not found: using synthetic weights (DEPTH_PRO_SYNTHETIC=1)")
        return DepthProConfig(**{**config.__dict__, "checkpoint_uri": None})
    return config


def _check_preset(preset: ViTPreset) -> None:
    if preset not in VIT_PRESETS:
        raise KeyError(f"Preset {preset} not found.")  # depth_pro.py:67


# DEPTH_PRO_COMPUTE_DTYPE values -> (ViT operand type, decoder/head operand type)
PRECISION_MODES = {"bf16": (DP_BF16, DP_BF16), "fp16": (DP_F16, DP_F16), "mixed": (DP_BF16, DP_F16)}


def _compute_dtype(precision: torch.dtype) -> Tuple[int, int]:
    """(ViT code, decoder code) for `precision` (or the DEPTH_PRO_COMPUTE_DTYPE override)."""
    env = os.environ.get("DEPTH_PRO_COMPUTE_DTYPE", "").lower()
    alias = {"f16": "fp16", "half": "fp16", "float16": "fp16", "bfloat16": "bf16", "bf16+f16": "mixed"}
    env = alias.get(env, env)
    if env in PRECISION_MODES:
        return PRECISION_MODES[env]
    if env:
        raise ValueError(f"DEPTH_PRO_COMPUTE_DTYPE={env!r}: expected one of {sorted(PRECISION_MODES)}")
    # precision=torch.half is the reference's model.half() (f16 everywhere); anything else gets the
    # default mode: bf16 ViTs (the bulk of the FLOPs) + f16 maps/decoder/heads, which keeps depth
    # within BASELINE's < 1e-3 relative L1 of the fp32 reference (DESIGN.md "Parity")
    return PRECISION_MODES["fp16"] if precision == torch.half else PRECISION_MODES["mixed"]


class Transform:
    """transform(image) for uint8 HxWx3 input (reference Compose, depth_pro.py:125-132).

    The uint8 frame is uploaded as-is (7 MB at 1536^2 instead of 28 MB fp32) and
    normalised to (x/255 - 0.5)/0.5 on the GPU by `dp_normalize_u8`.
    """

    def __init__(self, device: torch.device, precision: torch.dtype):
        self.device = device
        self.precision = precision

    def __call__(self, image) -> torch.Tensor:
        if torch.is_tensor(image):          # a uint8 HxWx3 frame on the device or in (pinned) host memory
            src = image.to(self.device, non_blocking=True)
            if src.dtype != torch.uint8 or src.dim() != 3 or src.shape[2] != 3:
                raise TypeError(f"transform expects an HxWx3 uint8 image, got {src.dtype} {tuple(src.shape)}")
            src = src.contiguous()
        else:
            a = np.asarray(image)
            if a.ndim == 2:
                a = a[:, :, None]
            if a.dtype != np.uint8 or a.shape[2] != 3:
                raise TypeError(f"transform expects an HxWx3 uint8 image, got {a.dtype} {a.shape}")
            src = torch.from_numpy(np.ascontiguousarray(a)).to(self.device, non_blocking=True)
        out = torch.empty(3, src.shape[0], src.shape[1], dtype=self.precision, device=self.device)
        ops.normalize_u8(src, out)
        return out


def _module_tree(spec, device, dtype) -> nn.Module:
    root = nn.Module()
    for name, shape in spec.items():
        *path, leaf = name.split(".")
        mod = root
        for p in path:
            if p not in mod._modules:
                mod.add_module(p, nn.Module())
            mod = mod._modules[p]
        mod.register_parameter(leaf, nn.Parameter(torch.empty(shape, device=device, dtype=dtype),
                                                  requires_grad=False))
    return root


class DepthPro(nn.Module):
    """DepthPro network (reference depth_pro.py:154-298) on the MI355X engine."""

    def __init__(self, use_fov_head: bool = True, device=torch.device("cpu"),
                 compute_dtype: Tuple[int, int] = (DP_BF16, DP_F16)):
        super().__init__()
        tree = _module_tree(param_spec(use_fov_head), device, torch.float32)
        for name, child in tree.named_children():
            self.add_module(name, child)
        self.use_fov_head = use_fov_head
        self.compute_dtype = compute_dtype
        self._engine: Optional[Engine] = None
        self._device: torch.device = torch.device(device)      # where the engine runs
        self._packed_device: Optional[torch.device] = None   # set by from_packed (meta parameters)
        self._use_graph = os.environ.get("DEPTH_PRO_HIPGRAPH", "0") == "1"
        self._last_status = None

    # -- engine lifecycle
    def _invalidate(self):
        self._engine = None

    def _apply(self, fn, *a, **k):
        """`.to(device)` / `.cuda()` / `.half()` (nn.Module._apply): the parameters stay in host
        memory as loaded (fp32); a new device re-targets the engine (packed on next use) and a
        dtype change is a no-op -- the compute precision is `compute_dtype`, fixed at creation
        (create_model_and_transforms' `precision`, as the reference's model.half())."""
        if self._packed_device is not None:
            return self
        try:
            fn(torch.empty(0, device="meta"))      # dtype-only (.half(), .float()): stays on meta
            return self
        except (NotImplementedError, RuntimeError):
            pass                                    # a device move: copying out of meta fails
        self._retarget(fn(torch.empty(0)).device)
        return self

    def _retarget(self, dev) -> None:
        dev = torch.device(dev)
        if dev != self._device:
            self._device = dev
            self._invalidate()

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        self._invalidate()
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    @classmethod
    def from_packed(cls, packed, device: torch.device, compute_dtype: Tuple[int, int],
                    use_fov_head: bool = True) -> "DepthPro":
        """A model whose engine runs on an already-packed weight set (`engine.pack_weights`
        output, e.g. received from rank 0 by `distributed.broadcast_packed`).  Its nn.Parameters
        live on the meta device: no checkpoint read, no fp32 copy in HBM."""
        m = cls(use_fov_head=use_fov_head, device=torch.device("meta"), compute_dtype=compute_dtype)
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:   # 'cuda' -> the current device, as tensors get
            device = torch.device("cuda", torch.cuda.current_device())
        m._packed_device = m._device = device
        m._engine = Engine(packed, m._packed_device, compute_dtype, use_fov=use_fov_head)
        m.eval()
        return m

    def engine(self) -> Engine:
        if self._engine is None:
            if self._packed_device is not None:
                raise DPError("this DepthPro was built from packed weights (from_packed); its parameters are "
                              "placeholders, so the engine cannot be rebuilt from them")
            dev = self._device
            if dev.type == "cuda" and dev.index is None:      # 'cuda' -> the current device
                dev = self._device = torch.device("cuda", torch.cuda.current_device())
            if dev.type != "cuda":
                raise DPError("DepthPro (MI355X engine) runs on a ROCm device; got device "
                              f"{dev} -- there is no CPU path")
            load()
            with torch.no_grad():
                # straight from the host tensors: each is uploaded, converted to its packed 16-bit
                # layout and dropped, so only the packed set stays in HBM
                packed = pack_weights(dict(self.state_dict()), dev, self.compute_dtype)
            self._engine = Engine(packed, dev, self.compute_dtype, use_fov=self.use_fov_head)
            if self._use_graph:
                self._engine.capture_graph()
        return self._engine

    def use_hip_graph(self, enable: bool = True) -> "DepthPro":
        """Replay the whole forward as one captured HIP graph (static shapes)."""
        self._use_graph = enable
        if self._engine is not None:
            if enable and self._engine.graph is None:
                self._engine.capture_graph()
            if not enable:
                self._engine.graph = None
        return self

    @property
    def img_size(self) -> int:
        """Return the internal image size of the network (1536)."""
        return IMG_SIZE

    def _run_frame(self, x3: torch.Tensor):
        """x3: (3, S, S) network-resolution frame on device -> (engine outputs (static buffers),
        FrameStatus)."""
        eng = self.engine()
        ops.resize(x3, eng.x0)  # dtype conversion / copy into the static input
        out = eng.run()
        return out, eng.finish_status()

    def last_status(self):
        """Status of the most recent `infer` / `forward` call (`engine.BatchStatus` over its frames):
        `.check()` raises DPError naming every invalid frame of that call (a timed-out stream-K
        hand-off, or NaN / inf in depth or focal length) -- waiting for those frames only.  The
        frame loops call it before writing a frame's files."""
        if self._last_status is None:
            return self.engine().last_status
        return self._last_status

    def _check_earlier(self, eng: Engine) -> None:
        """Non-blocking health check of earlier frames: a finished bad frame that no
        caller has checked raises here, on the next call, instead of going unnoticed."""
        eng.check_status(block=False)

    def forward(self, x: torch.Tensor) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """Canonical inverse depth (B,1,1536,1536) and FOV in degrees (B,1,1,1)."""
        _, _, H, W = x.shape
        assert H == self.img_size and W == self.img_size
        eng = self.engine()
        self._check_earlier(eng)
        outs, fovs, sts = [], [], []
        for b in range(x.shape[0]):
            (canonical, fov), st = self._run_frame(x[b])
            outs.append(canonical.clone())
            fovs.append(fov.clone())
            sts.append(st)
        self._last_status = BatchStatus(sts)
        canonical = torch.cat(outs, 0)
        fov_deg = torch.cat(fovs, 0) if self.use_fov_head else None
        return canonical, fov_deg

    @torch.no_grad()
    def infer(
        self,
        x: torch.Tensor,
        f_px: Optional[Union[float, torch.Tensor]] = None,
        interpolation_mode="bilinear",
    ) -> Mapping[str, torch.Tensor]:
        """Infer depth [m] and focal length [px] (reference depth_pro.py:243-298).

        x: (3,H,W) or (B,3,H,W).  As in the reference, a batch gives depth (B,H,W) and,
        without a given f_px, one focal length per frame (B,); frames run one at a time
        through the engine (each a full 1536^2 forward).  `interpolation_mode` is the
        F.interpolate mode of both resizes (to 1536^2 and back): "bilinear" or "bicubic".
        """
        mode_ok = ops.interp_mode(interpolation_mode)  # noqa: F841  (ValueError for another mode)
        if len(x.shape) == 3:
            x = x.unsqueeze(0)
        B, _, H, W = x.shape
        eng = self.engine()
        if x.device.type != eng.dev.type or (x.device.index or 0) != eng.dev.index:
            raise DPError(f"input on {x.device}, model on {eng.dev}")
        if f_px is None and not self.use_fov_head:
            raise TypeError("f_px is required when the model has no FOV head")
        self._check_earlier(eng)
        given = None
        if f_px is not None:
            given = float(f_px.detach().float().reshape(-1)[0].item()) if torch.is_tensor(f_px) else float(f_px)
        depth = torch.empty(B, H, W, dtype=torch.float32, device=x.device)
        f_out = torch.empty(B, dtype=torch.float32, device=x.device) if f_px is None else None
        sts = []
        for b in range(B):
            # prologue: (resize to) 1536^2 fp32 straight into the engine's static input
            ops.resize(x[b], eng.x0, interpolation_mode)
            canonical, fov_deg = eng.run()
            bad = eng.status_dev[-1:]     # NaN / inf outputs of this frame (FrameStatus)
            if f_px is None:
                ops.infer_epilogue(canonical, fov_deg, None, H, W, depth[b], f_out[b], bad, mode=interpolation_mode)
            else:
                ops.infer_epilogue(canonical, None, given, H, W, depth[b], None, bad, mode=interpolation_mode)
            sts.append(eng.finish_status())
        self._last_status = BatchStatus(sts)
        if f_px is None:
            f_px = f_out.squeeze()
        else:
            f_px = f_px.squeeze()  # mirrors depth_pro.py:286 (a plain Python float has no .squeeze)
        return {"depth": depth.squeeze(), "focallength_px": f_px}


def create_model_and_transforms(
    config: DepthProConfig = DEFAULT_MONODEPTH_CONFIG_DICT,
    device: torch.device = torch.device("cpu"),
    precision: torch.dtype = torch.float32,
    seed: int = 0,
) -> Tuple[DepthPro, Transform]:
    """Create a DepthPro model and load weights from `config.checkpoint_uri`.

    Reference: depth_pro.py:72-151.  `seed` picks the synthetic weight set used
    when `config.checkpoint_uri` is None.
    """
    _check_preset(config.patch_encoder_preset)
    _check_preset(config.image_encoder_preset)
    use_fov = bool(config.use_fov_head and config.fov_encoder_preset is not None)
    if use_fov:
        _check_preset(config.fov_encoder_preset)
    if config.decoder_features != 256:
        raise KeyError(f"decoder_features={config.decoder_features} not supported (the dinov2l16_384 model uses 256)")
    device = torch.device(device)
    model = DepthPro(use_fov_head=use_fov, device=torch.device("cpu"), compute_dtype=_compute_dtype(precision))

    if config.checkpoint_uri is not None:
        state_dict = torch.load(config.checkpoint_uri, map_location="cpu", weights_only=True)
    else:
        state_dict = synthetic_state_dict(seed, use_fov_head=use_fov)
    missing_keys, unexpected_keys = model.load_state_dict(state_dict=state_dict, strict=True)
    if len(unexpected_keys) != 0:
        raise KeyError(f"Found unexpected keys when loading monodepth: {unexpected_keys}")
    missing_keys = [key for key in missing_keys if "fc_norm" not in key]
    if len(missing_keys) != 0:
        raise KeyError(f"Keys are missing when loading monodepth: {missing_keys}")
    del state_dict
    # the engine's device; the fp32 parameters stay on the host (DepthPro._apply), and
    # precision == torch.half (the reference's model.half()) is already the f16 compute_dtype
    model._retarget(device)
    model.eval()
    transform = Transform(device, precision)
    return model, transform
