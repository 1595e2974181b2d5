"""The MI355X forward engine: packed weights + static HBM workspace + HIP kernels.

`Engine.forward(x0)` runs `DepthPro.forward` (reference `depth_pro.py:218-241`)
for one 1536x1536 frame entirely through libdp_mi355x.so kernels on the
current stream:

  patchify (pyramid + 35 windows, encoder.py:151-263)
  -> 3 x ViT-L/16 (patch x35 windows, image x1, fov x1; timm Block x24 each)
  -> merge + project/upsample (encoder.py:190-324)
  -> MultiresConvDecoder (decoder.py:74-206) -> head (depth_pro.py:182-207)
  -> FOV head (fov.py:56-82)

All buffers are allocated once per engine, so a forward is hipGraph-capturable
(`capture_graph`).  Activations are token-major / NHWC in 16-bit (bf16 or
f16), the ViT residual streams fp32.
"""

from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch

from . import ops
from ._lib import DP_ACT_GELU, DP_ACT_RELU, DP_BF16, DP_F16, DP_F32, DPError, load
from .spec import DEPTH, EMBED_DIM, HEADS, IMG_SIZE, MLP_DIM, TOKENS

# Timing ablations for tools/frame_ablation.py only (results are wrong when set):
# comma list of {side, img, fovenc, attn, ln, vitgemm, decoder, head}.
_ABLATE = set(filter(None, os.environ.get("DP_ABLATE", "").split(",")))

NWIN = 35
TOK = TOKENS            # 577
PTOK = TOKENS - 1       # 576
D = EMBED_DIM


# --------------------------------------------------------------------- packing
def _conv_w(w: torch.Tensor, dt) -> torch.Tensor:
    """Conv2d [Cout, Cin, kh, kw] -> B[Cout][(ci/64, ky, kx, ci%64)] (ops.conv_weight)."""
    return ops.conv_weight(w, dt)


def _deconv_w(w: torch.Tensor, dt) -> torch.Tensor:
    """ConvTranspose2d [Cin, Cout, 2, 2] -> B[(dy, dx, co)][ci]."""
    ci, co = w.shape[0], w.shape[1]
    return w.permute(2, 3, 1, 0).reshape(4 * co, ci).to(dt).contiguous()


def _f32(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to(torch.float32).contiguous()


def compose_head(wd: torch.Tensor, bd: torch.Tensor, w2: torch.Tensor, b2: torch.Tensor, dt) -> Dict[str, object]:
    """Compose the depth head's ConvTranspose2d(k2, s2) (head.1) with the 3x3 conv after it
    (head.2) -- linear, nothing in between (depth_pro.py:182-207) -- into ONE 3x3 conv over
    the pre-upsampling map whose 128 outputs are (parity q = 2*dy + dx, channel o):

        W'[q, o, ty, tx, ci] = sum over taps (a, b) of head.2 that land in h0 pixel
                               (y + ty - 1, x + tx - 1) of  W2[o, c, a, b] Wd[ci, c, py, px]

    with (py, px) the deconv sub-pixel each tap reads.  The deconv bias rides along as a
    per-column bias; `corr[a, b, o] = sum_c W2[o, c, a, b] bd[c]` is what a tap that falls
    in head.2's zero padding must NOT contribute (subtracted at the image border).
    Removes the 1536^2 x 128 intermediate (604 MB written + re-read 9x) from the frame.
    """
    ci_n, c_n = wd.shape[0], wd.shape[1]
    o_n = w2.shape[0]
    wc = torch.zeros(4, o_n, 3, 3, ci_n, dtype=torch.float32, device=wd.device)
    for dy in range(2):
        for dx in range(2):
            q = 2 * dy + dx
            for a in range(-1, 2):
                ry = dy + a
                ty, py = ry // 2 + 1, ry & 1
                for b in range(-1, 2):
                    rx = dx + b
                    tx, px = rx // 2 + 1, rx & 1
                    wc[q, :, ty, tx, :] += w2[:, :, a + 1, b + 1] @ wd[:, :, py, px].t()
    corr = torch.einsum("ocab,c->abo", w2, bd).contiguous()             # [3, 3, o]
    bias = (b2 + corr.sum(dim=(0, 1))).repeat(4).contiguous()           # interior: all 9 taps
    w_conv = wc.reshape(4 * o_n, 3, 3, ci_n).permute(0, 3, 1, 2)            # as a Conv2d weight [(q,o), ci, ty, tx]
    return {"head.ps.w": ops.conv_weight(w_conv, dt), "head.ps.b": bias,
            "head.ps.corr": corr.reshape(-1).contiguous()}


def compose_head0(w0: torch.Tensor, b0: torch.Tensor, wo: torch.Tensor, bo: torch.Tensor, dt) -> Dict[str, object]:
    """Compose the decoder's last 1x1 `out_conv` (decoder.fusions.0.out_conv, decoder.py:184) with
    the head's first 3x3 conv (head.0, depth_pro.py:182-207) -- linear, nothing in between -- into
    ONE 3x3 conv over the fusion block's output:

        W'[o, c, ky, kx] = sum_m W0[o, m, ky, kx] Wo[m, c],   corr[ky, kx, o] = sum_m W0[o, m, ky, kx] bo[m]

    with bias b0 + sum over the 9 taps of corr; a tap that falls in head.0's zero padding must not
    contribute its corr (the 1x1's output is 0 there, not bo): the GEMM epilogue subtracts it at
    the image border (DP_STORE_ROWS with head_corr).  Removes the 768^2 x 256 1x1 GEMM and its
    302 MB map from the frame."""
    wc = torch.einsum("omyx,mc->ocyx", w0, wo)
    corr = torch.einsum("omyx,m->yxo", w0, bo).contiguous()          # [3, 3, o]
    bias = (b0 + corr.sum(dim=(0, 1))).contiguous()
    return {"head.0c.w": ops.conv_weight(wc, dt), "head.0c.b": bias, "head.0c.corr": corr.reshape(-1).contiguous()}


def precision_codes(codes) -> Tuple[int, int]:
    """(ViT code, decoder code) from one DP_BF16 / DP_F16 code or a pair of them.

    The ViTs (qkv / attention / proj / fc1 / fc2, fp32 residual stream) run in the
    first type; everything from the final ViT LayerNorm output on -- merged maps,
    project/upsample, decoder, heads, FOV tail -- in the second.
    """
    if isinstance(codes, (tuple, list)):
        v, d = int(codes[0]), int(codes[1])
    else:
        v = d = int(codes)
    for c in (v, d):
        if c not in (DP_BF16, DP_F16):
            raise DPError("compute dtype must be bf16 or f16")
    return v, d


def pack_weights(sd: Dict[str, torch.Tensor], device: torch.device, dtype_code) -> Dict[str, object]:
    """Convert a (reference-named) state dict into GEMM-ready device tensors.

    `dtype_code`: one DP_BF16 / DP_F16 code, or (ViT code, decoder code) -- see
    `precision_codes`.

    Linear weights stay [N][K]; conv weights become [Cout][ky][kx][Cin]; k2s2
    deconvs [(dy,dx,Cout)][Cin].  Each decoder fusion's deconv (no bias) and the
    1x1 out_conv that follows it (decoder.py:180-184) are linear with nothing in
    between, so they are composed once here into one deconv with bias
    (W'[ci,co] = sum_c Wd[ci,c] Wo[co,c]): the 1x1 pass at the upsampled
    resolution disappears from the frame.
    """
    vcode, dcode = precision_codes(dtype_code)
    vdt, dt = ops.torch_dtype(vcode), ops.torch_dtype(dcode)
    g = lambda k: sd[k].detach().to(device)  # noqa: E731
    P: Dict[str, object] = {}
    for vit in ("encoder.patch_encoder.", "encoder.image_encoder.", "fov.encoder.0."):
        if vit + "cls_token" not in sd:
            continue
        P[vit + "cls"] = _f32(g(vit + "cls_token")).reshape(D)
        P[vit + "pos"] = _f32(g(vit + "pos_embed")).reshape(TOK, D)
        P[vit + "pe.w"] = g(vit + "patch_embed.proj.weight").reshape(D, -1).to(vdt).contiguous()
        P[vit + "pe.b"] = _f32(g(vit + "patch_embed.proj.bias"))
        for i in range(DEPTH):
            b = f"{vit}blocks.{i}."
            for n in ("norm1.weight", "norm1.bias", "norm2.weight", "norm2.bias", "attn.qkv.bias",
                      "attn.proj.bias", "mlp.fc1.bias", "mlp.fc2.bias", "ls1.gamma", "ls2.gamma"):
                P[b + n] = _f32(g(b + n))
            for n in ("attn.qkv.weight", "attn.proj.weight", "mlp.fc1.weight", "mlp.fc2.weight"):
                P[b + n] = g(b + n).to(vdt).contiguous()
        P[vit + "norm.weight"] = _f32(g(vit + "norm.weight"))
        P[vit + "norm.bias"] = _f32(g(vit + "norm.bias"))
    # encoder project / upsample
    for name, n_up in (("upsample_latent0", 3), ("upsample_latent1", 2), ("upsample0", 1),
                       ("upsample1", 1), ("upsample2", 1)):
        p = f"encoder.{name}."
        P[p + "0"] = _conv_w(g(p + "0.weight"), dt)
        for i in range(1, n_up + 1):
            P[p + str(i)] = _deconv_w(g(p + f"{i}.weight"), dt)
    P["encoder.upsample_lowres.w"] = _deconv_w(g("encoder.upsample_lowres.weight"), dt)
    P["encoder.upsample_lowres.b"] = _f32(g("encoder.upsample_lowres.bias")).repeat(4)
    P["encoder.fuse_lowres.w"] = _conv_w(g("encoder.fuse_lowres.weight"), dt)
    P["encoder.fuse_lowres.b"] = _f32(g("encoder.fuse_lowres.bias"))
    # decoder
    for i in range(1, 5):
        P[f"decoder.convs.{i}"] = _conv_w(g(f"decoder.convs.{i}.weight"), dt)
    for i in range(5):
        p = f"decoder.fusions.{i}."
        for r in ("resnet1", "resnet2"):
            for j in (1, 3):
                P[p + f"{r}.{j}.w"] = _conv_w(g(p + f"{r}.residual.{j}.weight"), dt)
                P[p + f"{r}.{j}.b"] = _f32(g(p + f"{r}.residual.{j}.bias"))
        wo = _f32(g(p + "out_conv.weight"))[:, :, 0, 0]  # [co, c]
        bo = _f32(g(p + "out_conv.bias"))
        if i != 0:
            wd = _f32(g(p + "deconv.weight"))  # [ci, c, 2, 2]
            wc = torch.einsum("icyx,oc->ioyx", wd, wo)  # composed deconv [ci, co, 2, 2]
            P[p + "up.w"] = _deconv_w(wc, dt)
            P[p + "up.b"] = bo.repeat(4)
        else:
            P[p + "out.w"] = wo.to(dt).contiguous()
            P[p + "out.b"] = bo
    # head
    P["head.0.w"] = _conv_w(g("head.0.weight"), dt)
    P["head.0.b"] = _f32(g("head.0.bias"))
    P.update(compose_head0(_f32(g("head.0.weight")), _f32(g("head.0.bias")),
                           _f32(g("decoder.fusions.0.out_conv.weight"))[:, :, 0, 0],
                           _f32(g("decoder.fusions.0.out_conv.bias")), dt))
    P.update(compose_head(_f32(g("head.1.weight")), _f32(g("head.1.bias")), _f32(g("head.2.weight")),
                          _f32(g("head.2.bias")), dt))
    P["head.4.w"] = _f32(g("head.4.weight")).reshape(-1)
    P["head.4.b"] = float(sd["head.4.bias"].detach().float().reshape(-1)[0])
    if "fov.encoder.1.weight" in sd:
        P["fov.lin.w"] = g("fov.encoder.1.weight").to(dt).contiguous()
        P["fov.lin.b"] = _f32(g("fov.encoder.1.bias"))
        P["fov.down.w"] = _conv_w(g("fov.downsample.0.weight"), dt)
        P["fov.down.b"] = _f32(g("fov.downsample.0.bias"))
        P["fov.h0.w"] = _conv_w(g("fov.head.0.weight"), dt)
        P["fov.h0.b"] = _f32(g("fov.head.0.bias"))
        P["fov.h2.w"] = _conv_w(g("fov.head.2.weight"), dt)
        P["fov.h2.b"] = _f32(g("fov.head.2.bias"))
        P["fov.h4.w"] = _f32(g("fov.head.4.weight")).reshape(-1)
        P["fov.h4.b"] = float(sd["fov.head.4.bias"].detach().float().reshape(-1)[0])
    return P


# ---------------------------------------------------------------------- engine
class _ViTBuffers:
    def __init__(self, rows: int, dt, dev, out_dt=None):
        self.rows = rows
        self.x = torch.empty(rows, D, dtype=torch.float32, device=dev)
        self.h = torch.empty(rows, D, dtype=dt, device=dev)
        self.qkv = torch.empty(rows, 3 * D, dtype=dt, device=dev)
        self.a = torch.empty(rows, D, dtype=dt, device=dev)
        self.m = torch.empty(rows, MLP_DIM, dtype=dt, device=dev)
        # final-norm output (the encoder features) in the decoder's type; it reuses the
        # attention-output buffer, which is dead once the last block has run
        out_dt = out_dt or dt
        self.out = self.h if out_dt == dt else self.a.view(out_dt)


class _Rows:
    """Rows [r0, r1) of a _ViTBuffers as contiguous views (one window group of the patch encoder)."""

    def __init__(self, buf: _ViTBuffers, r0: int, r1: int):
        self.rows = r1 - r0
        for n in ("x", "h", "qkv", "a", "m", "out"):
            setattr(self, n, getattr(buf, n)[r0:r1])


def window_groups(n: int):
    """Split the 35 windows into n contiguous groups of near-equal size: [(w0, w1), ...]."""
    n = max(1, min(int(n), NWIN))
    cuts = [round(i * NWIN / n) for i in range(n + 1)]
    return [(cuts[i], cuts[i + 1]) for i in range(n)]


class Engine:
    """One frame (batch 1) per forward; static workspace (~4 GB)."""

    def __init__(self, packed: Dict[str, object], device: torch.device, dtype_code,
                 use_fov: bool = True):
        load()
        if device.type != "cuda":
            raise DPError("the MI355X Depth Pro engine needs a ROCm/HIP device")
        self.vcode, self.code = precision_codes(dtype_code)
        if packed[next(k for k in packed if k.endswith("attn.qkv.weight"))].dtype != ops.torch_dtype(self.vcode) \
                or packed["decoder.convs.4"].dtype != ops.torch_dtype(self.code):
            raise DPError("packed weights were made for another compute precision")
        self.P = packed
        self.dev = device
        self.vdt = ops.torch_dtype(self.vcode)   # ViT GEMM / attention operands
        self.dt = ops.torch_dtype(self.code)     # encoder maps, decoder, heads
        self.use_fov = use_fov and "fov.lin.w" in packed
        dt, vdt, dev = self.dt, self.vdt, device
        e = lambda *s, dtype=None: torch.empty(*s, dtype=dtype or dt, device=dev)  # noqa: E731
        S = IMG_SIZE
        self.x0 = e(3, S, S, dtype=torch.float32)           # network input (normalized, 1536^2)
        self.cols = e(NWIN * PTOK, 768, dtype=vdt)
        self.vp = _ViTBuffers(NWIN * TOK, vdt, dev, dt)     # patch encoder (35 windows)
        self.vi = _ViTBuffers(TOK, vdt, dev, dt)            # image encoder
        self.vf = _ViTBuffers(TOK, vdt, dev, dt) if self.use_fov else None
        # merged encoder maps (NHWC)
        self.lat0 = e(96 * 96, D)
        self.lat1 = e(96 * 96, D)
        self.f0 = e(96 * 96, D)
        self.f1 = e(48 * 48, D)
        self.f2 = e(24 * 24, D)
        self.g = e(24 * 24, D)
        # upsample chains
        self.t96_256 = e(96 * 96, 256)
        self.t192_256 = e(192 * 192, 256)
        self.t384_256 = e(384 * 384, 256)
        self.enc0 = e(768 * 768, 256)
        self.t96_256b = e(96 * 96, 256)
        self.t192_256b = e(192 * 192, 256)
        self.enc1 = e(384 * 384, 256)
        self.t96_512 = e(96 * 96, 512)
        self.enc2 = e(192 * 192, 512)
        self.t48_1024 = e(48 * 48, D)
        self.enc3 = e(96 * 96, D)
        self.t24_1024 = e(24 * 24, D)
        self.cat = e(48 * 48, 2 * D)
        self.enc4 = e(48 * 48, D)
        # decoder (one set of scratch maps per resolution)
        self.dec = {}
        for s in (48, 96, 192, 384, 768):
            self.dec[s] = {k: e(s * s, 256) for k in ("c", "t", "x", "y")}
        self.low = self.dec[48]["c"]
        self.up = {s: e(s * s, 256) for s in (96, 192, 384, 768)}
        self.feats = e(768 * 768, 256)
        # head
        self.h0 = e(768 * 768, 128)
        self.canonical = e(1, 1, S, S, dtype=torch.float32)
        # fov
        self.fov_tok = e(PTOK, 128)
        self.fx = e(24 * 24, 128)
        self.f12 = e(12 * 12, 64)
        self.f6 = e(6 * 6, 32)
        self.fov_deg = e(1, 1, 1, 1, dtype=torch.float32)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.side = torch.cuda.Stream(device=dev)
        self.side2 = torch.cuda.Stream(device=dev)     # FOV encoder when DP_SIDE_STREAMS=2
        # stream-K GEMM scratch, one per stream that issues GEMMs (main / side)
        self.ws_main = ops.gemm_workspace(dev)
        self.ws_side = ops.gemm_workspace(dev)
        self.ws_side2 = ops.gemm_workspace(dev)
        # project/upsample chains and the decoder's encoder-feature projections beside the main
        # stream (DP_DEC_STREAMS=1, see _forward): two more streams, one of them issuing stream-K
        self.dec_a = torch.cuda.Stream(device=dev)
        self.dec_b = torch.cuda.Stream(device=dev)
        self.dec_c = torch.cuda.Stream(device=dev)
        self.ws_dec = ops.gemm_workspace(dev)
        self.dec_streams = os.environ.get("DP_DEC_STREAMS", "1") == "1"
        self.small_conv_tile = int(os.environ.get("DP_SMALL_CONV_TILE", "0"))
        self.conv768_tile = int(os.environ.get("DP_CONV768_TILE", "0"))
        self.qkv_tile = int(os.environ.get("DP_QKV_TILE", "0"))   # A/B: patch-encoder qkv engine
        self.side_sync = os.environ.get("DP_SIDE_SYNC", "0") == "1"
        # decoder out_conv composed into the head's first conv (compose_head0); DP_HEAD0_COMPOSE=0: separate
        self.head0_compose = os.environ.get("DP_HEAD0_COMPOSE", "1") == "1" and "head.0c.w" in packed
        self.fov_at = int(os.environ.get("DP_FOV_AT", "-1"))
        self.lat0_sk = os.environ.get("DP_LAT0_SK", "1") == "1"
        # The 35 windows of the patch encoder are independent through all 24 blocks: run them as
        # `DP_PATCH_GROUPS` window groups on their own streams, so one group's bandwidth-bound
        # phases (LayerNorm, GEMM epilogues) overlap another group's MFMA phases.
        self.set_patch_groups(int(os.environ.get("DP_PATCH_GROUPS", "1")), _init=True)
        # their sticky error words (dp_mi355x.h DP_GEMM_WS_ERROR_OFFSET), read back asynchronously
        # after every forward into pinned memory and checked by `check_status`
        wss = [self.ws_main, self.ws_side, self.ws_side2, self.ws_dec] + self.ws_groups
        self._err_dev = [w[ops.WS_ERROR_OFFSET:ops.WS_ERROR_OFFSET + 4].view(torch.int32) for w in wss]
        self._err_host = torch.zeros(len(wss), dtype=torch.int32, pin_memory=True)
        self._err_ev: Optional[torch.cuda.Event] = None
        self.sync_check = os.environ.get("DP_CHECK_SYNC", "0") == "1"
        self.serial_side = False   # True: run the side encoders on the current stream (profiling)

        # FOV encoder + head beside the decoder instead of the patch encoder (measured: 0.3 ms
        # slower on MI355X, so off by default; DP_FOV_LATE=1 to try)
        self.fov_late = os.environ.get("DP_FOV_LATE", "0") == "1"
        # Measured and rejected: the side encoders' fc2 (M = 577, K = 4096, 24 workgroups) as 2 / 4
        # accumulating K-slice launches, to shorten the workgroups that block the patch
        # encoder's CUs: frame 24.32 -> 24.67 / 25.41 ms.
        # where the image (+ FOV) encoders run (A/B switch, DP_SIDE_MODE):
        #   concurrent -- side stream beside the patch encoder (default);
        #   serial     -- main stream, ahead of the patch encoder;
        #   late       -- side stream beside the project/upsample chain, after the patch encoder
        self.side_mode = os.environ.get("DP_SIDE_MODE", "concurrent")
        # the FOV encoder on a second side stream, joined only at the FOV head, so the join before
        # fuse_lowres waits for the image encoder alone: 24.41-24.43 -> 24.16-24.25 ms per frame
        # (DP_SIDE_STREAMS=1: both encoders on one side stream)
        self.side_streams = int(os.environ.get("DP_SIDE_STREAMS", "2"))
        # GEMM engine of the side encoders' block GEMMs (DP_SIDE_TILE, a DP_TILE_* value; 0 = planner)
        self.side_tile = int(os.environ.get("DP_SIDE_TILE", "0"))
        # softmax scale * log2(e) folded into the qkv epilogue (per-column gamma on Q) so that attention
        # takes one exp2 per score (dp_attention_log2q); DP_ATTN_LOG2Q=0: scale inside the attention
        self.qkv_gamma = (ops.log2q_gamma(HEADS, D // HEADS, dev)
                          if os.environ.get("DP_ATTN_LOG2Q", "1") == "1" else None)
        # ViT LayerNorms fused into the patch encoder's proj / fc2 epilogues (dp_gemm_ln, DP_LN_FUSE=1).
        # Measured and rejected (round 2, profiles/r02k_ln_fuse/): 40.35 / 40.44 fps fused vs 41.84 /
        # 41.73 separate; eager proj + LN 100.6 us fused vs 67.8 + 22.5, fc2 + LN 194.2 vs 169.8 + 22.5:
        # the row-band wait (every workgroup waits for the slowest of its band) and the normalise
        # pass after it cost more than the LayerNorm pass they replace.
        self.ln_fuse = os.environ.get("DP_LN_FUSE", "0") == "1"
        if self.side_mode not in ("concurrent", "serial", "late"):
            raise DPError(f"DP_SIDE_MODE={self.side_mode!r}")

    # ------------------------------------------------------------------ ViT
    def _vit(self, pre: str, buf: _ViTBuffers, n_img: int, cols_off_rows: int, hooks=None, ln_fuse=False,
             pre_fc1=None, pre_fc2=None):
        for _ in self._vit_iter(pre, buf, n_img, cols_off_rows, hooks, ln_fuse, pre_fc1, pre_fc2):
            pass

    def _vit_iter(self, pre: str, buf: _ViTBuffers, n_img: int, cols_off_rows: int, hooks=None, ln_fuse=False,
                  pre_fc1=None, pre_fc2=None):
        """The ViT as a generator: yields after each block (the side encoders step block by block
        beside the patch encoder, DP_SIDE_SYNC); pre_fc1 / pre_fc2: callbacks before those GEMMs."""
        P, M = self.P, n_img * TOK
        # side encoders (one image, M = 577): engine choice for CU-time, not latency (DP_SIDE_TILE)
        t = self.side_tile if n_img == 1 else 0
        # patch embed (k16 s16 conv as GEMM over the im2col rows) + bias + pos -> rows 1..576
        ops.gemm(self.cols, P[pre + "pe.w"], buf.x, M=n_img * PTOK, N=D, K=768,
                 A_off=cols_off_rows * 768, bias=P[pre + "pe.b"], pos=P[pre + "pos"], ldpos=D,
                 pos_group=PTOK, pos_off=1, row_group=PTOK, row_group_out=TOK, row_off=1)
        ops.vit_cls_rows(buf.x, P[pre + "cls"], P[pre + "pos"], n_img)
        # LayerNorms fused into the residual GEMMs (dp_gemm_ln): norm2 rides on attn.proj, the
        # next block's norm1 (or the final norm) on mlp.fc2; only block 0's norm1 -- after the
        # patch embedding, whose cls rows come from another kernel -- is a pass of its own
        # Its workgroups wait for the other workgroups of their row band, so two such launches
        # must never run at once (each could hold CUs the other's missing workgroups need):
        # only the patch encoder, alone on the main stream, uses it (ln_fuse), never the side
        # encoders beside it nor concurrent window groups.
        fuse = ln_fuse and self.ln_fuse and "ln" not in _ABLATE and "vitgemm" not in _ABLATE
        for i in range(DEPTH):
            b = f"{pre}blocks.{i}."
            if "ln" not in _ABLATE and (i == 0 or not fuse):
                ops.layernorm(buf.x, P[b + "norm1.weight"], P[b + "norm1.bias"], buf.h, M, D)
            if "vitgemm" not in _ABLATE:
                ops.gemm(buf.h, P[b + "attn.qkv.weight"], buf.qkv, M=M, N=3 * D, K=D, bias=P[b + "attn.qkv.bias"],
                         gamma=self.qkv_gamma, tile=t or (self.qkv_tile if n_img > 1 else 0))
            if "attn" not in _ABLATE:
                ops.attention(buf.qkv, buf.a, n_img, TOK, HEADS, D // HEADS, log2q=self.qkv_gamma is not None)
            ln2 = (P[b + "norm2.weight"], P[b + "norm2.bias"], buf.h, 1e-6) if fuse else None
            if "vitgemm" not in _ABLATE:
                ops.gemm(buf.a, P[b + "attn.proj.weight"], buf.x, M=M, N=D, K=D, bias=P[b + "attn.proj.bias"],
                         gamma=P[b + "ls1.gamma"], accumulate=True, tile=t, ln=ln2)
            if "ln" not in _ABLATE and not fuse:
                ops.layernorm(buf.x, P[b + "norm2.weight"], P[b + "norm2.bias"], buf.h, M, D)
            nb = f"{pre}blocks.{i + 1}."
            ln1 = None
            if fuse:
                ln1 = ((P[nb + "norm1.weight"], P[nb + "norm1.bias"], buf.h, 1e-6) if i + 1 < DEPTH else
                       (P[pre + "norm.weight"], P[pre + "norm.bias"], buf.out, 1e-6))
            if pre_fc1:
                pre_fc1(i)
            if "vitgemm" not in _ABLATE:
                ops.gemm(buf.h, P[b + "mlp.fc1.weight"], buf.m, M=M, N=MLP_DIM, K=D, bias=P[b + "mlp.fc1.bias"],
                         act=DP_ACT_GELU, tile=t)
            if pre_fc2:
                pre_fc2(i)
            if "vitgemm" not in _ABLATE:
                ops.gemm(buf.m, P[b + "mlp.fc2.weight"], buf.x, M=M, N=D, K=MLP_DIM, bias=P[b + "mlp.fc2.bias"],
                         gamma=P[b + "ls2.gamma"], accumulate=True, tile=t, ln=ln1)
            if hooks and i in hooks:
                hooks[i]()
            yield i
        if not fuse:
            ops.layernorm(buf.x, P[pre + "norm.weight"], P[pre + "norm.bias"], buf.out, M, D)

    # -------------------------------------------------------- conv helpers
    def _conv3(self, x, s_in, cin, w, out, cout, bias=None, relu_a=False, act=0, R1=None, R2=None,
               stride=1, head_w=None, head_b=0.0, border_corr=None):
        s_out = (s_in + 2 - 3) // stride + 1
        # A/B (DP_SMALL_CONV_TILE, a DP_TILE_* value): engine of the decoder's small-grid
        # ResidualBlock convs (48^2 / 96^2: 9 / 36 tiles of 256 x 256 on 256 CUs)
        tile = self.small_conv_tile if (self.small_conv_tile and s_out <= 96 and cout == 256 and cin == 256) else 0
        # A/B (DP_CONV768_TILE): engine of the 768^2 ResidualBlock convs (default: persistent 256 x 256)
        if self.conv768_tile and s_out == 768 and cout == 256 and cin == 256:
            tile = self.conv768_tile
        ops.gemm(x, w, out, M=s_out * s_out, N=cout, K=9 * cin,
                 conv=dict(in_h=s_in, in_w=s_in, in_c=cin, k=3, stride=stride, pad=1, out_h=s_out, out_w=s_out),
                 relu_a=relu_a, bias=bias, act=act, R1=R1, ldr1=cout, R2=R2, ldr2=cout,
                 head_w=head_w, head_b=head_b, ldc=cout, tile=tile, border_corr=border_corr)

    def _deconv(self, x, s_in, cin, w, out, cout, bias=None, C_off=0, ldc=None):
        ops.gemm(x, w, out, M=s_in * s_in, N=4 * cout, K=cin, bias=bias, deconv=(s_in, s_in, cout),
                 C_off=C_off, ldc=cout if ldc is None else ldc)

    def _resblock(self, pre: str, x, s, out, extra=None):
        """out = x (+ extra) + conv(relu(conv(relu(x)))) at s x s x 256."""
        t = self.dec[s]["t"]
        P = self.P
        self._conv3(x, s, 256, P[pre + ".1.w"], t, 256, bias=P[pre + ".1.b"], relu_a=True, act=DP_ACT_RELU)
        self._conv3(t, s, 256, P[pre + ".3.w"], out, 256, bias=P[pre + ".3.b"], R1=x, R2=extra)

    def _fusion(self, i: int, feats, s, x1):
        """FeatureFusionBlock2d i at resolution s (output at 2s for i != 0)."""
        P, d = self.P, self.dec[s]
        p = f"decoder.fusions.{i}."
        x = feats
        if x1 is not None:
            self._resblock(p + "resnet1", x1, s, d["x"], extra=feats)
            x = d["x"]
        self._resblock(p + "resnet2", x, s, d["y"])
        if i != 0:
            out = self.up[2 * s]
            self._deconv(d["y"], s, 256, P[p + "up.w"], out, 256, bias=P[p + "up.b"])
            return out
        if self.head0_compose:   # out_conv is composed into head.0 (compose_head0)
            return d["y"]
        ops.gemm(d["y"], P[p + "out.w"], self.feats, M=s * s, N=256, K=256, bias=P[p + "out.b"])
        return self.feats

    def set_patch_groups(self, n: int, _init: bool = False) -> None:
        """Run the patch encoder as `n` concurrent window groups (drops a captured graph)."""
        self.patch_groups = window_groups(n)
        self.gstreams = [torch.cuda.Stream(device=self.dev) for _ in self.patch_groups[1:]]
        self.ws_groups = [ops.gemm_workspace(self.dev) for _ in self.patch_groups[1:]]
        if not _init:
            self.graph = None
            wss = [self.ws_main, self.ws_side, self.ws_side2, self.ws_dec] + self.ws_groups
            self._err_dev = [w[ops.WS_ERROR_OFFSET:ops.WS_ERROR_OFFSET + 4].view(torch.int32) for w in wss]
            self._err_host = torch.zeros(len(wss), dtype=torch.int32, pin_memory=True)
            self._err_ev = None

    def _patch_groups(self, main) -> None:
        """The patch encoder as independent window groups, group g on stream g (group 0 on
        `main`); each merges its own windows' share of the hooked block outputs."""
        vp = self.vp
        for g, (w0, w1) in enumerate(self.patch_groups):
            serial = self.serial_side or g == 0
            st = main if serial else self.gstreams[g - 1]
            ws = self.ws_main if serial else self.ws_groups[g - 1]
            if st is not main:
                st.wait_stream(main)
            lo, hi = min(w0, 25), min(w1, 25)   # their windows in the 5 x 5 hook grid
            hooks = {}
            if lo < hi:
                hooks = {5: lambda lo=lo, hi=hi: ops.merge_windows(vp.x, 0, 5, 3, self.lat0, windows=(lo, hi)),
                         11: lambda lo=lo, hi=hi: ops.merge_windows(vp.x, 0, 5, 3, self.lat1, windows=(lo, hi))}
            with torch.cuda.stream(st), ops.use_workspace(ws):
                self._vit("encoder.patch_encoder.", _Rows(vp, w0 * TOK, w1 * TOK), w1 - w0, w0 * PTOK, hooks)
        if not self.serial_side:
            for st in self.gstreams:
                main.wait_stream(st)

    # -------------------------------------------------------------- forward
    def _image_encoder_iter(self):
        """_image_encoder as a generator (one step per ViT block, the tail after the last)."""
        P, e = self.P, "encoder."
        yield from self._vit_iter("encoder.image_encoder.", self.vi, 1, 34 * PTOK)
        ops.merge_windows(self.vi.out, 0, 1, 0, self.g)
        self._deconv(self.g, 24, D, P[e + "upsample_lowres.w"], self.cat, D, bias=P[e + "upsample_lowres.b"],
                     C_off=D, ldc=2 * D)

    def _fov_encoder_iter(self):
        vf, P = self.vf, self.P
        yield from self._vit_iter("fov.encoder.0.", vf, 1, 34 * PTOK)
        ops.gemm(vf.out, P["fov.lin.w"], self.fov_tok, M=PTOK, N=128, K=D, A_off=D, bias=P["fov.lin.b"])

    def _image_encoder(self):
        """Image encoder (+ lowres upsample): ~2.5 % of the frame's FLOPs at M = 577
        rows, far too few tiles to fill 256 CUs alone, so it runs on a side stream
        beside the patch encoder."""
        P, e = self.P, "encoder."
        self._vit("encoder.image_encoder.", self.vi, 1, 34 * PTOK)
        ops.merge_windows(self.vi.out, 0, 1, 0, self.g)
        self._deconv(self.g, 24, D, P[e + "upsample_lowres.w"], self.cat, D, bias=P[e + "upsample_lowres.b"],
                     C_off=D, ldc=2 * D)

    def _fov_encoder(self):
        """FOV encoder ViT + Linear (fov.py:45-47, 66-72)."""
        vf, P = self.vf, self.P
        self._vit("fov.encoder.0.", vf, 1, 34 * PTOK)
        ops.gemm(vf.out, P["fov.lin.w"], self.fov_tok, M=PTOK, N=128, K=D, A_off=D, bias=P["fov.lin.b"])

    def _fov_head(self):
        """FOV head (fov.py:56-82): needs the low-res decoder features and the FOV tokens."""
        P = self.P
        self._conv3(self.low, 48, 256, P["fov.down.w"], self.fx, 128, bias=P["fov.down.b"], act=DP_ACT_RELU,
                    R1=self.fov_tok, stride=2)
        self._conv3(self.fx, 24, 128, P["fov.h0.w"], self.f12, 64, bias=P["fov.h0.b"], act=DP_ACT_RELU, stride=2)
        self._conv3(self.f12, 12, 64, P["fov.h2.w"], self.f6, 32, bias=P["fov.h2.b"], act=DP_ACT_RELU, stride=2)
        ops.fov_tail(self.f6, P["fov.h4.w"], P["fov.h4.b"], self.fov_deg)

    def forward(self, phase: str = "all") -> Tuple[torch.Tensor, torch.Tensor]:
        """Run the network on `self.x0`; results in self.canonical / self.fov_deg.

        `phase` splits the forward for the frame pipeline (depth_pro.pipeline): "side" = window
        im2col + the image and FOV encoders, "enc" = the patch encoder, "dec" = everything after
        it; the caller orders them (side before dec, enc before dec).  "all" = the whole frame."""
        if phase not in ("all", "side", "enc", "dec"):
            raise DPError(f"unknown forward phase {phase!r}")
        with ops.use_workspace(self.ws_main):
            return self._forward(phase)

    def _forward(self, phase: str = "all") -> Tuple[torch.Tensor, torch.Tensor]:
        """Body of `forward`.

        Two streams: the current stream runs the patch encoder -> decoder -> head;
        `self.side` runs the image encoder beside the patch encoder (forked after
        the window im2col, joined before fuse_lowres), then -- `fov_late` -- the
        FOV encoder + FOV head beside the decoder (forked once the low-res
        decoder features exist, joined at the end), so that only one M = 577
        encoder competes with the patch encoder's full-chip GEMMs.
        """
        P = self.P
        main = torch.cuda.current_stream(self.dev)
        side_ok = "side" not in _ABLATE
        serial = self.serial_side or self.side_mode == "serial"
        fov_side = self.use_fov and self.fov_late and not serial
        if phase != "all" and (serial or fov_side or self.side_mode != "concurrent" or len(self.patch_groups) != 1):
            raise DPError("forward phases need the default schedule (concurrent side encoders, one window group)")
        if phase in ("all", "side"):
            ops.patchify_pyramid(self.x0, self.cols)
        if phase == "side":
            # the image encoder on this stream, the FOV encoder on side2, joined before returning
            with ops.use_workspace(self.ws_side):
                self._image_encoder()
            if self.use_fov:
                self.side2.wait_stream(main)
                with torch.cuda.stream(self.side2), ops.use_workspace(self.ws_side2):
                    self._fov_encoder()
                main.wait_stream(self.side2)
            return self.canonical, self.fov_deg

        def side_encoders():
            if serial:
                self._image_encoder()
                if self.use_fov:
                    self._fov_encoder()
                return
            self.side.wait_stream(main)
            with torch.cuda.stream(self.side), ops.use_workspace(self.ws_side):
                if side_ok and "img" not in _ABLATE:
                    self._image_encoder()
                if side_ok:
                    if self.use_fov and not fov_side and self.side_streams == 1:
                        self._fov_encoder()
            if self.use_fov and not fov_side and self.side_streams == 2 and fov_at < 0:
                fov_encoder_side2()

        def fov_encoder_side2():
            self.side2.wait_stream(main)
            with torch.cuda.stream(self.side2), ops.use_workspace(self.ws_side2):
                if side_ok and "fovenc" not in _ABLATE:
                    self._fov_encoder()

        # DP_FOV_AT=b (A/B): start the FOV encoder after patch-encoder block b instead of with the
        # image encoder (it is needed only at the FOV head, after the decoder's first conv)
        fov_at = self.fov_at if (self.use_fov and not fov_side and self.side_streams == 2 and not serial
                                 and len(self.patch_groups) == 1) else -1
        # DP_SIDE_SYNC (A/B): the side encoders step one block per patch-encoder block, each step
        # beside that block's fc1 (multi-round, its last round leaves CUs free) and joined before
        # its fc2, so they never hold CUs when a one-round proj / fc2 launches
        sync = (self.side_sync and phase == "all" and not serial and not fov_side and self.side_mode == "concurrent"
                and self.side_streams == 2 and self.use_fov and side_ok and fov_at < 0 and len(self.patch_groups) == 1)
        side_its = None
        if sync:
            side_its = [(self.side, self.ws_side, self._image_encoder_iter()),
                        (self.side2, self.ws_side2, self._fov_encoder_iter())]

            def side_step(i):
                for st, ws, it in side_its:
                    st.wait_stream(main)
                    with torch.cuda.stream(st), ops.use_workspace(ws):
                        next(it)

            def side_join(i):
                main.wait_stream(self.side)
                main.wait_stream(self.side2)
        elif phase == "all" and (self.side_mode != "late" or serial):
            side_encoders()
        vp = self.vp
        if phase == "dec":
            pass
        elif len(self.patch_groups) == 1:
            hooks = {
                5: lambda: ops.merge_windows(vp.x, 0, 5, 3, self.lat0),
                11: lambda: ops.merge_windows(vp.x, 0, 5, 3, self.lat1),
            }
            if fov_at >= 0:
                prev = hooks.get(fov_at)
                hooks[fov_at] = (lambda: (prev(), fov_encoder_side2())) if prev else fov_encoder_side2
            if sync:
                self._vit("encoder.patch_encoder.", vp, NWIN, 0, hooks, ln_fuse=True, pre_fc1=side_step,
                          pre_fc2=side_join)
                for st, ws, it in side_its:          # the side encoders' final norm and tails
                    with torch.cuda.stream(st), ops.use_workspace(ws):
                        for _ in it:
                            pass
            else:
                self._vit("encoder.patch_encoder.", vp, NWIN, 0, hooks, ln_fuse=True)
        else:
            self._patch_groups(main)
        if phase != "dec":
            ops.merge_windows(vp.out, 0, 5, 3, self.f0)
            ops.merge_windows(vp.out, 25, 3, 6, self.f1)
            ops.merge_windows(vp.out, 34, 1, 0, self.f2)
        if phase == "enc":
            return self.canonical, self.fov_deg
        if self.side_mode == "late" and not serial:
            side_encoders()
        # project / upsample (encoder.py:314-324)
        e = "encoder."
        par = self.dec_streams and not serial and not fov_side

        def lat0_pre():
            ops.gemm(self.lat0, P[e + "upsample_latent0.0"], self.t96_256, M=96 * 96, N=256, K=D)
            self._deconv(self.t96_256, 96, 256, P[e + "upsample_latent0.1"], self.t192_256, 256)
            self._deconv(self.t192_256, 192, 256, P[e + "upsample_latent0.2"], self.t384_256, 256)

        def lat0_last():   # 384^2 -> 768^2: 2304 tiles of K = 256, the stream-K engine's best case
            self._deconv(self.t384_256, 384, 256, P[e + "upsample_latent0.3"], self.enc0, 256)

        def lat0_chain():
            lat0_pre()
            lat0_last()

        def lat1_chain():
            ops.gemm(self.lat1, P[e + "upsample_latent1.0"], self.t96_256b, M=96 * 96, N=256, K=D)
            self._deconv(self.t96_256b, 96, 256, P[e + "upsample_latent1.1"], self.t192_256b, 256)
            self._deconv(self.t192_256b, 192, 256, P[e + "upsample_latent1.2"], self.enc1, 256)

        def f1_chain():
            ops.gemm(self.f1, P[e + "upsample1.0"], self.t48_1024, M=48 * 48, N=D, K=D)
            self._deconv(self.t48_1024, 48, D, P[e + "upsample1.1"], self.enc3, D)

        def f0_chain():
            ops.gemm(self.f0, P[e + "upsample0.0"], self.t96_512, M=96 * 96, N=512, K=D)
            self._deconv(self.t96_512, 96, 512, P[e + "upsample0.1"], self.enc2, 512)

        enc_ev = {}
        if par:
            # The latent chains and the f0 / f1 chains (small grids, ~0.6 ms in a row) beside the
            # main stream's f2 chain -> fuse_lowres -> convs.4, in the order the decoder's
            # projections need their outputs (enc3, enc2, enc1; enc0 last).  Side streams issue no
            # stream-K launch that could overlap one of the main stream's (workgroups that wait on
            # each other, dp_mi355x.h): no workspace here.
            lat0_sk = self.lat0_sk
            for st, chains in ((self.dec_a, (("enc0pre", lat0_pre) if lat0_sk else ("enc0", lat0_chain),)),
                               (self.dec_b, (("enc3", f1_chain), ("enc2", f0_chain), ("enc1", lat1_chain)))):
                st.wait_stream(main)
                with torch.cuda.stream(st), ops.use_workspace(None):
                    for name, chain in chains:
                        chain()
                        enc_ev[name] = torch.cuda.Event()
                        enc_ev[name].record(st)
        else:
            lat0_chain()
            lat1_chain()
            f0_chain()
            f1_chain()
        ops.gemm(self.f2, P[e + "upsample2.0"], self.t24_1024, M=24 * 24, N=D, K=D)
        self._deconv(self.t24_1024, 24, D, P[e + "upsample2.1"], self.cat, D, ldc=2 * D)
        if not serial and phase == "all":
            main.wait_stream(self.side)  # join: image-encoder half of `cat` and fov tokens ready
        ops.gemm(self.cat, P[e + "fuse_lowres.w"], self.enc4, M=48 * 48, N=D, K=2 * D, bias=P[e + "fuse_lowres.b"])
        # decoder (decoder.py:74-93)
        self._conv3(self.enc4, 48, D, P["decoder.convs.4"], self.low, 256)
        if par:
            # FOV head (fov.py:56-82; needs only the low-res features) on the FOV encoder's stream,
            # off the main stream's critical path (its 24^2 - 6^2 convs leave the chip idle)
            if self.use_fov:
                self.side2.wait_stream(main)
                with torch.cuda.stream(self.side2), ops.use_workspace(self.ws_side2):
                    self._fov_head()
            # convs.3 / .2 / .1 (the encoder features' projections, decoder.py:74-93) on dec_c in
            # the order the fusions need them, each beside the previous fusion block: after
            # convs.4 (the main stream's last stream-K launch before fusion 1's deconv, which
            # waits for convs.1), so dec_c's stream-K launches never overlap the main stream's
            self.dec_c.wait_stream(main)
            evs = {}
            with torch.cuda.stream(self.dec_c), ops.use_workspace(self.ws_dec):
                for i, (enc, s_, cin) in ((3, (self.enc3, 96, D)), (2, (self.enc2, 192, 512)),
                                          (1, (self.enc1, 384, 256))):
                    self.dec_c.wait_event(enc_ev[f"enc{i}"])
                    self._conv3(enc, s_, cin, P[f"decoder.convs.{i}"], self.dec[s_]["c"], 256)
                    evs[i] = torch.cuda.Event()
                    evs[i].record(self.dec_c)
                # the lat0 chain's last deconv (on stream-K: 164 vs 446 us data-parallel) here, on the
                # stream-K side stream; the main stream waits for it before fusion 1, whose deconv
                # is its next stream-K launch
                if lat0_sk:
                    self.dec_c.wait_event(enc_ev["enc0pre"])
                    lat0_last()
                    enc_ev["enc0"] = torch.cuda.Event()
                    enc_ev["enc0"].record(self.dec_c)
        elif self.use_fov and not fov_side:  # FOV head (fov.py:56-82) only needs the lowres features
            if self.side_streams == 2 and not serial and phase == "all":
                main.wait_stream(self.side2)
            self._fov_head()
        elif fov_side:
            self.side.wait_stream(main)
            with torch.cuda.stream(self.side), ops.use_workspace(self.ws_side):
                if side_ok:
                    self._fov_encoder()
                    self._fov_head()
        if "decoder" not in _ABLATE:
            f = self._fusion(4, self.low, 48, None)
            for i, (enc, s, cin) in ((3, (self.enc3, 96, D)), (2, (self.enc2, 192, 512)), (1, (self.enc1, 384, 256))):
                c = self.dec[s]["c"]
                if par:
                    main.wait_event(evs[i])
                    if i == 1:
                        main.wait_event(enc_ev["enc0"])
                else:
                    self._conv3(enc, s, cin, P[f"decoder.convs.{i}"], c, 256)
                f = self._fusion(i, f, s, c)
            if par:
                main.wait_event(enc_ev["enc0"])     # lat0 chain for fusion 0
            feats = self._fusion(0, f, 768, self.enc0)
        else:
            feats = self.feats
        if par:
            main.wait_stream(self.dec_a)
            main.wait_stream(self.dec_b)
            main.wait_stream(self.dec_c)
            if self.use_fov:
                main.wait_stream(self.side2)
        if fov_side:
            main.wait_stream(self.side)
        if "head" in _ABLATE:
            return self.canonical, self.fov_deg
        # head (depth_pro.py:182-207): conv3x3, then deconv -> conv3x3 -> ReLU -> 1x1 -> ReLU as ONE
        # composed 3x3 conv over h0 with a pixel-shuffle + fused 1x1 epilogue (compose_head)
        if self.head0_compose and "decoder" not in _ABLATE:
            self._conv3(feats, 768, 256, P["head.0c.w"], self.h0, 128, bias=P["head.0c.b"],
                        border_corr=P["head.0c.corr"])
        else:
            self._conv3(feats, 768, 256, P["head.0.w"], self.h0, 128, bias=P["head.0.b"])
        ops.gemm(self.h0, P["head.ps.w"], self.canonical, M=768 * 768, N=128, K=9 * 128,
                 conv=dict(in_h=768, in_w=768, in_c=128, k=3, stride=1, pad=1, out_h=768, out_w=768),
                 bias=P["head.ps.b"], head_w=P["head.4.w"], head_b=P["head.4.b"], head_corr=P["head.ps.corr"])
        return self.canonical, self.fov_deg

    # ---------------------------------------------------------------- graphs
    def capture_graph(self) -> None:
        """Capture `forward` into a HIP graph (static shapes); replay with `run`."""
        s = torch.cuda.Stream(device=self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            self.forward()  # warm-up outside capture (first-launch code object loads)
        torch.cuda.current_stream(self.dev).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.forward()
        self.graph = g

    def run(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """One forward (graph replay if captured).  Raises DPError if an EARLIER forward's
        stream-K hand-off timed out (or this one's, with DP_CHECK_SYNC=1)."""
        self.check_status(block=False)
        if self.graph is not None:
            self.graph.replay()
        else:
            self.forward()
        self._stage_status()
        if self.sync_check:
            self.check_status(block=True)
        return self.canonical, self.fov_deg

    def _stage_status(self) -> None:
        for i, w in enumerate(self._err_dev):
            self._err_host[i:i + 1].copy_(w, non_blocking=True)
        self._err_ev = torch.cuda.Event()
        self._err_ev.record()

    def check_status(self, block: bool = True) -> None:
        """Raise DPError if a stream-K GEMM of a forward run so far gave up waiting for a
        partial tile (its output -- that frame's depth -- is wrong).  block=False only looks
        at read-backs that have already landed (no synchronisation)."""
        ev = self._err_ev
        if ev is None:
            return
        if block:
            ev.synchronize()
        elif not ev.query():
            return
        self._err_ev = None
        if int(self._err_host.abs().sum()) != 0:
            self._err_host.zero_()
            for w in [self.ws_main, self.ws_side, self.ws_side2, self.ws_dec] + self.ws_groups:
                w.zero_()   # error word, and any hand-off flag the timed-out launch left set
            raise DPError("dp_gemm: a stream-K partial-tile or fused-LayerNorm row-band hand-off timed out; "
                          "the depth map of a recent frame is invalid (workspace error word set)")
