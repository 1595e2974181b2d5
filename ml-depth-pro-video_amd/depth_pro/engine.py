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
from ._lib import (DP_ACT_GELU, DP_ACT_RELU, DP_BF16, DP_F16, DP_F32, DP_TILE_P8PH_256x256, DP_TILE_SPLITK_256x256,
                   DPError, load)
from .spec import DEPTH, EMBED_DIM, HEADS, IMG_SIZE, MLP_DIM, TOKENS

# Timing ablations for tools/frame_ablation.py only (results are wrong when set):
# comma list of {side, attn, ln, vitgemm, decoder, head}.
_ABLATE = set(filter(None, os.environ.get("DP_ABLATE", "").split(",")))


def ln_fold_enabled() -> bool:
    """Whether the patch encoder runs with its LayerNorms folded into qkv / fc1: always,
    except under the 'ln' / 'vitgemm' timing ablations -- those drop the standalone LayerNorms / the
    ViT GEMMs, which only the unfolded path has as separate launches.  Read once at
    pack time: the packed set holds only the weights of the path chosen here."""
    return not ({"ln", "vitgemm"} & _ABLATE)


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
    fold = ln_fold_enabled()
    for vit in ("encoder.patch_encoder.", "encoder.image_encoder.", "fov.encoder.0."):
        if vit + "cls_token" not in sd:
            continue
        # the patch encoder with its LayerNorms folded reads only the folded qkv / fc1 (below): the
        # unfolded ones (350 MB of 16-bit weights) are not packed
        folded = fold and vit == "encoder.patch_encoder."
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
                if folded and n in ("attn.qkv.weight", "mlp.fc1.weight"):
                    continue
                P[b + n] = g(b + n).to(vdt).contiguous()
        P[vit + "norm.weight"] = _f32(g(vit + "norm.weight"))
        P[vit + "norm.bias"] = _f32(g(vit + "norm.bias"))
        if folded:
            # norm1 / norm2 folded into the qkv / fc1 that consume them (ops.fold_layernorm): the
            # patch encoder's residual GEMMs hand the next Linear 16-bit rows + chunk statistics
            # instead of a LayerNorm pass (Engine._vit); the qkv's log2q gamma rides
            # in the folded weights
            qg = ops.log2q_gamma(HEADS, D // HEADS, device)
            for i in range(DEPTH):
                b = f"{vit}blocks.{i}."
                for lin, ln, cs in (("attn.qkv", "norm1", qg), ("mlp.fc1", "norm2", None)):
                    wf, bf, sf = ops.fold_layernorm(g(b + lin + ".weight").float(), g(b + lin + ".bias").float(),
                                                    g(b + ln + ".weight").float(), g(b + ln + ".bias").float(),
                                                    vdt, cs)
                    P[b + lin + ".fold.w"], P[b + lin + ".fold.b"], P[b + lin + ".fold.s"] = wf, bf, sf
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
    def __init__(self, rows: int, dt, dev, out_dt=None, ln_fold: bool = False):
        self.rows = rows
        self.x = torch.empty(rows, D, dtype=torch.float32, device=dev)
        # folded LayerNorm: (mean, M2) of each 128-column chunk of the rows in `h` (un-normalised)
        self.part = torch.empty(rows, D // 128, 2, dtype=torch.float32, device=dev) if ln_fold else None
        self.h = torch.empty(rows, D, dtype=dt, device=dev)
        # folded path: the residual stream between blocks is split, x = h (16 bits) + an 8-bit low
        # part xl (steps of ulp(h) / 256; the proj / fc2 epilogues read and update both, dp_gemm's
        # ln_xl); `x` (fp32) holds it only where an fp32 reader needs it (the patch embed's output, the
        # hooks, the final norm)
        self.xl = torch.empty(rows, D, dtype=torch.int8, device=dev) if ln_fold else None
        # (ABI 13): every row's (rstd, -rstd * mean), merged by the proj / fc2 producers' last
        # workgroup per row tile for the qkv / fc1 consumers on the persistent engine; padded to whole
        # 256-row tiles, the rows the consumer's constant-slot DMA reads
        self.rs = (torch.empty((rows + 255) // 256 * 256, 2, dtype=torch.float32, device=dev)
                   if ln_fold else None)
        self.qkv = torch.empty(rows, 3 * D, dtype=dt, device=dev)
        self.a = torch.empty(rows, D, dtype=dt, device=dev)
        self.m = torch.empty(rows, MLP_DIM, dtype=dt, device=dev)
        # final-norm output (the encoder features) in the decoder's type; it reuses the
        # attention-output buffer, which is dead once the last block has run
        out_dt = out_dt or dt
        self.out = self.h if out_dt == dt else self.a.view(out_dt)


class _ViTRows:
    """Rows [lo, hi) of a _ViTBuffers (one encoder of the grouped side pair)."""

    def __init__(self, buf: _ViTBuffers, lo: int, hi: int):
        self.rows = hi - lo
        self.x = buf.x[lo:hi]
        self.out = buf.out[lo:hi]


class FrameStatus:
    """Health of ONE forward, read without stalling the stream that ran it.

    The forward ends with `dp_gemm_workspace_check` per GEMM workspace: the frame's error word
    (a stream-K partial-tile hand-off that timed out) goes to the engine's status buffer and a set
    word is cleared with every hand-off flag, so the next frame starts clean and reports only its
    own launches.  `DepthPro.infer` adds a non-finite-output count from its epilogue kernel
    (depth or focal length NaN / inf, e.g. an f16 overflow in the decoder), and
    `Engine.finish_status` copies the words into pinned host memory on the same stream.
    `check()` waits for that frame's copy only and raises DPError if the frame is bad, so a caller
    that checks before writing a frame's files drops exactly the bad frame (generate_depth_maps,
    depth-pro-run).  A status is reported once: after `check()` (or `Engine.check_status`) has
    seen it, later `check_status` sweeps skip it.  A caller that takes a frame's status to check it
    itself later (`claim()`, the frame loop's writer threads) OWNS it: the engine-wide sweep then
    never reports that frame, so it is reported (and dropped) by its owner only -- not also by
    whichever `infer` call happens to run after it finished."""

    def __init__(self, frame: int, words: torch.Tensor, event: torch.cuda.Event):
        self.frame = frame
        self.words = words            # pinned int32: [workspace error words..., non-finite count]
        self.event = event
        self.reported = False
        self.owned = False            # claimed by a caller that checks it itself (claim)

    def ready(self) -> bool:
        return self.event.query()

    def error(self) -> Optional[str]:
        """None if the frame is good, else why not (synchronises on this frame's event)."""
        self.event.synchronize()
        w = self.words.tolist()
        if any(w[:-1]):
            return ("dp_gemm: a stream-K partial-tile hand-off timed out in this forward "
                    "(workspace error word set): its depth map is invalid")
        if w[-1]:
            return f"{w[-1]} non-finite depth / focal-length value(s) in this frame's output"
        return None

    def check(self) -> None:
        msg = self.error()
        self.reported = True
        if msg is not None:
            raise DPError(f"frame {self.frame}: {msg}")

    def claim(self) -> "FrameStatus":
        """Take ownership (see the class doc): the engine's sweep no longer reports this frame."""
        self.owned = True
        return self


class BatchStatus:
    """The FrameStatus of every frame of one `DepthPro.infer` / `forward` call, as one status:
    bad if any frame is; `check()` raises naming every bad frame (last_status() of a batched call)."""

    def __init__(self, frames: list):
        self.frames = list(frames)
        self.frame = self.frames[-1].frame if self.frames else -1

    @property
    def reported(self) -> bool:
        return all(f.reported for f in self.frames)

    def ready(self) -> bool:
        return all(f.ready() for f in self.frames)

    def claim(self) -> "BatchStatus":
        """Take ownership of these frames' health: the caller promises to `check()` this status
        itself (e.g. in a writer thread after the frame's event), so the engine's non-blocking
        sweep at the next `infer` / `forward` never reports them (a bad frame is dropped once, by
        its owner, and the next frame is not dropped in its place).  Returns self."""
        for f in self.frames:
            f.owned = True
        return self

    def error(self) -> Optional[str]:
        bad = [(f.frame, e) for f in self.frames for e in [f.error()] if e is not None]
        if not bad:
            return None
        return "; ".join(f"frame {n}: {e}" for n, e in bad)

    def check(self) -> None:
        msg = self.error()
        for f in self.frames:
            f.reported = True
        if msg is not None:
            raise DPError(msg)


class Engine:
    """One frame (batch 1) per forward; static workspace (~4 GB).

    Streams (`_forward`): the main stream runs patchify -> patch encoder -> merges -> decoder ->
    head; `side` runs the image and FOV encoders beside the patch encoder, as ONE grouped ViT
    (M = 577 rows each: far too few tiles to fill the chip alone, and paired, half the launches
    with twice the workgroups each); after the patch encoder the
    project/upsample chains run on `dec_a` / `dec_b` and the decoder's encoder-feature projections,
    the lat0 chain's last deconv and the FOV head on `dec_c`, beside the main stream's decoder.
    At most four streams carry work at any time (HIP's default of four hardware queues per
    process).  `serial_side = True` (profiling: bench.py's per-launch timing) issues everything
    on the current stream in one order."""

    def __init__(self, packed: Dict[str, object], device: torch.device, dtype_code,
                 use_fov: bool = True):
        load()
        if device.type != "cuda":
            raise DPError("the MI355X Depth Pro engine needs a ROCm/HIP device")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
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
        # patch encoder LayerNorms folded into its GEMMs (pack_weights, _vit): whichever path the packed
        # set was made for (DP_LN_FOLD / ablations at pack time, ln_fold_enabled)
        self.ln_fold = "encoder.patch_encoder.blocks.0.attn.qkv.fold.w" in packed
        if self.ln_fold != ln_fold_enabled():
            raise DPError("packed weights were made for the other LayerNorm path (DP_ABLATE differs from "
                          "when they were packed)")
        self.vp = _ViTBuffers(NWIN * TOK, vdt, dev, dt, ln_fold=self.ln_fold)     # patch encoder (35 windows)
        # image + FOV encoders, run as one grouped ViT (rows 0..576 image, 577..1153 FOV)
        self.side_vits = ["encoder.image_encoder."] + (["fov.encoder.0."] if self.use_fov else [])
        self.vs = _ViTBuffers(len(self.side_vits) * TOK, vdt, dev, dt)
        self.vi = _ViTRows(self.vs, 0, TOK)
        self.vf = _ViTRows(self.vs, TOK, 2 * TOK) if self.use_fov else None
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
        self.side = torch.cuda.Stream(device=dev)      # image + FOV encoders (grouped)
        self.dec_a = torch.cuda.Stream(device=dev)     # lat0 project/upsample chain
        self.dec_b = torch.cuda.Stream(device=dev)     # f1 / f0 / lat1 chains
        self.dec_c = torch.cuda.Stream(device=dev)     # decoder projections, lat0's last deconv, FOV head
        # stream-K GEMM scratch, one per stream that issues stream-K GEMMs (main / dec_c); the side
        # encoders' and the dec_a / dec_b chains' GEMMs never take the stream-K engine (no
        # workspace), so no two launches whose workgroups wait on each other run at once
        self.ws_main = ops.gemm_workspace(dev)
        self.ws_dec = ops.gemm_workspace(dev)
        # decoder out_conv composed into the head's first conv (compose_head0); DP_HEAD0_COMPOSE=0:
        # separate (the per-stage parity test reads fusion 0's output on that path)
        self.head0_compose = os.environ.get("DP_HEAD0_COMPOSE", "1") == "1" and "head.0c.w" in packed
        # softmax scale * log2(e) folded into the qkv epilogue (per-column gamma on Q) so that attention
        # takes one exp2 per score (dp_attention_log2q)
        self.qkv_gamma = ops.log2q_gamma(HEADS, D // HEADS, dev)
        self.serial_side = False   # True: every launch on the current stream, in one order (profiling)
        # device status of the current frame: [error word of each workspace (forward's end),
        # non-finite output count (the infer epilogue)]
        self._wss = [self.ws_main, self.ws_dec]
        self.status_dev = torch.zeros(len(self._wss) + 1, dtype=torch.int32, device=dev)
        self._frames = 0
        self._recent: list = []           # FrameStatus of the frames not checked yet (check_status)
        self._unreported: list = []       # finished bad frames owed to the next check_status
        self.last_status: Optional[FrameStatus] = None
        self.sync_check = os.environ.get("DP_CHECK_SYNC", "0") == "1"
        # the decoder's convs.4 (1024 -> 256 3x3 at 48^2: 9 tiles) on the split-K engine: 103 -> 41 us
        # alone, +0.23 / +0.12 / +0.09 fps in three same-box A/Bs; convs.3, upsample2.0, fuse_lowres or
        # the fusions' 48^2 / 96^2 ResidualBlock convs there too did not gain (profiles/r05ah_splitk_dec/)
        # -- depth rel-L1 8.741e-4 -> 8.769e-4
        # the patch encoder's folded qkv on the persistent 8-phase engine, as fc1: 948 tiles of 256 x 256
        # over 256 workgroups instead of 3 rounds of 320 x 256 tiles, each tile's epilogue under the next
        # one's K loop: 48.41 / 48.27 -> 49.14 / 49.06 fps same box (profiles/r05i_qkv_p8ph/)
        self.qkv_tile = DP_TILE_P8PH_256x256

    # ------------------------------------------------------------------ ViT
    def _vit(self, pres, buf: _ViTBuffers, n_img: int, cols_off_rows: int, hooks=None):
        """timm forward_features (vit_factory.py:97-99 -> vision_transformer.py): patch embed + cls /
        pos, 24 Blocks, final norm; `hooks[i]()` runs after block i (encoder.py:133-144)."""
        for _ in self._vit_steps(pres, buf, n_img, cols_off_rows, hooks):
            pass

    def _vit_steps(self, pres, buf: _ViTBuffers, n_img: int, cols_off_rows: int, hooks=None):
        """`_vit` as a generator: yields after the embedding and after each Block (the final norm
        runs on the last step) -- lets a caller issue another stream's ViT block by block.

        `pres`: the weight prefixes of G ViTs of one shape over the same im2col rows (G = 2: the
        image and FOV encoders, encoder.py:308-311 and fov.py:66-72); ViT g owns rows
        [g * n_img * 577, (g + 1) * n_img * 577) of `buf`, and every op runs as ONE grouped launch
        for the G of them (dp_gemm_grouped / dp_layernorm_grouped, attention over G * n_img)."""
        P, M = self.P, n_img * TOK
        G = len(pres)
        # ablations (A/B timing only): 'ln' / 'vitgemm' everywhere; 'sideln': the grouped side pair's
        # LayerNorm launches only (is the side chain's latency on the frame's critical path?)
        ln_on = "ln" not in _ABLATE and not (G > 1 and "sideln" in _ABLATE)
        gemm_on = "vitgemm" not in _ABLATE

        def lin(A, key, C, N, K, a_rows=True, **kw):
            """The G problems' `key` Linear: A rows / C rows of problem g at g * M (A shared when
            not a_rows); per-problem bias / gamma / pos given as key suffixes in kw."""
            per = {k: kw.pop(k) for k in ("bias", "gamma", "pos") if isinstance(kw.get(k), str)}
            A_off = kw.pop("A_off", 0)
            groups = []
            for g, pre in enumerate(pres):
                d = dict(A=A, B=P[pre + key], C=C, A_off=A_off + (g * M * K if a_rows else 0), C_off=g * M * N)
                d.update({k: P[pre + v] for k, v in per.items()})
                groups.append(d)
            ops.gemm_grouped(groups, M=kw.pop("M", M), N=N, K=K, **kw)

        def norm(key, out):
            ops.layernorm_grouped(buf.x, [P[pre + key + ".weight"] for pre in pres],
                                  [P[pre + key + ".bias"] for pre in pres], out, M, D)

        # patch embed (k16 s16 conv as GEMM over the im2col rows) + bias + pos -> rows 1..576
        lin(self.cols, "pe.w", buf.x, D, 768, a_rows=False, M=n_img * PTOK, A_off=cols_off_rows * 768,
            bias="pe.b", pos="pos", ldpos=D, pos_group=PTOK, pos_off=1, row_group=PTOK, row_group_out=TOK,
            row_off=1)
        for g, pre in enumerate(pres):
            ops.vit_cls_rows(buf.x[g * M:], P[pre + "cls"], P[pre + "pos"], n_img)
        if G == 1 and buf.part is not None:
            yield from self._vit_blocks_folded(pres[0], buf, M, hooks)
            return
        yield
        for i in range(DEPTH):
            b = f"blocks.{i}."
            if ln_on:
                norm(b + "norm1", buf.h)
            if gemm_on:
                lin(buf.h, b + "attn.qkv.weight", buf.qkv, 3 * D, D, bias=b + "attn.qkv.bias", gamma=self.qkv_gamma)
            if "attn" not in _ABLATE:
                ops.attention(buf.qkv, buf.a, G * n_img, TOK, HEADS, D // HEADS, log2q=True)
            if gemm_on:
                lin(buf.a, b + "attn.proj.weight", buf.x, D, D, bias=b + "attn.proj.bias", gamma=b + "ls1.gamma",
                    accumulate=True)
            if ln_on:
                norm(b + "norm2", buf.h)
            if gemm_on:
                lin(buf.h, b + "mlp.fc1.weight", buf.m, MLP_DIM, D, bias=b + "mlp.fc1.bias", act=DP_ACT_GELU)
            if gemm_on:
                lin(buf.m, b + "mlp.fc2.weight", buf.x, D, MLP_DIM, bias=b + "mlp.fc2.bias", gamma=b + "ls2.gamma",
                    accumulate=True)
            if hooks and i in hooks:
                hooks[i]()
            if i == DEPTH - 1:
                norm("norm", buf.out)
            yield

    def _vit_blocks_folded(self, pre: str, buf: _ViTBuffers, M: int, hooks=None):
        """The 24 Blocks with norm1 / norm2 folded across the GEMM boundary (dp_gemm_args.ln_*):
        `h` carries the un-normalised residual rows in 16 bits and `part` their 128-column chunk
        statistics, written by the producer (block 0: dp_layernorm_stats; then every proj / fc2
        epilogue beside its split-residual update); qkv / fc1 run on the folded weights
        (ops.fold_layernorm) and apply LN's per-row mean / rstd in their epilogue.  Same
        arithmetic as LN -> Linear up to where the 16-bit rounding falls (x instead of LN(x);
        tools/ln_fold_emul.py: rel-L1 vs fp32 unchanged, 2.377e-3 vs 2.379e-3 bf16).  A generator
        like _vit_steps."""
        P = self.P
        n_img = M // TOK
        # the stream enters as fp32 (patch embed + cls rows): split it into h + xl, with the stats
        ops.layernorm_stats(buf.x, buf.h, buf.part, M, D, xl=buf.xl)
        yield
        qkv_tile = self.qkv_tile
        rs = buf.rs       # producer-merged row statistics (ABI 13), for the persistent consumers
        for i in range(DEPTH):
            b = f"{pre}blocks.{i}."
            rs_q = rs if i > 0 else None     # block 0: the stats pass wrote `part` only
            ops.gemm(buf.h, P[b + "attn.qkv.fold.w"], buf.qkv, M=M, N=3 * D, K=D, bias=P[b + "attn.qkv.fold.b"],
                     ln_in=(None if rs_q is not None else buf.part, P[b + "attn.qkv.fold.s"]), ln_rs_in=rs_q,
                     tile=qkv_tile)
            if "attn" not in _ABLATE:
                ops.attention(buf.qkv, buf.a, n_img, TOK, HEADS, D // HEADS, log2q=True)
            ops.gemm(buf.a, P[b + "attn.proj.weight"], None, M=M, N=D, K=D,
                     bias=P[b + "attn.proj.bias"], gamma=P[b + "ls1.gamma"], accumulate=True,
                     ln_out=(buf.h, buf.part), ln_xl=buf.xl, ln_rs_out=rs)
            ops.gemm(buf.h, P[b + "mlp.fc1.fold.w"], buf.m, M=M, N=MLP_DIM, K=D, bias=P[b + "mlp.fc1.fold.b"],
                     act=DP_ACT_GELU, ln_in=(None, P[b + "mlp.fc1.fold.s"]), ln_rs_in=rs)
            last = i == DEPTH - 1    # the final norm reads x itself
            # fp32 rows only where they are read: the hooks (merge_windows) and the final norm
            need_x = last or bool(hooks and i in hooks)
            ops.gemm(buf.m, P[b + "mlp.fc2.weight"], buf.x if need_x else None, M=M, N=D, K=MLP_DIM,
                     bias=P[b + "mlp.fc2.bias"], gamma=P[b + "ls2.gamma"], accumulate=True,
                     ln_out=(buf.h, None if last else buf.part), ln_xl=buf.xl, ln_rs_out=None if last else rs)
            if hooks and i in hooks:
                hooks[i]()
            if last:
                ops.layernorm(buf.x, P[pre + "norm.weight"], P[pre + "norm.bias"], buf.out, M, D)
            yield

    # -------------------------------------------------------- conv helpers
    def _conv3(self, x, s_in, cin, w, out, cout, bias=None, relu_a=False, act=0, R1=None, R2=None,
               stride=1, border_corr=None, tile=0):
        s_out = (s_in + 2 - 3) // stride + 1
        ops.gemm(x, w, out, M=s_out * s_out, N=cout, K=9 * cin,
                 conv=dict(in_h=s_in, in_w=s_in, in_c=cin, k=3, stride=stride, pad=1, out_h=s_out, out_w=s_out),
                 relu_a=relu_a, bias=bias, act=act, R1=R1, ldr1=cout, R2=R2, ldr2=cout, ldc=cout,
                 border_corr=border_corr, tile=tile)

    def _deconv(self, x, s_in, cin, w, out, cout, bias=None, C_off=0, ldc=None):
        ops.gemm(x, w, out, M=s_in * s_in, N=4 * cout, K=cin, bias=bias, deconv=(s_in, s_in, cout),
                 C_off=C_off, ldc=cout if ldc is None else ldc)

    def _resblock(self, pre: str, x, s, out, extra=None, t=None):
        """out = x (+ extra) + conv(relu(conv(relu(x)))) at s x s x 256 (decoder.py:96-118); with
        `t` given, the first conv's output is already there (_resblock_head)."""
        P = self.P
        if t is None:
            t = self.dec[s]["t"]
            self._resblock_head(pre, x, s, t)
        self._conv3(t, s, 256, P[pre + ".3.w"], out, 256, bias=P[pre + ".3.b"], R1=x, R2=extra)

    def _resblock_head(self, pre: str, x, s, t):
        """t = relu(conv(relu(x))): the first half of a ResidualBlock (decoder.py:96-118)."""
        P = self.P
        self._conv3(x, s, 256, P[pre + ".1.w"], t, 256, bias=P[pre + ".1.b"], relu_a=True, act=DP_ACT_RELU)

    def _fusion(self, i: int, feats, s, x1, t1=None):
        """FeatureFusionBlock2d i at resolution s (decoder.py:121-206; output at 2s for i != 0);
        `t1`: resnet1's first conv already computed (the early fusion-0 schedule of _forward)."""
        P, d = self.P, self.dec[s]
        p = f"decoder.fusions.{i}."
        x = feats
        if x1 is not None:
            self._resblock(p + "resnet1", x1, s, d["x"], extra=feats, t=t1)
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

    # -------------------------------------------------------------- encoders
    def _side_encoders(self):
        """Image encoder ViT on x2 (encoder.py:308-311) and FOV encoder ViT (fov.py:66-72) as one
        grouped ViT, then the lowres upsample into `cat` and the FOV Linear (fov.py:45-47)."""
        for _ in self._side_steps():
            pass

    def _side_steps(self):
        """_side_encoders as a generator: the embedding, then one step per Block (the final norm
        with the last), then the lowres upsample + FOV Linear after the last yield."""
        P, e = self.P, "encoder."
        yield from self._vit_steps(self.side_vits, self.vs, 1, 34 * PTOK)
        ops.merge_windows(self.vi.out, 0, 1, 0, self.g)
        self._deconv(self.g, 24, D, P[e + "upsample_lowres.w"], self.cat, D, bias=P[e + "upsample_lowres.b"],
                     C_off=D, ldc=2 * D)
        if self.use_fov:
            ops.gemm(self.vf.out, P["fov.lin.w"], self.fov_tok, M=PTOK, N=128, K=D, A_off=D, bias=P["fov.lin.b"])

    def _fov_head(self):
        """FOV head (fov.py:56-82): needs the low-res decoder features and the FOV tokens."""
        P = self.P
        self._conv3(self.low, 48, 256, P["fov.down.w"], self.fx, 128, bias=P["fov.down.b"], act=DP_ACT_RELU,
                    R1=self.fov_tok, stride=2)
        self._conv3(self.fx, 24, 128, P["fov.h0.w"], self.f12, 64, bias=P["fov.h0.b"], act=DP_ACT_RELU, stride=2)
        self._conv3(self.f12, 12, 64, P["fov.h2.w"], self.f6, 32, bias=P["fov.h2.b"], act=DP_ACT_RELU, stride=2)
        ops.fov_tail(self.f6, P["fov.h4.w"], P["fov.h4.b"], self.fov_deg)

    # -------------------------------------------------------------- forward
    def forward(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """Run the network on `self.x0`; results in self.canonical / self.fov_deg.  Ends with the
        workspace checks (part of a captured graph): status_dev[i] = workspace i's error word, and
        a set word is cleared together with the hand-off flags, so the next forward starts clean."""
        with ops.use_workspace(self.ws_main):
            out = self._forward()
        for i, w in enumerate(self._wss):
            ops.workspace_check(w, self.status_dev[i:i + 1])
        return out

    def _on(self, st: torch.cuda.Stream, after=None):
        """Context: launches issued inside go to `st` (the current stream when serial) after `after`
        (a stream or an event) has reached this point; GEMMs there take no stream-K engine unless
        the caller sets a workspace inside."""
        main = torch.cuda.current_stream(self.dev)
        if self.serial_side:
            return ops.use_workspace(self.ws_main)
        if isinstance(after, torch.cuda.Event):
            st.wait_event(after)
        else:
            st.wait_stream(after if after is not None else main)
        return _StreamCtx(st)

    def _forward(self) -> Tuple[torch.Tensor, torch.Tensor]:
        P, e = self.P, "encoder."
        main = torch.cuda.current_stream(self.dev)
        serial = self.serial_side
        side_ok = "side" not in _ABLATE

        def mark(st):
            ev = torch.cuda.Event()
            ev.record(main if serial else st)
            return ev

        # pyramid + 35 windows + patch-embed im2col (encoder.py:151-263)
        ops.patchify_pyramid(self.x0, self.cols)
        # image and FOV encoders (one grouped ViT, M = 2 x 577 rows) beside the patch encoder, free-running
        # on the side stream (measured and rejected, round 4: side blocks gated into chosen patch-encoder
        # launches, -1.1 to -2.6 fps, profiles/r04e_ab/, r04f_ab/)
        if side_ok:
            with self._on(self.side):
                self._side_encoders()
        # patch encoder; hooks after blocks 5 / 11 (encoder.py:133-144, 267-288)
        vp = self.vp
        ev = {}

        def lat0_chain():       # encoder.py:314-324, the latent-0 project / upsample (to 384^2)
            with self._on(self.dec_a):
                ops.gemm(self.lat0, P[e + "upsample_latent0.0"], self.t96_256, M=96 * 96, N=256, K=D)
                self._deconv(self.t96_256, 96, 256, P[e + "upsample_latent0.1"], self.t192_256, 256)
                self._deconv(self.t192_256, 192, 256, P[e + "upsample_latent0.2"], self.t384_256, 256)
                ev["lat0pre"] = mark(self.dec_a)

        def lat1_chain():       # ... latent 1 (to enc1, 384^2)
            with self._on(self.dec_b):
                ops.gemm(self.lat1, P[e + "upsample_latent1.0"], self.t96_256b, M=96 * 96, N=256, K=D)
                self._deconv(self.t96_256b, 96, 256, P[e + "upsample_latent1.1"], self.t192_256b, 256)
                self._deconv(self.t192_256b, 192, 256, P[e + "upsample_latent1.2"], self.enc1, 256)
                ev["enc1"] = mark(self.dec_b)

        # (measured and rejected: the latent chains started at their hooks, beside the patch encoder's
        # blocks 6..23: 47.88 / 47.76 vs 48.17 / 48.07 fps, profiles/r05g_lat_early/)
        hooks = {5: lambda: ops.merge_windows(vp.x, 0, 5, 3, self.lat0),
                 11: lambda: ops.merge_windows(vp.x, 0, 5, 3, self.lat1)}
        self._vit(["encoder.patch_encoder."], vp, NWIN, 0, hooks)
        ops.merge_windows(vp.out, 0, 5, 3, self.f0)
        ops.merge_windows(vp.out, 25, 3, 6, self.f1)
        ops.merge_windows(vp.out, 34, 1, 0, self.f2)

        # project / upsample (encoder.py:314-324): the latent and f0 / f1 chains (small grids) beside
        # the main stream's f2 chain -> fuse_lowres -> convs.4, in the order the decoder's
        # projections need their outputs
        # fusion 0's resnet1 first conv (768^2; needs only enc0, its output in dec[768]["c"], unused at
        # 768^2) on dec_c right after the lat0 chain's last deconv, beside fusion 1 (384^2) instead of
        # after it: 48.17 / 48.19 -> 48.60 / 48.74 fps same box (profiles/r05f_dec_early/); on dec_a with
        # the whole lat0 chain, beside fuse_lowres and fusions 4..1, it was slower (47.61 / 47.48): the
        # small-grid fusions then wait for CUs
        early = "decoder" not in _ABLATE
        t1 = self.dec[768]["c"] if early else None
        lat0_chain()
        with self._on(self.dec_b):
            ops.gemm(self.f1, P[e + "upsample1.0"], self.t48_1024, M=48 * 48, N=D, K=D)
            self._deconv(self.t48_1024, 48, D, P[e + "upsample1.1"], self.enc3, D)
            ev["enc3"] = mark(self.dec_b)
            ops.gemm(self.f0, P[e + "upsample0.0"], self.t96_512, M=96 * 96, N=512, K=D)
            self._deconv(self.t96_512, 96, 512, P[e + "upsample0.1"], self.enc2, 512)
            ev["enc2"] = mark(self.dec_b)
        lat1_chain()
        sk = DP_TILE_SPLITK_256x256
        ops.gemm(self.f2, P[e + "upsample2.0"], self.t24_1024, M=24 * 24, N=D, K=D)
        self._deconv(self.t24_1024, 24, D, P[e + "upsample2.1"], self.cat, D, ldc=2 * D)
        if not serial:
            main.wait_stream(self.side)  # join: the image-encoder half of `cat`
        ops.gemm(self.cat, P[e + "fuse_lowres.w"], self.enc4, M=48 * 48, N=D, K=2 * D, bias=P[e + "fuse_lowres.b"])
        # decoder (decoder.py:74-93)
        self._conv3(self.enc4, 48, D, P["decoder.convs.4"], self.low, 256,
                    tile=sk)
        # dec_c (after convs.4, the main stream's last stream-K launch before fusion 1's deconv, which
        # waits for convs.1 -- so dec_c's stream-K launches never overlap the main stream's):
        # convs.3 / .2 / .1 in the order the fusions need them, the lat0 chain's 384^2 -> 768^2
        # deconv (stream-K), then the FOV head (needs only the low-res features and the FOV tokens)
        with self._on(self.dec_c), ops.use_workspace(self.ws_main if serial else self.ws_dec):
            for i, (enc, s_, cin) in ((3, (self.enc3, 96, D)), (2, (self.enc2, 192, 512)),
                                      (1, (self.enc1, 384, 256))):
                if not serial:
                    self.dec_c.wait_event(ev[f"enc{i}"])
                self._conv3(enc, s_, cin, P[f"decoder.convs.{i}"], self.dec[s_]["c"], 256)
                ev[f"c{i}"] = mark(self.dec_c)
            if not serial:
                self.dec_c.wait_event(ev["lat0pre"])
            self._deconv(self.t384_256, 384, 256, P[e + "upsample_latent0.3"], self.enc0, 256)
            ev["enc0"] = mark(self.dec_c)
            if early:
                self._resblock_head("decoder.fusions.0.resnet1", self.enc0, 768, t1)
                ev["r1a"] = mark(self.dec_c)
            if self.use_fov and side_ok:
                if not serial:
                    self.dec_c.wait_stream(self.side)
                self._fov_head()
        if "decoder" not in _ABLATE:
            f = self._fusion(4, self.low, 48, None)
            for i, s in ((3, 96), (2, 192), (1, 384)):
                if not serial:
                    main.wait_event(ev[f"c{i}"])
                    if i == 1:
                        main.wait_event(ev["enc0"])
                f = self._fusion(i, f, s, self.dec[s]["c"])
            if early and not serial:
                main.wait_event(ev["r1a"])
            feats = self._fusion(0, f, 768, self.enc0, t1=t1)
        else:
            feats = self.feats
        if not serial:
            for st in (self.dec_a, self.dec_b, self.dec_c, self.side):
                main.wait_stream(st)
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
        """One forward (graph replay if captured) on the current stream.  Its health lands in
        `status_dev`; `finish_status` (after whatever else writes it, e.g. the infer epilogue's
        non-finite count) turns it into this frame's FrameStatus."""
        if self.graph is not None:
            self.graph.replay()
        else:
            self.forward()
        return self.canonical, self.fov_deg

    def finish_status(self) -> FrameStatus:
        """Snapshot this frame's status words into pinned memory (asynchronously, on the current
        stream), reset the non-finite counter for the next frame, and return the FrameStatus."""
        words = torch.empty(self.status_dev.numel(), dtype=torch.int32, pin_memory=True)
        words.copy_(self.status_dev, non_blocking=True)
        self.status_dev[-1:].zero_()
        ev = torch.cuda.Event()
        ev.record()
        st = FrameStatus(self._frames, words, ev)
        self._frames += 1
        self._recent.append(st)
        if len(self._recent) > 64:
            # bounded list: move finished frames out (bad ones stay owed to the next check_status);
            # if none has finished, wait for the oldest
            self._sweep(block_oldest=True)
        self.last_status = st
        if self.sync_check:
            st.check()
        return st

    def _sweep(self, block: bool = False, block_oldest: bool = False) -> None:
        keep = []
        for j, st in enumerate(self._recent):
            if st.reported or st.owned:       # checked already, or its owner checks it (claim)
                continue
            if block or st.ready() or (block_oldest and j == 0):
                if st.error() is not None:
                    self._unreported.append(st)
            else:
                keep.append(st)
        self._recent = keep

    def check_status(self, block: bool = True) -> None:
        """Raise DPError naming EVERY bad frame not reported yet (block=False: only frames already
        done).  Each frame's status is reported once: checked frames leave the list, so a bad
        frame does not fail every later check."""
        self._sweep(block=block)
        bad, self._unreported = [st for st in self._unreported if not (st.reported or st.owned)], []
        if bad:
            for st in bad:
                st.reported = True
            raise DPError("; ".join(f"frame {st.frame}: {st.error()}" for st in bad))


class _StreamCtx:
    """torch.cuda.stream(st) + no stream-K workspace for the GEMMs issued inside."""

    def __init__(self, st):
        self.st = torch.cuda.stream(st)
        self.ws = ops.use_workspace(None)

    def __enter__(self):
        self.st.__enter__()
        self.ws.__enter__()
        return self

    def __exit__(self, *exc):
        self.ws.__exit__(*exc)
        return self.st.__exit__(*exc)
