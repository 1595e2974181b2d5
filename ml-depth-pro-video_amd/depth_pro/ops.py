"""Typed launchers: torch tensors -> C-ABI calls on the current HIP stream.

Every function takes device tensors (PyTorch owns the memory), passes their
`data_ptr()` and the current stream to libdp_mi355x.so and raises
`_lib.DPError` on any non-zero return.  Nothing here computes on the host.
"""

from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib
from ._lib import (DP_A_CONV, DP_A_DENSE, DP_ACT_NONE, DP_BF16, DP_F16, DP_F32,
                   DP_STORE_DECONV2X2, DP_STORE_HEAD_PS, DP_STORE_ROWS, GemmArgs, check)

_TORCH_DT = {DP_BF16: torch.bfloat16, DP_F16: torch.float16, DP_F32: torch.float32}


def torch_dtype(code: int) -> torch.dtype:
    return _TORCH_DT[code]


def dtype_code(dt: torch.dtype) -> int:
    for k, v in _TORCH_DT.items():
        if v == dt:
            return k
    raise _lib.DPError(f"unsupported dtype {dt}")


# Optional per-launch timing (bench.py's roofline leg): list of (kind, flops, shape, dtype, ev0, ev1, stream).
_PROF: Optional[list] = None
_PROF_T0: Optional[torch.cuda.Event] = None
# While profiling: what selects a GEMM's kernel instantiation beyond its tile, per (kind, shape, dtype)
# -- the epilogue activation and whether it is a folded-LN consumer / a deconv store (bench.py names
# the dominant launch's rocprof kernel from it instead of guessing from the shape)
PROF_GEMM_META: dict = {}


def profile_begin() -> None:
    global _PROF, _PROF_T0
    _PROF = []
    _PROF_T0 = torch.cuda.Event(enable_timing=True)
    _PROF_T0.record()


def profile_end(timeline: bool = False) -> list:
    """Stop recording; returns [(kind, flops, shape, operand dtype, milliseconds)] (synchronizes).
    timeline=True: [(kind, flops, shape, dtype, start ms, end ms, stream)] relative to
    profile_begin on the current stream (events of every stream share the device clock)."""
    global _PROF
    rec, _PROF = _PROF or [], None
    torch.cuda.synchronize()
    if timeline:
        return [(k, f, sh, dt, _PROF_T0.elapsed_time(a), _PROF_T0.elapsed_time(b), st)
                for (k, f, sh, dt, a, b, st) in rec]
    return [(k, f, sh, dt, a.elapsed_time(b)) for (k, f, sh, dt, a, b, st) in rec]


class _Timed:
    def __init__(self, kind: str, flops: float, shape: tuple = (), dtype=None):
        self.kind, self.flops, self.shape, self.dtype = kind, flops, shape, dtype

    def __enter__(self):
        if _PROF is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *exc):
        if _PROF is not None:
            self.e1.record()
            _PROF.append((self.kind, self.flops, self.shape, self.dtype, self.e0, self.e1,
                          torch.cuda.current_stream().cuda_stream))
        return False


# Stream-K workspace for the GEMMs issued inside `use_workspace(ws)` (one per
# stream that may run a GEMM concurrently with another; see Engine).
_WS: Optional[torch.Tensor] = None


class use_workspace:
    """Context manager: GEMMs issued inside it may use the persistent stream-K engine with `ws`."""

    def __init__(self, ws: Optional[torch.Tensor]):
        self.ws = ws

    def __enter__(self):
        global _WS
        self.prev, _WS = _WS, self.ws
        return self

    def __exit__(self, *exc):
        global _WS
        _WS = self.prev
        return False


WS_ERROR_OFFSET = 4092   # dp_mi355x.h DP_GEMM_WS_ERROR_OFFSET: sticky stream-K timeout word


def workspace_error(ws: torch.Tensor) -> int:
    """The sticky stream-K error word of `ws` (synchronises)."""
    return int(ws[WS_ERROR_OFFSET:WS_ERROR_OFFSET + 4].view(torch.int32).item())


def workspace_check(ws: torch.Tensor, status: torch.Tensor) -> None:
    """dp_gemm_workspace_check: status (device int32, one element) = the sticky error word of `ws`;
    a set word is cleared with every hand-off flag (stream-ordered, graph-capturable)."""
    check(_lib.load().dp_gemm_workspace_check(ws.data_ptr(), status.data_ptr(), _stream(status)),
          "dp_gemm_workspace_check")


def gemm_workspace(device: torch.device) -> torch.Tensor:
    """A zeroed device buffer of dp_gemm_workspace_size() bytes."""
    return torch.zeros(int(_lib.load().dp_gemm_workspace_size()), dtype=torch.uint8, device=device)


def conv_weight(w: torch.Tensor, dt: Optional[torch.dtype] = None) -> torch.Tensor:
    """Conv2d weight [Cout][Cin][kh][kw] -> dp_gemm implicit-conv B operand [Cout][Cin/64][kh][kw][64].

    The K order puts the taps of one 64-channel block next to each other (see conv_tap in
    dp_gemm.hip: neighbouring taps re-read the same input lines one K step apart, in L2).
    """
    co, ci, kh, kw = w.shape
    if ci % 64:
        raise _lib.DPError(f"conv input channels must be a multiple of 64, got {ci}")
    b = w.reshape(co, ci // 64, 64, kh, kw).permute(0, 1, 3, 4, 2).reshape(co, -1)
    return (b if dt is None else b.to(dt)).contiguous()


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def gemm(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor, *, M: int, N: int, K: int,
         lda: Optional[int] = None, ldb: Optional[int] = None, ldc: Optional[int] = None,
         conv: Optional[dict] = None, relu_a: bool = False,
         bias: Optional[torch.Tensor] = None, act: int = DP_ACT_NONE,
         gamma: Optional[torch.Tensor] = None,
         pos: Optional[torch.Tensor] = None, ldpos: int = 0, pos_group: int = 0, pos_off: int = 0,
         R1: Optional[torch.Tensor] = None, ldr1: int = 0,
         R2: Optional[torch.Tensor] = None, ldr2: int = 0,
         accumulate: bool = False, deconv: Optional[tuple] = None,
         row_group: int = 0, row_group_out: int = 0, row_off: int = 0,
         head_w: Optional[torch.Tensor] = None, head_b: float = 0.0,
         head_corr: Optional[torch.Tensor] = None,
         A_off: int = 0, C_off: int = 0, B_off: int = 0, tile: int = 0,
         workspace: Optional[torch.Tensor] = None,
         plan_only: bool = False, border_corr: Optional[torch.Tensor] = None,
         ln_out: Optional[tuple] = None, ln_in: Optional[tuple] = None, ln_eps: float = 1e-6,
         ln_xl: Optional[torch.Tensor] = None, ln_rs_out: Optional[torch.Tensor] = None,
         ln_rs_in: Optional[torch.Tensor] = None):
    """dp_gemm. `A_off`/`B_off`/`C_off` are element offsets into A / B / C (sub-views, e.g. a
    K slice of a split-K GEMM: A_off = B_off = k0 with lda / ldb the full row lengths).

    `workspace` (or the one set by `use_workspace`) enables the stream-K engine.
    `plan_only=True` launches nothing and returns (tile, workgroups) from dp_gemm_plan.
    Folded LayerNorm (dp_gemm_args.ln_*): `ln_out=(xb, part)` -- the residual GEMM also writes the
    new C rows in 16 bits to `xb` and their 128-column chunk statistics to `part`; `ln_in=(part,
    colsum)` -- A holds un-normalised 16-bit rows with statistics `part`, B / bias are folded
    (`fold_layernorm`) and `colsum` = the row sums of B.
    Split residual (ABI 12, `ln_xl` with `ln_out=(xb, part or None)`, accumulate=True): the
    residual stream is x = xb (16-bit) + the int8 low part ln_xl (`split_residual`), updated in place;
    `C` (fp32) is then only an optional output of the new rows (None: not written).
    Producer-merged row statistics (ABI 13): `ln_rs_out` (fp32 [M][2], with the split producer's
    `ln_out=(xb, part)`, N = 1024, eps `ln_eps`, a workspace) -- the producer's last workgroup of each
    row tile also writes every row's (rstd, -rstd * mean); a persistent-engine consumer takes it as
    `ln_rs_in` with `ln_in=(None, colsum)` instead of merging `part` in a pre-pass launch.
    """
    if C is None:
        if ln_xl is None:
            raise _lib.DPError("dp_gemm: C is required (only a split-residual producer may omit it)")
        C = torch.empty(0, dtype=torch.float32, device=ln_xl.device)     # placeholder: C = NULL
    a = _gemm_args(A, B, C, M=M, N=N, K=K, lda=lda, ldb=ldb, ldc=ldc, conv=conv, relu_a=relu_a, bias=bias,
                   act=act, gamma=gamma, pos=pos, ldpos=ldpos, pos_group=pos_group, pos_off=pos_off, R1=R1,
                   ldr1=ldr1, R2=R2, ldr2=ldr2, accumulate=accumulate, deconv=deconv, row_group=row_group,
                   row_group_out=row_group_out, row_off=row_off, head_w=head_w, head_b=head_b,
                   head_corr=head_corr, A_off=A_off, C_off=C_off, B_off=B_off, tile=tile, workspace=workspace,
                   border_corr=border_corr)
    if ln_out is not None:
        xb, part = ln_out
        if xb.numel() < (M - 1) * a.ldc + N or xb.dtype != B.dtype or (part is None and ln_xl is None) or \
                (part is not None and (part.numel() < M * (N // 128) * 2 or part.dtype != torch.float32)):
            raise _lib.DPError("dp_gemm: ln_out buffers too small or of the wrong type")
        a.ln_xb_out, a.ln_part_out = xb.data_ptr(), _p(part)
    if ln_xl is not None:
        if ln_out is None or ln_xl.numel() < (M - 1) * a.ldc + N or ln_xl.dtype != torch.int8:
            raise _lib.DPError("dp_gemm: ln_xl needs ln_out and [M][ldc] int8 rows")
        a.ln_xl = ln_xl.data_ptr()
        if C.numel() == 0:
            a.C = None
    if ln_rs_out is not None:
        if ln_out is None or ln_rs_out.numel() < 2 * M or ln_rs_out.dtype != torch.float32:
            raise _lib.DPError("dp_gemm: ln_rs_out needs ln_out and fp32 [M][2]")
        a.ln_rs_out, a.ln_eps = ln_rs_out.data_ptr(), float(ln_eps)
    if ln_in is not None:
        part, colsum = ln_in
        if (part is None) == (ln_rs_in is None) or colsum.numel() < N or colsum.dtype != torch.float32 or \
                (part is not None and part.numel() < M * (K // 128) * 2) or \
                (ln_rs_in is not None and (ln_rs_in.numel() < 2 * (M + (M & 1)) or ln_rs_in.dtype != torch.float32)):
            raise _lib.DPError("dp_gemm: ln_in buffers too small or of the wrong type")
        a.ln_part_in, a.ln_colsum, a.ln_eps = _p(part), colsum.data_ptr(), float(ln_eps)
        a.ln_rs_in = _p(ln_rs_in)
    elif ln_rs_in is not None:
        raise _lib.DPError("dp_gemm: ln_rs_in needs ln_in=(None, colsum)")
    if plan_only:
        t, g = ctypes.c_int32(), ctypes.c_int32()
        check(_lib.load().dp_gemm_plan(ctypes.byref(a), ctypes.byref(t), ctypes.byref(g)), "dp_gemm_plan")
        return t.value, g.value
    _check_gemm_extents(A, B, C if a.C else None, a, A_off, C_off, conv, deconv, head_w is not None,
                        head_corr is not None, B_off)
    kind = "gemm_conv" if conv is not None else ("gemm_deconv" if deconv is not None else "gemm")
    if _PROF is not None:
        PROF_GEMM_META[(kind, (M, N, K), B.dtype)] = {"act": int(act), "ln_consumer": bool(a.ln_colsum),
                                                     "deconv": deconv is not None}
    with _Timed(kind, 2.0 * M * N * K, (M, N, K), B.dtype):
        check(_lib.load().dp_gemm(ctypes.byref(a), _stream(B)), "dp_gemm")


def gemm_grouped(groups, **common) -> None:
    """dp_gemm_grouped: len(groups) dense GEMMs of one shape in one launch.  Each entry of `groups`
    is a dict with that problem's tensors -- A, B, C and optionally bias, gamma, pos, R1, R2 and the
    element offsets A_off / C_off -- and `common` holds the shared arguments of `gemm` (M, N, K,
    act, accumulate, row_group, ...).  Same result as one `gemm` call per problem."""
    arr = (GemmArgs * len(groups))()
    for i, g in enumerate(groups):
        kw = dict(common)
        kw.update(g)
        A, B, C = kw.pop("A"), kw.pop("B"), kw.pop("C")
        arr[i] = _gemm_args(A, B, C, **kw)
        _check_gemm_extents(A, B, C, arr[i], kw.get("A_off", 0), kw.get("C_off", 0), None, None, False, False)
    M, N, K = common["M"], common["N"], common["K"]
    with _Timed("gemm", 2.0 * M * N * K * len(groups), (M, N, K), groups[0]["B"].dtype):
        check(_lib.load().dp_gemm_grouped(arr, len(groups), _stream(groups[0]["C"])), "dp_gemm_grouped")


def _gemm_args(A, B, C, *, M, N, K, lda=None, ldb=None, ldc=None, conv=None, relu_a=False, bias=None,
               act=DP_ACT_NONE, gamma=None, pos=None, ldpos=0, pos_group=0, pos_off=0, R1=None, ldr1=0, R2=None,
               ldr2=0, accumulate=False, deconv=None, row_group=0, row_group_out=0, row_off=0, head_w=None,
               head_b=0.0, head_corr=None, A_off=0, C_off=0, B_off=0, tile=0, workspace=None,
               border_corr=None) -> "GemmArgs":
    a = GemmArgs()
    a.M, a.N, a.K = M, N, K
    a.dtype = dtype_code(B.dtype)
    a.A = A.data_ptr() + A_off * A.element_size()
    a.lda = K if lda is None else lda
    a.B = B.data_ptr() + B_off * B.element_size()
    a.ldb = K if ldb is None else ldb
    if conv is not None:
        a.a_mode = DP_A_CONV
        a.in_h, a.in_w, a.in_c = conv["in_h"], conv["in_w"], conv["in_c"]
        a.k_h, a.k_w = conv["k"], conv["k"]
        a.stride, a.pad = conv.get("stride", 1), conv.get("pad", 0)
        a.out_h, a.out_w = conv["out_h"], conv["out_w"]
        a.lda = 0
    else:
        a.a_mode = DP_A_DENSE
    a.relu_a = int(relu_a)
    a.bias = _p(bias)
    a.act = act
    a.gamma = _p(gamma)
    a.pos = _p(pos)
    a.ldpos, a.pos_group, a.pos_off = ldpos, pos_group, pos_off
    a.R1, a.ldr1 = _p(R1), ldr1
    a.R2, a.ldr2 = _p(R2), ldr2
    a.C = C.data_ptr() + C_off * C.element_size()
    a.ldc = N if ldc is None else ldc
    a.c_dtype = dtype_code(C.dtype)
    a.accumulate = int(accumulate)
    if deconv is not None:
        a.store_mode = DP_STORE_DECONV2X2
        a.dc_h, a.dc_w, a.dc_cout = deconv
    elif head_corr is not None:
        a.store_mode = DP_STORE_HEAD_PS
    else:
        a.store_mode = DP_STORE_ROWS
    a.row_group, a.row_group_out, a.row_off = row_group, row_group_out, row_off
    a.head_w = _p(head_w)
    a.head_b = float(head_b)
    if border_corr is not None and border_corr.numel() < 9 * N:
        raise _lib.DPError("dp_gemm: border_corr needs 9 * N values")
    a.head_corr = _p(head_corr if head_corr is not None else border_corr)
    a.tile = tile
    ws = workspace if workspace is not None else _WS
    if ws is not None:
        a.workspace, a.workspace_bytes = ws.data_ptr(), ws.numel() * ws.element_size()
    return a


def _check_gemm_extents(A, B, C, a, A_off, C_off, conv, deconv, head, head_ps, B_off=0) -> None:
    """Host-side bounds check: every element dp_gemm will read or write lies inside the
    tensors passed (a wrong leading dimension would otherwise write past the buffer on
    the GPU)."""
    def need(t, off, n, what):
        if off + n > t.numel():
            raise _lib.DPError(f"dp_gemm: {what} needs {off + n} elements, tensor has {t.numel()}")

    M, N, K = a.M, a.N, a.K
    if conv is not None:
        need(A, A_off, (M // (a.out_h * a.out_w)) * a.in_h * a.in_w * a.in_c, "A (conv input)")
    else:
        need(A, A_off, (M - 1) * a.lda + K, "A")
    need(B, B_off, (N - 1) * a.ldb + K, "B")
    if C is None:       # a split-residual producer with no fp32 output (its xb / xl checked by gemm)
        return
    if head_ps:
        need(C, C_off, (M // (a.out_h * a.out_w)) * 4 * a.out_h * a.out_w, "C (pixel-shuffle head)")
    elif head:
        need(C, C_off, M, "C (fused head)")
    elif deconv is not None:
        need(C, C_off, (4 * M - 1) * a.ldc + a.dc_cout, "C (deconv)")
    else:
        last = M - 1
        if a.row_group:
            last = (last // a.row_group) * a.row_group_out + a.row_off + last % a.row_group
        need(C, C_off, last * a.ldc + N, "C")


def layernorm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, y: torch.Tensor, rows: int, cols: int,
              eps: float = 1e-6) -> None:
    with _Timed("layernorm", 0.0, (rows, cols), y.dtype):
        check(_lib.load().dp_layernorm(x.data_ptr(), cols, w.data_ptr(), b.data_ptr(), y.data_ptr(), cols,
                                       rows, cols, eps, dtype_code(y.dtype), _stream(y)), "dp_layernorm")


def layernorm_stats(x: torch.Tensor, xb: torch.Tensor, part: torch.Tensor, rows: int, cols: int,
                    xl: Optional[torch.Tensor] = None) -> None:
    """dp_layernorm_stats: x (fp32 rows) -> xb (16 bits) + 128-column chunk statistics `part` --
    the input side of a folded LayerNorm for rows no residual GEMM produced (ViT block 0); `xl`:
    also the split residual's int8 low part (dp_gemm's ln_xl encoding, `split_residual`)."""
    if x.numel() < rows * cols or xb.numel() < rows * cols or part.numel() < rows * (cols // 128) * 2:
        raise _lib.DPError("dp_layernorm_stats: buffers smaller than rows * cols")
    if xl is not None and (xl.numel() < rows * cols or xl.dtype != torch.int8):
        raise _lib.DPError("dp_layernorm_stats: xl must be int8 rows * cols")
    with _Timed("layernorm", 0.0, (rows, cols), xb.dtype):
        check(_lib.load().dp_layernorm_stats(x.data_ptr(), cols, rows, cols, xb.data_ptr(), cols,
                                             xl.data_ptr() if xl is not None else None, part.data_ptr(),
                                             dtype_code(xb.dtype), _stream(xb)), "dp_layernorm_stats")


def split_residual(x: torch.Tensor, dt: torch.dtype):
    """Host restatement of the split residual's encoding (dp_gemm ln_xl, ABI 12): hi = x in 16 bits,
    q = clamp(rint((x - hi) 2^(S - e)), -128, 127) with e the frexp exponent of hi and S = 16 (bf16)
    / 19 (f16).  Returns (hi, q int8); every step is exact in fp32, so this matches the kernels bit
    for bit (tests)."""
    s = 16 if dt == torch.bfloat16 else 19
    hi = x.to(dt)
    hf = hi.float()
    e = torch.frexp(hf).exponent
    q = torch.round(torch.ldexp(x.float() - hf, (s - e).float())).clamp(-128, 127).to(torch.int8)
    return hi, q


def merge_residual(hi: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
    """x = hi + q 2^(e - S) in fp32 (the inverse of `split_residual`, exact)."""
    s = 16 if hi.dtype == torch.bfloat16 else 19
    hf = hi.float()
    e = torch.frexp(hf).exponent
    return hf + torch.ldexp(q.float(), (e - s).float())


def fold_layernorm(w: torch.Tensor, b: torch.Tensor, ln_w: torch.Tensor, ln_b: torch.Tensor, dt: torch.dtype,
                   col_scale: Optional[torch.Tensor] = None):
    """The consumer side of a LayerNorm folded into the Linear after it (pack time):
    LN(x) W^T + b = rstd * (x (W o ln_w)^T - mean * S) + (b + W ln_b), so the GEMM takes the
    un-normalised rows with B = W o ln_w (per input column; times `col_scale` per output, e.g.
    the qkv's log2q gamma), bias = (b + W ln_b) * col_scale and S = the row sums of B exactly as
    the 16-bit values the MFMA multiplies (fp64 sums, fp32 result).  Returns (B, bias, S)."""
    w64, b64 = w.double(), b.double()
    s = torch.ones(w.shape[0], dtype=torch.float64, device=w.device) if col_scale is None else col_scale.double()
    wf = (w64 * ln_w.double()[None, :] * s[:, None]).to(dt).contiguous()
    bias = ((b64 + w64 @ ln_b.double()) * s).float().contiguous()
    colsum = wf.double().sum(1).float().contiguous()
    return wf, bias, colsum


def layernorm_grouped(x: torch.Tensor, ws, bs, y: torch.Tensor, rows_per_group: int, cols: int,
                      eps: float = 1e-6) -> None:
    """dp_layernorm_grouped: rows [g * rows_per_group, (g + 1) * rows_per_group) normalised with
    ws[g] / bs[g] -- one launch for several LayerNorms of one shape."""
    n = len(ws)
    pw = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ws])
    pb = (ctypes.c_void_p * n)(*[t.data_ptr() for t in bs])
    if x.numel() < n * rows_per_group * cols or y.numel() < n * rows_per_group * cols:
        raise _lib.DPError("dp_layernorm_grouped: x / y smaller than groups * rows_per_group * cols")
    with _Timed("layernorm", 0.0, (n * rows_per_group, cols), y.dtype):
        check(_lib.load().dp_layernorm_grouped(x.data_ptr(), cols, pw, pb, n, y.data_ptr(), cols, rows_per_group,
                                               cols, eps, dtype_code(y.dtype), _stream(y)), "dp_layernorm_grouped")


def attention(qkv: torch.Tensor, out: torch.Tensor, batch: int, seq: int, heads: int = 16,
              head_dim: int = 64, log2q: bool = False) -> None:
    """dp_attention; `log2q=True`: dp_attention_log2q, the Q columns of `qkv` already hold
    Q * head_dim^-0.5 * log2(e) (see `log2q_gamma`)."""
    with _Timed("attention", 4.0 * batch * heads * seq * seq * head_dim, (batch, seq), out.dtype):
        if log2q:
            check(_lib.load().dp_attention_log2q(qkv.data_ptr(), out.data_ptr(), batch, seq, heads, head_dim,
                                                 dtype_code(out.dtype), _stream(out)), "dp_attention_log2q")
        else:
            check(_lib.load().dp_attention(qkv.data_ptr(), out.data_ptr(), batch, seq, heads, head_dim,
                                           head_dim ** -0.5, dtype_code(out.dtype), _stream(out)), "dp_attention")


LOG2E = 1.4426950408889634


def log2q_gamma(heads: int, head_dim: int, device) -> torch.Tensor:
    """Per-column gamma for the qkv Linear's epilogue that leaves Q scaled by head_dim^-0.5 *
    log2(e) (the softmax scale in log2 units) and K, V unchanged: input of dp_attention_log2q."""
    g = torch.ones(3 * heads * head_dim, dtype=torch.float32)
    g[:heads * head_dim] = float(head_dim ** -0.5 * LOG2E)
    return g.to(device)


def normalize_u8(img: torch.Tensor, out: torch.Tensor) -> None:
    H, W = img.shape[0], img.shape[1]
    check(_lib.load().dp_normalize_u8(img.data_ptr(), H, W, out.data_ptr(), dtype_code(out.dtype),
                                      _stream(out)), "dp_normalize_u8")


def interp_mode(mode: str) -> int:
    """F.interpolate mode name -> DP_INTERP_* (the modes DepthPro.infer can pass with
    align_corners=False: bilinear, bicubic)."""
    if mode not in _lib.INTERP_MODES:
        raise ValueError(f"interpolation_mode={mode!r}: expected one of {sorted(_lib.INTERP_MODES)}")
    return _lib.INTERP_MODES[mode]


def resize(src: torch.Tensor, dst: torch.Tensor, mode: str = "bilinear") -> None:
    """dp_resize: planar (C,H,W) -> dst (C,OH,OW) fp32, F.interpolate(mode, align_corners=False)."""
    src = src.contiguous()
    C, H, W = src.shape[-3:]
    OH, OW = dst.shape[-2:]
    check(_lib.load().dp_resize(src.data_ptr(), dtype_code(src.dtype), C, H, W, dst.data_ptr(),
                                OH, OW, interp_mode(mode), _stream(dst)), "dp_resize")


def resize_bilinear(src: torch.Tensor, dst: torch.Tensor) -> None:
    resize(src, dst, "bilinear")


def patchify_pyramid(x0: torch.Tensor, cols: torch.Tensor) -> None:
    check(_lib.load().dp_patchify_pyramid(x0.data_ptr(), cols.data_ptr(), dtype_code(cols.dtype),
                                          _stream(cols)), "dp_patchify_pyramid")


def vit_cls_rows(x: torch.Tensor, cls: torch.Tensor, pos: torch.Tensor, n: int) -> None:
    check(_lib.load().dp_vit_cls_rows(x.data_ptr(), cls.data_ptr(), pos.data_ptr(), n, _stream(x)),
          "dp_vit_cls_rows")


def merge_windows(src: torch.Tensor, first_window: int, steps: int, padding: int, dst: torch.Tensor,
                  ld: int = 1024, windows: Optional[tuple] = None) -> None:
    """windows=(lo, hi): only grid windows lo <= w < hi (dp_merge_windows_range)."""
    lib = _lib.load()
    if windows is None:
        check(lib.dp_merge_windows(src.data_ptr(), dtype_code(src.dtype), ld, first_window, steps, padding,
                                   dst.data_ptr(), dtype_code(dst.dtype), _stream(dst)), "dp_merge_windows")
    else:
        check(lib.dp_merge_windows_range(src.data_ptr(), dtype_code(src.dtype), ld, first_window, steps, padding,
                                         int(windows[0]), int(windows[1]), dst.data_ptr(), dtype_code(dst.dtype),
                                         _stream(dst)), "dp_merge_windows_range")


def fov_tail(x6: torch.Tensor, w: torch.Tensor, bias: float, out: torch.Tensor) -> None:
    check(_lib.load().dp_fov_tail(x6.data_ptr(), dtype_code(x6.dtype), w.data_ptr(), float(bias),
                                  out.data_ptr(), _stream(out)), "dp_fov_tail")


def infer_epilogue(canonical: torch.Tensor, fov_deg: Optional[torch.Tensor], f_given: Optional[float],
                   H: int, W: int, depth: torch.Tensor, f_px_out: Optional[torch.Tensor],
                   nonfinite: Optional[torch.Tensor] = None, mode: str = "bilinear") -> None:
    """dp_infer_epilogue_mode; `nonfinite` (device int32, optional) counts NaN / inf outputs;
    `mode` the F.interpolate mode of the resize back to (H, W)."""
    SH, SW = canonical.shape[-2:]
    use_given = f_given is not None
    check(_lib.load().dp_infer_epilogue_mode(canonical.data_ptr(), SH, SW, _p(fov_deg), int(use_given),
                                             float(f_given) if use_given else 0.0, H, W, depth.data_ptr(),
                                             _p(f_px_out), _p(nonfinite), interp_mode(mode), _stream(depth)),
          "dp_infer_epilogue_mode")


def resize_u8_cv(img: torch.Tensor, out_h: int, out_w: int, area: bool) -> torch.Tensor:
    """cv2.resize of a uint8 HxWx3 device frame (dp_resize_u8_cv): INTER_AREA if `area`, else
    INTER_LINEAR -- the reference's --downscale_factor picks INTER_AREA for factor < 1
    (generate_depth_maps.py:95-110)."""
    if img.dtype != torch.uint8 or img.dim() != 3 or img.shape[2] != 3:
        raise _lib.DPError(f"resize_u8_cv expects a uint8 HxWx3 tensor, got {img.dtype} {tuple(img.shape)}")
    img = img.contiguous()
    H, W = img.shape[0], img.shape[1]
    out = torch.empty(out_h, out_w, 3, dtype=torch.uint8, device=img.device)
    interp = _lib.DP_CV_INTER_AREA if area else _lib.DP_CV_INTER_LINEAR
    check(_lib.load().dp_resize_u8_cv(img.data_ptr(), H, W, out.data_ptr(), out_h, out_w, interp, _stream(out)),
          "dp_resize_u8_cv")
    return out


_LUTS = {}


def colormap_lut(cmap: str, device: torch.device):
    """(uint8 [(N + 3)][3] device table, N) of a matplotlib colormap, built from matplotlib itself
    the way the reference's colorize_depth converts (generate_depth_maps.py:15-44): the colormap's
    float64 RGBA at integer indices 0..N-1 (Colormap.__call__ indexes the table directly for
    integers), under / over / bad entries, then (rgba * 255).astype(uint8)."""
    key = (cmap, str(device))
    if key not in _LUTS:
        import matplotlib.pyplot as plt
        import numpy as np

        m = plt.get_cmap(cmap)
        n = m.N
        rgba = np.concatenate([m(np.arange(n)), m(np.array([-1.0])), m(np.array([2.0])), m(np.array([np.nan]))])
        lut = (rgba[:, :3] * 255).astype(np.uint8)
        _LUTS[key] = (torch.from_numpy(lut).to(device), n)
    return _LUTS[key]


def depth_to_image(depth: torch.Tensor, colored: bool = True, cmap: str = "turbo",
                   out: Optional[torch.Tensor] = None, scratch: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dp_depth_to_image: the frame loop's PNG content on the GPU -- colorize_depth (uint8 HxWx3,
    `cmap`) or the --raw uint16 HxW encoding (reference generate_depth_maps.py:15-44, 135-143),
    byte-identical, stream-ordered (no host sync)."""
    if depth.dtype != torch.float32 or not depth.is_contiguous():
        raise _lib.DPError("depth_to_image expects a contiguous fp32 depth map")
    H, W = depth.shape[-2:]
    if scratch is None:
        scratch = torch.empty(2, dtype=torch.int32, device=depth.device)
    if colored:
        lut, n = colormap_lut(cmap, depth.device)
        if out is None:
            out = torch.empty(H, W, 3, dtype=torch.uint8, device=depth.device)
        mode, lp = _lib.DP_DEPTH_IMG_COLOR, lut.data_ptr()
    else:   # uint16 bits in an int16 tensor (host: .numpy().view(np.uint16))
        if out is None:
            out = torch.empty(H, W, dtype=torch.int16, device=depth.device)
        mode, lp, n = _lib.DP_DEPTH_IMG_RAW16, None, 0
    check(_lib.load().dp_depth_to_image(depth.data_ptr(), H * W, scratch.data_ptr(), lp, n, mode, out.data_ptr(),
                                        _stream(depth)), "dp_depth_to_image")
    return out
