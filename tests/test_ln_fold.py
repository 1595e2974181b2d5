"""LayerNorm folded across the GEMM boundary (ops.fold_layernorm, pack time; CPU, exact algebra):
LN(x) W^T + b == rstd * (x (W o ln_w)^T - mean * rowsum(W o ln_w)) + (b + W ln_b), times an optional
per-output-column scale (the qkv's log2q factor on Q).  The GPU epilogues that evaluate the right
side are tested in test_gpu_kernels.py (test_gemm_8ph320_ln_consumer, test_gemm_8ph320_ln_producer)."""

import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ml-depth-pro-video_amd"))
from depth_pro import ops  # noqa: E402


def _case(seed, scale=None):
    g = torch.Generator().manual_seed(seed)
    M, K, N = 37, 1024, 96
    x = torch.randn(M, K, generator=g, dtype=torch.float64) * 3 + 0.5
    w = torch.randn(N, K, generator=g, dtype=torch.float64) * K ** -0.5
    b = torch.randn(N, generator=g, dtype=torch.float64)
    lw = torch.rand(K, generator=g, dtype=torch.float64) + 0.5
    lb = torch.randn(K, generator=g, dtype=torch.float64) * 0.1
    s = None if scale is None else torch.rand(N, generator=g, dtype=torch.float64) + scale
    return x, w, b, lw, lb, s


def test_fold_is_exact_algebra_in_fp64():
    for seed, scale in ((0, None), (1, 0.25)):
        x, w, b, lw, lb, s = _case(seed, scale)
        eps = 1e-6
        ref = torch.nn.functional.layer_norm(x, (x.shape[1],), lw, lb, eps) @ w.t() + b
        if s is not None:
            ref = ref * s
        wf, bias, colsum = ops.fold_layernorm(w, b, lw, lb, torch.float64, col_scale=s)
        mean = x.mean(1, keepdim=True)
        rstd = (x.var(1, unbiased=False, keepdim=True) + eps).rsqrt()
        out = rstd * (x @ wf.t() - mean * colsum.double()) + bias.double()
        # bias / colsum come back in fp32 (what the epilogue reads): agreement to fp32 rounding
        assert torch.allclose(out, ref, rtol=1e-5, atol=1e-5), (out - ref).abs().max().item()


def test_fold_colsum_is_the_sum_of_the_rounded_weights():
    """S must be the row sums of B exactly as the MFMA sees it (the 16-bit values), summed in fp64,
    so that x (W o ln_w)^T - mean * S cancels the mean of x to the GEMM's own rounding."""
    x, w, b, lw, lb, s = _case(2, 0.5)
    for dt in (torch.bfloat16, torch.float16):
        wf, bias, colsum = ops.fold_layernorm(w, b, lw, lb, dt, col_scale=s)
        assert wf.dtype == dt and bias.dtype == torch.float32 and colsum.dtype == torch.float32
        assert torch.equal(colsum, wf.double().sum(1).float())
        # a constant row (x = c) has LN(x) = ln_b: the folded form gives b' + 0 up to rounding
        c = torch.full((1, w.shape[1]), 7.25, dtype=torch.float64)
        got = (c @ wf.double().t() - 7.25 * colsum.double()).abs().max().item()
        assert got < 1e-4 * wf.double().abs().sum(1).max().item(), got
