"""Host restatement of the split residual stream (dp_gemm ln_xl / dp_layernorm_stats xl, ABI 12):
x = hi (16 bits) + q * 2^(e - S), q int8 -- the encoding the GPU tests check the kernels against
bit for bit (tests/test_gpu_kernels.py) and whose precision DESIGN.md 4 quotes (CPU)."""
import torch

from depth_pro import ops


def test_split_merge_precision_and_range():
    g = torch.Generator().manual_seed(3)
    x = torch.randn(512, 1024, generator=g) * torch.logspace(-3, 3, 1024)[None, :]
    for dt, s in ((torch.bfloat16, 16), (torch.float16, 19)):
        hi, q = ops.split_residual(x, dt)
        assert hi.dtype == dt and q.dtype == torch.int8
        y = ops.merge_residual(hi, q)
        # one step 2^(e - S) = ulp(hi) / 256 at most (half a step, or one where |x - hi| rounds to 128
        # steps and is clamped to 127), below the 16-bit format's normal range its absolute grid
        e = torch.frexp(hi.float()).exponent.float()
        step = torch.ldexp(torch.ones_like(x), e - s)
        floor = 0.0 if dt == torch.bfloat16 else 2.0 ** -25
        assert torch.all((y - x).abs() <= step + floor)
        normal = x.abs() >= 2.0 ** -14   # (f16: below its normal range only the absolute grid holds)
        assert (y - x)[normal].abs().div(x[normal].abs()).mean() < (8e-6 if dt == torch.bfloat16 else 1e-6)
        # merging is exact: an unclamped value re-splits into the same parts
        ok = (q > -128) & (q < 127)
        hi2, q2 = ops.split_residual(y, dt)
        assert torch.equal(hi2[ok], hi[ok]) and torch.equal(q2[ok], q[ok])


def test_split_exact_ties_and_zero():
    # zero and values exactly on the 16-bit grid: q = 0
    x = torch.tensor([0.0, 1.0, -2.5, 1024.0])
    hi, q = ops.split_residual(x, torch.bfloat16)
    assert torch.equal(q, torch.zeros(4, dtype=torch.int8))
    assert torch.equal(ops.merge_residual(hi, q), x)
