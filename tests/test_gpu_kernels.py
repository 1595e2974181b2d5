"""Per-kernel parity of libdp_mi355x.so against plain PyTorch fp32 references.

Tolerances: inputs are exactly representable in the 16-bit compute type, so the
only error sources are fp32 accumulation order and the final rounding of a
16-bit output (relative 2^-8 for bf16, 2^-11 for f16).
"""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from depth_pro import ops  # noqa: E402
from depth_pro._lib import (DP_ACT_GELU, DP_ACT_RELU, DP_TILE_8PH_256x256, DP_TILE_BIG_256x128,  # noqa: E402
                            DP_TILE_BIG_256x256, DP_TILE_BIG_320x256, DP_TILE_BIG_512x128,
                            DP_TILE_DUAL_256x128, DP_TILE_SPLITK_256x256, DP_TILE_STREAMK_256x256)

DTYPES = [torch.bfloat16, torch.float16]


def rnd(*shape, dt, dev, scale=1.0, gen=None):
    return (torch.randn(*shape, generator=gen) * scale).to(dt).to(dev)


def tol(dt):
    return 2e-2 if dt == torch.bfloat16 else 4e-3


def close(out, ref, dt, what):
    out, ref = out.float().cpu(), ref.float().cpu()
    err = (out - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    assert err <= tol(dt) * scale, f"{what}: max|d|={err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M,N,K", [(577, 3072, 1024), (1000, 128, 64), (257, 32, 128), (20195, 1024, 1024)])
def test_gemm_dense_bias(cuda, dt, M, N, K):
    g = torch.Generator().manual_seed(M + N + K)
    A = rnd(M, K, dt=dt, dev=cuda, gen=g)
    B = rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    bias = torch.randn(N, generator=g).to(cuda)
    C = torch.empty(M, N, dtype=dt, device=cuda)
    ops.gemm(A, B, C, M=M, N=N, K=K, bias=bias)
    ref = A.float() @ B.float().t() + bias
    close(C, ref, dt, "gemm")


def test_gemm_past_32bit_element_offsets(cuda):
    """M * lda >= 2^31 (a 4.3 GB A): the planner leaves the 32-bit-offset engines (8-phase 320 x 256,
    persistent) for the 64-bit-pointer ones; the last rows (offsets past 2^31 elements) and the
    first rows vs fp32 torch."""
    M, N, K = (1 << 21) + 5, 1024, 1024
    dt = torch.bfloat16
    g = torch.Generator(device=cuda).manual_seed(11)
    A = torch.empty(M, K, dtype=dt, device=cuda)
    for r0 in range(0, M, 1 << 18):
        A[r0:r0 + (1 << 18)] = torch.randn(min(1 << 18, M - r0), K, device=cuda, generator=g).to(dt)
    B = (torch.randn(N, K, device=cuda, generator=g) * K ** -0.5).to(dt)
    bias = torch.randn(N, device=cuda, generator=g)
    C = torch.full((M, N), float("nan"), dtype=dt, device=cuda)
    tile, _ = ops.gemm(A, B, C, M=M, N=N, K=K, bias=bias, plan_only=True)
    assert tile == DP_TILE_BIG_320x256
    ops.gemm(A, B, C, M=M, N=N, K=K, bias=bias)
    for rows in (slice(0, 2048), slice(M - 4096, M)):
        ref = A[rows].float() @ B.float().t() + bias
        close(C[rows], ref, dt, f"gemm rows {rows.start}..{rows.stop}")
    assert torch.isfinite(C[::4099].float()).all()


@pytest.mark.parametrize("dt", DTYPES)
def test_gemm_gelu_and_residual_accumulate(cuda, dt):
    g = torch.Generator().manual_seed(3)
    M, N, K = 700, 1024, 4096
    A = rnd(M, K, dt=dt, dev=cuda, gen=g)
    B = rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    bias = torch.randn(N, generator=g).to(cuda)
    gamma = torch.rand(N, generator=g).to(cuda)
    X = torch.randn(M, N, generator=g).to(cuda)
    C = X.clone()
    ops.gemm(A, B, C, M=M, N=N, K=K, bias=bias, gamma=gamma, accumulate=True)
    ref = X + gamma * (A.float() @ B.float().t() + bias)
    close(C, ref, torch.float32 if dt == torch.float16 else dt, "proj+ls+residual")
    H = torch.empty(M, N, dtype=dt, device=cuda)
    ops.gemm(A, B, H, M=M, N=N, K=K, bias=bias, act=DP_ACT_GELU)
    close(H, F.gelu(A.float() @ B.float().t() + bias), dt, "fc1+gelu")


@pytest.mark.parametrize("dt", DTYPES)
def test_gemm_patch_embed_rows_pos(cuda, dt):
    g = torch.Generator().manual_seed(5)
    n, K, N = 3, 768, 1024
    A = rnd(n * 576, K, dt=dt, dev=cuda, gen=g)
    B = rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    bias = torch.randn(N, generator=g).to(cuda)
    pos = torch.randn(577, N, generator=g).to(cuda)
    cls = torch.randn(N, generator=g).to(cuda)
    X = torch.full((n * 577, N), float("nan"), device=cuda)
    ops.gemm(A, B, X, M=n * 576, N=N, K=K, bias=bias, pos=pos, ldpos=N, pos_group=576, pos_off=1,
             row_group=576, row_group_out=577, row_off=1)
    ops.vit_cls_rows(X, cls, pos, n)
    t = (A.float() @ B.float().t() + bias).reshape(n, 576, N)
    ref = torch.cat((cls.expand(n, 1, N), t), 1) + pos
    close(X.reshape(n, 577, N), ref, torch.float32, "patch-embed rows")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("S,cin,cout,stride", [(48, 1024, 256, 1), (96, 256, 256, 1), (48, 256, 128, 2),
                                                (12, 64, 32, 2), (37, 128, 64, 1)])
def test_conv3x3_implicit_gemm(cuda, dt, S, cin, cout, stride):
    g = torch.Generator().manual_seed(S * cin + cout)
    x = rnd(1, cin, S, S, dt=dt, dev=cuda, gen=g)
    w = rnd(cout, cin, 3, 3, dt=dt, dev=cuda, gen=g, scale=(9 * cin) ** -0.5)
    b = torch.randn(cout, generator=g).to(cuda)
    r1 = rnd(1, cout, (S + 2 - 3) // stride + 1, (S + 2 - 3) // stride + 1, dt=dt, dev=cuda, gen=g)
    so = (S + 2 - 3) // stride + 1
    xh = x.permute(0, 2, 3, 1).contiguous()
    wp = ops.conv_weight(w)
    r1h = r1.permute(0, 2, 3, 1).contiguous()
    out = torch.empty(so * so, cout, dtype=dt, device=cuda)
    ops.gemm(xh, wp, out, M=so * so, N=cout, K=9 * cin,
             conv=dict(in_h=S, in_w=S, in_c=cin, k=3, stride=stride, pad=1, out_h=so, out_w=so),
             relu_a=True, bias=b, act=DP_ACT_RELU, R1=r1h, ldr1=cout)
    ref = F.relu(F.conv2d(F.relu(x.float()), w.float(), b, stride=stride, padding=1)) + r1.float()
    close(out.reshape(1, so, so, cout).permute(0, 3, 1, 2), ref, dt, "conv3x3")


@pytest.mark.parametrize("dt", DTYPES)
def test_deconv2x2_pixel_shuffle_store(cuda, dt):
    g = torch.Generator().manual_seed(11)
    S, cin, cout = 24, 1024, 512
    x = rnd(1, cin, S, S, dt=dt, dev=cuda, gen=g)
    w = rnd(cin, cout, 2, 2, dt=dt, dev=cuda, gen=g, scale=cin ** -0.5)
    b = torch.randn(cout, generator=g).to(cuda)
    xh = x.permute(0, 2, 3, 1).reshape(S * S, cin).contiguous()
    wp = w.permute(2, 3, 1, 0).reshape(4 * cout, cin).contiguous()
    out = torch.zeros(2 * S * 2 * S, 2 * cout, dtype=dt, device=cuda)  # into a concat buffer, 2nd half
    ops.gemm(xh, wp, out, M=S * S, N=4 * cout, K=cin, bias=b.repeat(4), deconv=(S, S, cout), C_off=cout, ldc=2 * cout)
    ref = F.conv_transpose2d(x.float(), w.float(), b, stride=2)
    got = out[:, cout:].reshape(1, 2 * S, 2 * S, cout).permute(0, 3, 1, 2)
    close(got, ref, dt, "deconv")
    assert out[:, :cout].abs().max().item() == 0


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("case", ["s96_c256_bias", "s40_c512_cat_nobias", "b2_s64_c256"])
def test_deconv2x2_persistent_8phase_bit_identical(cuda, dt, case):
    """The persistent 8-phase engine with the 2x2 stride-2 deconv store (output pixel (2y + q/2,
    2x + q%2) per GEMM row and column group q): bit-identical to the 256 x 256 engine -- into a
    concat buffer's second half, without bias, ragged last row tile, 2 images -- and vs
    F.conv_transpose2d."""
    from depth_pro._lib import DP_TILE_P8PH_256x256

    g = torch.Generator().manual_seed(sum(map(ord, case)))
    S, cin, cout, nb, bias, cat = {"s96_c256_bias": (96, 256, 256, 1, True, False),
                                   "s40_c512_cat_nobias": (40, 512, 256, 1, False, True),
                                   "b2_s64_c256": (64, 256, 256, 2, True, False)}[case]
    x = rnd(nb, cin, S, S, dt=dt, dev=cuda, gen=g)
    w = rnd(cin, cout, 2, 2, dt=dt, dev=cuda, gen=g, scale=cin ** -0.5)
    b = torch.randn(cout, generator=g).to(cuda) if bias else None
    xh = x.permute(0, 2, 3, 1).reshape(nb * S * S, cin).contiguous()
    wp = w.permute(2, 3, 1, 0).reshape(4 * cout, cin).contiguous()
    ldc = 2 * cout if cat else cout
    kw = dict(M=nb * S * S, N=4 * cout, K=cin, bias=b.repeat(4) if bias else None, deconv=(S, S, cout),
              C_off=cout if cat else 0, ldc=ldc)
    out1 = torch.full((nb * 4 * S * S, ldc), 3.0, dtype=dt, device=cuda)
    out2 = out1.clone()
    ops.gemm(xh, wp, out1, tile=DP_TILE_P8PH_256x256, **kw)
    ops.gemm(xh, wp, out2, tile=DP_TILE_BIG_256x256, **kw)
    torch.cuda.synchronize()
    assert torch.equal(out1, out2), (out1.float() - out2.float()).abs().max().item()
    ref = F.conv_transpose2d(x.float(), w.float(), b, stride=2)
    got = out1[:, ldc - cout:].reshape(nb, 2 * S, 2 * S, cout).permute(0, 3, 1, 2)
    close(got, ref, dt, f"p8ph deconv {case}")
    if cat:
        assert (out1[:, :cout] == 3.0).all()


@pytest.mark.parametrize("dt", DTYPES)
def test_head_conv_with_fused_1x1(cuda, dt):
    g = torch.Generator().manual_seed(13)
    S, cin = 40, 128
    x = rnd(1, cin, S, S, dt=dt, dev=cuda, gen=g)
    w = rnd(32, cin, 3, 3, dt=dt, dev=cuda, gen=g, scale=(9 * cin) ** -0.5)
    b = torch.randn(32, generator=g).to(cuda)
    w4 = torch.rand(32, generator=g).to(cuda)
    out = torch.empty(S * S, dtype=torch.float32, device=cuda)
    ops.gemm(x.permute(0, 2, 3, 1).contiguous(), ops.conv_weight(w), out,
             M=S * S, N=32, K=9 * cin, conv=dict(in_h=S, in_w=S, in_c=cin, k=3, stride=1, pad=1, out_h=S, out_w=S),
             bias=b, act=DP_ACT_RELU, head_w=w4, head_b=0.25)
    h = F.relu(F.conv2d(x.float(), w.float(), b, padding=1))
    ref = F.relu(F.conv2d(h, w4.reshape(1, 32, 1, 1), torch.tensor([0.25], device=cuda)))
    close(out.reshape(1, 1, S, S), ref, dt, "head conv+1x1")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("batch,seq,spike", [(2, 577, None), (1, 100, None), (3, 64, None), (1, 1, None),
                                             (2, 66, None), (1, 2, None), (1, 67, None),
                                             (2, 577, "tail"), (1, 130, "tail"), (2, 577, "mid"),
                                             (1, 100, "mid"), (1, 576, None), (1, 640, None), (1, 1024, None),
                                             (1, 200, None), (1, 1024, "mid")])
@pytest.mark.parametrize("log2q", [False, True])
def test_attention(cuda, dt, batch, seq, spike, log2q):
    """seq 577 / 66 / 2 / 130 end in 1-2 leftover keys (the VALU tail), 100 / 67 / 200 in a partial
    MFMA tile; 576 / 640 / 1024 are whole key tiles (the steady loop with both score halves issued
    ahead, the scalar-base LDS-DMA of full tiles), 576 with a half-empty last query block.  spike "tail": the LAST key of every sequence is the scaled query of token 0, so
    that query's running max jumps inside the tail -- the rescale branch there is exercised;
    "mid": key 70 (second key tile) is 40x that query, far above the max the first half key
    tile set: P overflows and the workgroup redoes its keys on the exact-max path.
    log2q: dp_attention_log2q on the same qkv with its Q columns pre-multiplied by
    hd^-0.5 * log2(e) and rounded to 16 bits (what the engine's qkv epilogue writes); the fp32
    reference takes its Q from those rounded values (in the model Q is rounded once either way:
    the test's second rounding would otherwise move the 40x spike's scores by ~0.5 log2 units)."""
    g = torch.Generator().manual_seed(seq)
    H, hd = 16, 64
    qkv = rnd(batch * seq, 3 * H * hd, dt=dt, dev=cuda, gen=g, scale=2.0)
    if spike:
        x = qkv.view(batch, seq, 3, H, hd)
        key, f = (seq - 1, 4.0) if spike == "tail" else (70, 40.0)
        x[:, key, 1] = (x[:, 0, 0].float() * f).to(dt)
    if log2q:
        g2 = ops.log2q_gamma(H, hd, cuda)
        qkv_in = (qkv.float() * g2).to(dt)
        qkv = qkv_in.float() / g2          # fp32: the reference sees exactly the rounded Q
    q, k, v = qkv.float().reshape(batch, seq, 3, H, hd).permute(2, 0, 3, 1, 4).unbind(0)
    ref = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(batch * seq, H * hd)
    out = torch.empty(batch * seq, H * hd, dtype=dt, device=cuda)
    if log2q:
        ops.attention(qkv_in, out, batch, seq, H, hd, log2q=True)
    else:
        ops.attention(qkv, out, batch, seq, H, hd)
    close(out, ref, dt, "attention")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("cols", [1024, 256, 512, 2048])
def test_layernorm(cuda, dt, cols):
    g = torch.Generator().manual_seed(17 + cols)
    x = (torch.randn(1234, cols, generator=g) * 3 + 1).to(cuda)
    w = torch.randn(cols, generator=g).to(cuda)
    b = torch.randn(cols, generator=g).to(cuda)
    y = torch.empty(1234, cols, dtype=dt, device=cuda)
    ops.layernorm(x, w, b, y, 1234, cols)
    close(y, F.layer_norm(x, (cols,), w, b, 1e-6), dt, "layernorm")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("groups", [2, 3])
def test_layernorm_grouped_matches_per_group(cuda, dt, groups):
    """dp_layernorm_grouped (the side encoders' norms in one launch) = one dp_layernorm per group,
    bit for bit, and each group uses its own affine parameters."""
    g = torch.Generator().manual_seed(23)
    R, cols = 577, 1024
    x = (torch.randn(groups * R, cols, generator=g) * 2 - 1).to(cuda)
    ws = [torch.randn(cols, generator=g).to(cuda) for _ in range(groups)]
    bs = [torch.randn(cols, generator=g).to(cuda) for _ in range(groups)]
    y = torch.empty(groups * R, cols, dtype=dt, device=cuda)
    ops.layernorm_grouped(x, ws, bs, y, R, cols)
    y1 = torch.empty_like(y)
    for i in range(groups):
        ops.layernorm(x[i * R:], ws[i], bs[i], y1[i * R:], R, cols)
    torch.cuda.synchronize()
    assert torch.equal(y, y1)
    close(y[R:2 * R], F.layer_norm(x[R:2 * R], (cols,), ws[1], bs[1], 1e-6), dt, "layernorm group 1")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("case", ["qkv", "proj", "fc1", "fc2", "patch"])
def test_gemm_grouped_bit_identical_to_single(cuda, dt, case):
    """dp_gemm_grouped (the image + FOV encoders' Linears / patch embed as one launch) gives each
    problem exactly what its own dp_gemm call gives -- same engine, same epilogue -- and each
    problem reads its own weights / bias / gamma / pos."""
    g = torch.Generator().manual_seed(11)
    N, K = {"qkv": (3072, 1024), "proj": (1024, 1024), "fc1": (4096, 1024), "fc2": (1024, 4096),
            "patch": (1024, 768)}[case]
    patch = case == "patch"
    M, R = (576 if patch else 577), 577
    A = rnd((1 if patch else 2) * M, K, dt=dt, dev=cuda, gen=g)
    acc = case in ("proj", "fc2")
    cdt = torch.float32 if acc or patch else dt
    C0 = torch.randn(2 * R, N, generator=g).to(cdt).to(cuda)
    kw = dict(M=M, N=N, K=K)
    if case == "fc1":
        kw["act"] = DP_ACT_GELU
    if acc:
        kw["accumulate"] = True
    if patch:
        kw.update(ldpos=N, pos_group=576, pos_off=1, row_group=576, row_group_out=577, row_off=1)
    per = []
    for i in range(2):
        d = dict(A=A, B=rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5),
                 bias=torch.randn(N, generator=g).to(cuda), A_off=0 if patch else i * M * K, C_off=i * R * N)
        if case in ("qkv", "proj", "fc2"):
            d["gamma"] = torch.rand(N, generator=g).to(cuda)
        if patch:
            d["pos"] = torch.randn(577, N, generator=g).to(cuda)
        per.append(d)
    Cg, Cs = C0.clone(), C0.clone()
    ops.gemm_grouped([dict(d, C=Cg) for d in per], **kw)
    for d in per:
        ops.gemm(d["A"], d["B"], Cs, **{k: v for k, v in d.items() if k not in ("A", "B")}, **kw)
    torch.cuda.synchronize()
    assert torch.equal(Cg, Cs), (Cg.float() - Cs.float()).abs().max().item()
    # problem 1 against fp32 torch (its own operands, not problem 0's)
    d = per[1]
    a = A.float()[d["A_off"] // K:d["A_off"] // K + M]
    v = a @ d["B"].float().t() + d["bias"]
    if case == "fc1":
        v = F.gelu(v)
    if "gamma" in d:
        v = v * d["gamma"]
    if patch:
        v = v + d["pos"][1:]
        ref, got = v, Cg[R + 1:2 * R]
    else:
        ref, got = v + (C0[R:2 * R].float() if acc else 0), Cg[R:2 * R]
    close(got, ref, torch.float32 if (acc or patch) and dt == torch.float16 else dt, f"grouped {case}")


@pytest.mark.parametrize("dt", DTYPES)
def test_patchify_pyramid_vs_oracle_split(cuda, dt):
    from oracle import depth_pro_oracle as O

    g = torch.Generator().manual_seed(19)
    x = torch.randn(1, 3, 1536, 1536, generator=g)
    cols = torch.empty(35 * 576, 768, dtype=dt, device=cuda)
    ops.patchify_pyramid(x[0].to(cuda), cols)
    x0, x1, x2 = O.pyramid(x)
    wins = torch.cat((O.split(x0, 0.25), O.split(x1, 0.5), x2), 0)  # (35,3,384,384)
    ref = F.unfold(wins, 16, stride=16).transpose(1, 2).reshape(35 * 576, 768)  # k = c*256+ky*16+kx
    assert torch.equal(cols.cpu(), ref.to(dt)) or (cols.float().cpu() - ref).abs().max() < 1e-2


@pytest.mark.parametrize("dt", DTYPES)
def test_merge_windows_vs_oracle(cuda, dt):
    from oracle import depth_pro_oracle as O

    g = torch.Generator().manual_seed(23)
    tok = torch.randn(35 * 577, 1024, generator=g)
    for (w0, steps, pad, S) in ((0, 5, 3, 96), (25, 3, 6, 48), (34, 1, 0, 24)):
        dst = torch.empty(S * S, 1024, dtype=dt, device=cuda)
        ops.merge_windows(tok.to(cuda), w0, steps, pad, dst)
        win = O.tokens_to_nchw(tok.reshape(35, 577, 1024)[w0:w0 + steps * steps])
        ref = O.merge(win, 1, pad)  # (1,1024,S,S)
        assert torch.equal(dst.cpu(), ref[0].permute(1, 2, 0).reshape(S * S, 1024).to(dt))
        dst2 = torch.empty_like(dst)
        ops.merge_windows(tok.to(cuda).to(dt), w0, steps, pad, dst2)
        assert torch.equal(dst2, dst)


@pytest.mark.parametrize("HW", [(1536, 1536), (1080, 1920), (2268, 3024), (500, 333)])
def test_resize_and_infer_epilogue(cuda, HW):
    H, W = HW
    g = torch.Generator().manual_seed(H)
    x = torch.randn(3, H, W, generator=g)
    out = torch.empty(3, 1536, 1536, device=cuda)
    ops.resize_bilinear(x.to(cuda), out)
    ref = F.interpolate(x[None], size=(1536, 1536), mode="bilinear", align_corners=False)[0]
    assert (out.cpu() - ref).abs().max() < 1e-5
    canon = torch.rand(1, 1, 1536, 1536, generator=g) * 3
    fov = torch.tensor([[[[57.3]]]])
    depth = torch.empty(H, W, device=cuda)
    fpx = torch.empty((), device=cuda)
    ops.infer_epilogue(canon.to(cuda), fov.to(cuda), None, H, W, depth, fpx)
    f_ref = 0.5 * W / torch.tan(0.5 * torch.deg2rad(fov.float()))
    inv = canon * (W / f_ref)
    if (H, W) != (1536, 1536):
        inv = F.interpolate(inv, size=(H, W), mode="bilinear", align_corners=False)
    dref = 1.0 / torch.clamp(inv, 1e-4, 1e4)
    assert abs(fpx.item() - f_ref.item()) <= 1e-5 * f_ref.item()
    np.testing.assert_allclose(depth.cpu().numpy(), dref[0, 0].numpy(), rtol=2e-5, atol=1e-6)
    ops.infer_epilogue(canon.to(cuda), None, 1234.5, H, W, depth, None)
    inv = canon * (W / 1234.5)
    if (H, W) != (1536, 1536):
        inv = F.interpolate(inv, size=(H, W), mode="bilinear", align_corners=False)
    np.testing.assert_allclose(depth.cpu().numpy(), (1.0 / torch.clamp(inv, 1e-4, 1e4))[0, 0].numpy(),
                               rtol=2e-5, atol=1e-6)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mode", ["bilinear", "bicubic"])
def test_resize_same_size_is_a_copy(cuda, dt, mode):
    """dp_resize at input size == output size (the infer prologue of a 1536^2 frame) copies: equal
    to F.interpolate bit for bit on finite inputs, and non-finite ones pass through unchanged (the
    copy of PyTorch's CUDA same-size fast path; its CPU kernel would spread a NaN to a neighbour
    through a zero-weight tap)."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(3, 1536, 1536, generator=g).to(dt)
    out = torch.full((3, 1536, 1536), 7.0, device=cuda)
    ops.resize(x.to(cuda), out, mode)
    ref = F.interpolate(x.float()[None], size=(1536, 1536), mode=mode, align_corners=False)[0]
    assert torch.equal(out.cpu(), ref)
    x[0, 5, 7], x[1, 100, 1535], x[2, 1535, 0] = float("nan"), float("inf"), -float("inf")
    ops.resize(x.to(cuda), out, mode)
    assert torch.equal(out.cpu().nan_to_num(123.0), x.float().nan_to_num(123.0))
    odd = torch.randn(3, 37, 53, generator=g)          # a ragged size, fp32 (the scalar tail)
    o2 = torch.empty(3, 37, 53, device=cuda)
    ops.resize(odd.to(cuda), o2, mode)
    assert torch.equal(o2.cpu(), odd)

@pytest.mark.parametrize("HW", [(1536, 1536), (1080, 1920), (500, 333), (3000, 2000)])
def test_resize_and_infer_epilogue_bicubic(cuda, HW):
    """interpolation_mode="bicubic" (reference depth_pro.py:273-291 passes it to both
    F.interpolate calls): dp_resize / dp_infer_epilogue_mode vs torch's upsample_bicubic2d
    (align_corners=False, A = -0.75, clamped border taps) in fp32 on the CPU."""
    H, W = HW
    g = torch.Generator().manual_seed(H + 7)
    x = torch.randn(3, H, W, generator=g)
    out = torch.empty(3, 1536, 1536, device=cuda)
    ops.resize(x.to(cuda), out, "bicubic")
    ref = F.interpolate(x[None], size=(1536, 1536), mode="bicubic", align_corners=False)[0]
    assert (out.cpu() - ref).abs().max() < 2e-5
    canon = torch.rand(1, 1, 1536, 1536, generator=g) * 3 + 0.01
    fov = torch.tensor([[[[61.0]]]])
    depth = torch.empty(H, W, device=cuda)
    fpx = torch.empty((), device=cuda)
    ops.infer_epilogue(canon.to(cuda), fov.to(cuda), None, H, W, depth, fpx, mode="bicubic")
    f_ref = 0.5 * W / torch.tan(0.5 * torch.deg2rad(fov.float()))
    inv = canon * (W / f_ref)
    if (H, W) != (1536, 1536):
        inv = F.interpolate(inv, size=(H, W), mode="bicubic", align_corners=False)
    # compared as inverse depth (1 / depth = the clamped resize): bicubic overshoot on this noise
    # puts some pixels near the 1e-4 clamp, where depth itself magnifies ulp-level differences
    np.testing.assert_allclose(1.0 / depth.cpu().numpy(), torch.clamp(inv, 1e-4, 1e4)[0, 0].numpy(),
                               rtol=2e-5, atol=2e-6)
    with pytest.raises(ValueError):
        ops.resize(x.to(cuda), out, "nearest")


@pytest.mark.parametrize("case", ["random", "nan", "const", "4k", "viridis"])
def test_depth_to_image_matches_reference_writers(cuda, case):
    """dp_depth_to_image == the reference writers byte for byte: colorize_depth (matplotlib
    turbo over the per-frame nanmin / nanmax, generate_depth_maps.py:15-44) and the --raw uint16
    encoding (:135-143), incl. NaN pixels and a constant map (0/0 -> matplotlib's bad colour)."""
    import generate_depth_maps as G

    rng = np.random.default_rng(len(case))
    H, W = (2160, 3840) if case == "4k" else (333, 517)
    d = (rng.random((H, W), dtype=np.float32) * 30 + 0.05).astype(np.float32)
    if case == "nan":
        d[rng.random((H, W)) < 0.01] = np.nan
    if case == "const":
        d[:] = 7.25
    cmap = "viridis" if case == "viridis" else "turbo"
    dev = torch.from_numpy(d).to(cuda)
    col = ops.depth_to_image(dev, colored=True, cmap=cmap).cpu().numpy()
    raw = ops.depth_to_image(dev, colored=False).cpu().numpy().view(np.uint16)
    with np.errstate(invalid="ignore", divide="ignore"):
        ref_col = G.colorize_depth(d, cmap=cmap)
        ref_raw = G.raw_depth_u16(d)
    assert np.array_equal(col, ref_col), (col != ref_col).sum()
    assert np.array_equal(raw, ref_raw), (raw != ref_raw).sum()


def test_normalize_u8(cuda):
    img = np.random.default_rng(0).integers(0, 256, (300, 200, 3), dtype=np.uint8)
    out = torch.empty(3, 300, 200, device=cuda)
    ops.normalize_u8(torch.from_numpy(img).to(cuda), out)
    ref = (torch.from_numpy(img).permute(2, 0, 1).float().div(255) - 0.5) / 0.5
    assert torch.equal(out.cpu(), ref)


TILES = {"128x128": 1, "256x64": 2, "256x32": 3, "big256x256": 4, "big256x128": 5, "big256x256k32": 6,
         "big256x128k32": 7, "8ph256x256": 8, "dual256x128": 17}


@pytest.mark.parametrize("tile", list(TILES))
def test_gemm_every_tile_engine(cuda, tile):
    """Every tile engine, dense (ragged M) and implicit-conv with ReLU prologue, vs fp32 torch."""
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(TILES[tile])
    M, N, K = 1000, 256, 1024
    A = rnd(M, K, dt=dt, dev=cuda, gen=g)
    B = rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    bias = torch.randn(N, generator=g).to(cuda)
    C = torch.empty(M, N, dtype=dt, device=cuda)
    ops.gemm(A, B, C, M=M, N=N, K=K, bias=bias, tile=TILES[tile])
    close(C, A.float() @ B.float().t() + bias, dt, f"dense {tile}")
    S, cin, cout = 40, 128, 256
    x = rnd(1, cin, S, S, dt=dt, dev=cuda, gen=g)
    w = rnd(cout, cin, 3, 3, dt=dt, dev=cuda, gen=g, scale=(9 * cin) ** -0.5)
    out = torch.empty(S * S, cout, dtype=dt, device=cuda)
    ops.gemm(x.permute(0, 2, 3, 1).contiguous(), ops.conv_weight(w), out,
             M=S * S, N=cout, K=9 * cin, conv=dict(in_h=S, in_w=S, in_c=cin, k=3, stride=1, pad=1, out_h=S, out_w=S),
             relu_a=True, tile=TILES[tile])
    ref = F.conv2d(F.relu(x.float()), w.float(), padding=1)
    close(out.reshape(1, S, S, cout).permute(0, 3, 1, 2), ref, dt, f"conv {tile}")


# ------------------------------------------------------------ stream-K engine
@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M,N,K,mode", [
    (20195, 3072, 1024, "bias"),          # qkv: 948 tiles over 256 persistent workgroups (split tiles)
    (20195, 1024, 1024, "acc"),           # proj: fp32 residual accumulate + LayerScale
    (5000, 1024, 4096, "acc"),            # fc2-like, long K
    (20195, 4096, 1024, "gelu"),          # fc1
    (300, 256, 64, "bias"),               # 2 tiles, 1 k-step
    (4100, 512, 192, "bias"),             # 34 tiles x 3 k-steps, ragged last m-tile
])
def test_gemm_stream_k_matches_reference_and_data_parallel(cuda, dt, M, N, K, mode):
    g = torch.Generator().manual_seed(M + 7 * N + K)
    A = rnd(M, K, dt=dt, dev=cuda, gen=g)
    B = rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    bias = torch.randn(N, generator=g).to(cuda)
    gamma = torch.rand(N, generator=g).to(cuda)
    ws = ops.gemm_workspace(cuda)
    kw = dict(M=M, N=N, K=K, bias=bias)
    ref = A.float() @ B.float().t() + bias
    if mode == "acc":
        X = torch.randn(M, N, generator=g).to(cuda)
        kw.update(gamma=gamma, accumulate=True)
        C1, C2 = X.clone(), X.clone()
        ref = X + gamma * ref
    else:
        if mode == "gelu":
            kw.update(act=DP_ACT_GELU)
            ref = F.gelu(ref)
        C1 = torch.empty(M, N, dtype=dt, device=cuda)
        C2 = torch.empty(M, N, dtype=dt, device=cuda)
    ops.gemm(A, B, C1, tile=DP_TILE_STREAMK_256x256, workspace=ws, **kw)
    ops.gemm(A, B, C2, tile=DP_TILE_BIG_256x256, **kw)
    torch.cuda.synchronize()
    assert int(ws[4092:4096].view(torch.int32).item()) == 0, "stream-K partial wait timed out"
    close(C1, ref, torch.float32 if (mode == "acc" and dt == torch.float16) else dt, "stream-K")
    # same tiles, same k order except where a tile's k range was split: fp32 sums agree to rounding
    d = (C1.float() - C2.float()).abs().max().item()
    assert d <= 1e-2 * (C2.float().abs().max().item() + 1e-6), d
    # deterministic: a second run is bit-identical
    C3 = X.clone() if mode == "acc" else torch.empty_like(C1)
    ops.gemm(A, B, C3, tile=DP_TILE_STREAMK_256x256, workspace=ws, **kw)
    assert torch.equal(C1, C3)


@pytest.mark.parametrize("dt", DTYPES)
def test_gemm_stream_k_conv3x3_relu_residual(cuda, dt):
    """Implicit-GEMM 3x3 conv (decoder ResidualBlock shape) through the stream-K engine."""
    g = torch.Generator().manual_seed(11)
    S, C = 96, 256
    x = rnd(1, C, S, S, dt=dt, dev=cuda, gen=g)
    w = rnd(C, C, 3, 3, dt=dt, dev=cuda, gen=g, scale=(9 * C) ** -0.5)
    b = torch.randn(C, generator=g).to(cuda)
    r = rnd(1, C, S, S, dt=dt, dev=cuda, gen=g)
    xh = x.permute(0, 2, 3, 1).reshape(S * S, C).contiguous()
    rh = r.permute(0, 2, 3, 1).reshape(S * S, C).contiguous()
    wp = ops.conv_weight(w)
    out = torch.empty(S * S, C, dtype=dt, device=cuda)
    ops.gemm(xh, wp, out, M=S * S, N=C, K=9 * C, conv=dict(in_h=S, in_w=S, in_c=C, k=3, stride=1, pad=1,
                                                            out_h=S, out_w=S),
             relu_a=True, bias=b, R1=rh, ldr1=C, tile=DP_TILE_STREAMK_256x256, workspace=ops.gemm_workspace(cuda))
    ref = F.conv2d(F.relu(x.float()), w.float(), b, padding=1) + r.float()
    close(out.reshape(1, S, S, C).permute(0, 3, 1, 2), ref, dt, "stream-K conv3x3")


SPLITK_CASES = [
    # (name, M, N, K, conv side / None, mode)
    ("rb conv 48^2 relu+res", 48 * 48, 256, 2304, 48, "rb"),
    ("proj conv 96^2 1024ch", 96 * 96, 256, 9216, 96, "bias"),
    ("dense ragged gelu", 2000, 512, 2048, None, "gelu"),
    ("dense fp32 accumulate", 1500, 256, 4096, None, "acc"),
]


@pytest.mark.parametrize("case", SPLITK_CASES, ids=[c[0] for c in SPLITK_CASES])
@pytest.mark.parametrize("dt", DTYPES)
def test_gemm_split_k_matches_reference_and_data_parallel(cuda, dt, case):
    """Split-K for small grids (DP_TILE_SPLITK_256x256 hint, with a workspace): the 256 x
    256 engine over K ranges writing fp32 partials, then the reduce launch with the row epilogue.
    vs an fp32 reference, close to the data-parallel engine (only the fp32 summation order
    differs), and bit-identical run to run (partials summed in split order)."""
    name, M, N, K, S, mode = case
    g = torch.Generator().manual_seed(M + N + K)
    ws = ops.gemm_workspace(cuda)
    B = rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    bias = torch.randn(N, generator=g).to(cuda)
    kw = dict(M=M, N=N, K=K, bias=bias)
    if S is not None:
        cin = K // 9
        x = rnd(1, cin, S, S, dt=dt, dev=cuda, gen=g)
        A = x.permute(0, 2, 3, 1).reshape(S * S, cin).contiguous()
        w = B.float().cpu().reshape(N, cin // 64, 3, 3, 64).permute(0, 1, 4, 2, 3).reshape(N, cin, 3, 3)
        kw["conv"] = dict(in_h=S, in_w=S, in_c=cin, k=3, stride=1, pad=1, out_h=S, out_w=S)
        xin = F.relu(x.float()) if mode == "rb" else x.float()
        ref = F.conv2d(xin, w.to(cuda), bias, padding=1).permute(0, 2, 3, 1).reshape(M, N)
    else:
        A = rnd(M, K, dt=dt, dev=cuda, gen=g)
        ref = A.float() @ B.float().t() + bias
    if mode == "rb":
        R = rnd(M, N, dt=dt, dev=cuda, gen=g)
        kw.update(relu_a=True, R1=R, ldr1=N)
        ref = ref + R.float()
    if mode == "gelu":
        kw.update(act=DP_ACT_GELU)
        ref = F.gelu(ref)
    if mode == "acc":
        X = torch.randn(M, N, generator=g).to(cuda)
        gamma = torch.rand(N, generator=g).to(cuda)
        kw.update(gamma=gamma, accumulate=True)
        ref = X + gamma * ref
        C1, C2, C3 = X.clone(), X.clone(), X.clone()
    else:
        C1, C2, C3 = (torch.empty(M, N, dtype=dt, device=cuda) for _ in range(3))
    SPK = DP_TILE_SPLITK_256x256
    tile, wgs = ops.gemm(A, B, C1, plan_only=True, workspace=ws, tile=SPK, **kw)
    assert tile == SPK and wgs > (M + 255) // 256 * (N // 256), (tile, wgs)
    ops.gemm(A, B, C1, workspace=ws, tile=SPK, **kw)
    ops.gemm(A, B, C2, tile=DP_TILE_BIG_256x256, **kw)
    ops.gemm(A, B, C3, workspace=ws, tile=SPK, **kw)
    torch.cuda.synchronize()
    close(C1, ref, torch.float32 if (mode == "acc" and dt == torch.float16) else dt, f"split-K {name}")
    d = (C1.float() - C2.float()).abs().max().item()
    assert d <= 1e-2 * (C2.float().abs().max().item() + 1e-6), d
    assert torch.equal(C1, C3)


ENGINES = [DP_TILE_BIG_256x256, DP_TILE_8PH_256x256, DP_TILE_BIG_320x256, DP_TILE_BIG_256x128, DP_TILE_BIG_512x128,
           DP_TILE_STREAMK_256x256, DP_TILE_DUAL_256x128]


@pytest.mark.parametrize("tile", ENGINES)
@pytest.mark.parametrize("dt", DTYPES)
def test_every_big_engine_on_ragged_conv_and_dense(cuda, dt, tile):
    """Each tile engine on a ragged-M dense GEMM (bias + GELU) and a strided 3x3 conv with ReLU-on-load."""
    g = torch.Generator().manual_seed(tile)
    ws = ops.gemm_workspace(cuda)
    M, N, K = 1337, 512, 320
    A = rnd(M, K, dt=dt, dev=cuda, gen=g)
    B = rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    bias = torch.randn(N, generator=g).to(cuda)
    C = torch.empty(M, N, dtype=dt, device=cuda)
    ops.gemm(A, B, C, M=M, N=N, K=K, bias=bias, act=DP_ACT_GELU, tile=tile, workspace=ws)
    close(C, F.gelu(A.float() @ B.float().t() + bias), dt, f"dense tile {tile}")
    S, Ci, Co = 50, 128, 256
    x = rnd(1, Ci, S, S, dt=dt, dev=cuda, gen=g)
    w = rnd(Co, Ci, 3, 3, dt=dt, dev=cuda, gen=g, scale=(9 * Ci) ** -0.5)
    So = (S + 2 - 3) // 2 + 1
    out = torch.empty(So * So, Co, dtype=dt, device=cuda)
    ops.gemm(x.permute(0, 2, 3, 1).reshape(S * S, Ci).contiguous(), ops.conv_weight(w),
             out, M=So * So, N=Co, K=9 * Ci, conv=dict(in_h=S, in_w=S, in_c=Ci, k=3, stride=2, pad=1, out_h=So, out_w=So),
             relu_a=True, tile=tile, workspace=ws)
    ref = F.conv2d(F.relu(x.float()), w.float(), stride=2, padding=1)
    close(out.reshape(1, So, So, Co).permute(0, 3, 1, 2), ref, dt, f"conv tile {tile}")


@pytest.mark.parametrize("dt", DTYPES)
def test_head_pixel_shuffle_epilogue(cuda, dt):
    """Composed depth head (deconv -> 3x3 -> ReLU -> 1x1 -> ReLU) as one HEAD_PS GEMM vs the layer order."""
    from depth_pro.engine import compose_head

    g = torch.Generator().manual_seed(21)
    ci, H, W = 128, 40, 36
    h0 = (torch.randn(1, ci, H, W, generator=g)).to(dt).float()
    wd = torch.randn(ci, ci, 2, 2, generator=g) * ci ** -0.5
    bd = torch.randn(ci, generator=g)
    w2 = torch.randn(32, ci, 3, 3, generator=g) * (9 * ci) ** -0.5
    b2 = torch.randn(32, generator=g)
    w4 = torch.randn(32, generator=g) * 32 ** -0.5
    P = {k: (v.to(cuda) if torch.is_tensor(v) else v) for k, v in compose_head(wd, bd, w2, b2, dt).items()}
    out = torch.full((2 * H, 2 * W), float("nan"), device=cuda)
    x = h0[0].permute(1, 2, 0).reshape(H * W, ci).contiguous().to(dt).to(cuda)
    ops.gemm(x, P["head.ps.w"], out, M=H * W, N=128, K=9 * ci,
             conv=dict(in_h=H, in_w=W, in_c=ci, k=3, stride=1, pad=1, out_h=H, out_w=W),
             bias=P["head.ps.b"], head_w=w4.to(cuda), head_b=0.25, head_corr=P["head.ps.corr"])
    ref = F.conv_transpose2d(h0, wd, bd, stride=2)
    ref = F.relu(F.conv2d(F.relu(F.conv2d(ref, w2, b2, padding=1)), w4.reshape(1, 32, 1, 1), torch.tensor([0.25])))
    close(out, ref[0, 0], dt, "head HEAD_PS")


def test_gemm_stream_k_timeout_sets_sticky_error_word(cuda):
    """Fault injection (debug bit 64: every partial wait gives up at once): the sticky
    error word of the workspace is set, survives the next launch's flag clear, and
    Engine-level callers see it through ops.workspace_error."""
    from depth_pro import _lib

    g = torch.Generator().manual_seed(5)
    M, N, K = 20195, 3072, 1024           # 948 tiles on 256 workgroups: split tiles -> hand-offs
    A = rnd(M, K, dt=torch.bfloat16, dev=cuda, gen=g)
    B = rnd(N, K, dt=torch.bfloat16, dev=cuda, gen=g, scale=K ** -0.5)
    C = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
    ws = ops.gemm_workspace(cuda)
    ops.gemm(A, B, C, M=M, N=N, K=K, tile=DP_TILE_STREAMK_256x256, workspace=ws)
    assert ops.workspace_error(ws) == 0
    lib = _lib.load()
    lib.dp_gemm_debug_flags(64)
    try:
        ops.gemm(A, B, C, M=M, N=N, K=K, tile=DP_TILE_STREAMK_256x256, workspace=ws)
        torch.cuda.synchronize()
    finally:
        lib.dp_gemm_debug_flags(0)
    assert ops.workspace_error(ws) != 0
    ops.gemm(A, B, C, M=M, N=N, K=K, tile=DP_TILE_STREAMK_256x256, workspace=ws)   # clean launch
    assert ops.workspace_error(ws) != 0, "error word must be sticky across launches"


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("pair", ["320", "256"])
@pytest.mark.parametrize("case", ["dense_bias", "gelu_ragged", "acc_f32", "conv_relu_res", "rowgroup"])
def test_persistent_engine_bit_identical_to_data_parallel(cuda, dt, pair, case):
    """The persistent big engine (DP_TILE_PBIG_*: tile loop, next tile's first K step under the
    epilogue, bounded buffer stores) computes every tile exactly as the data-parallel engine:
    bit-identical C, including ragged last tiles (dropped out-of-range stores) and the fp32
    accumulate / residual / row-group-remap epilogues."""
    from depth_pro._lib import DP_TILE_PBIG_256x256, DP_TILE_PBIG_320x256

    tp, tb = (DP_TILE_PBIG_320x256, DP_TILE_BIG_320x256) if pair == "320" else (DP_TILE_PBIG_256x256,
                                                                                  DP_TILE_BIG_256x256)
    g = torch.Generator().manual_seed(sum(map(ord, case)))
    kw = {}
    if case == "conv_relu_res":
        S, C = 96, 256
        A = rnd(S * S, C, dt=dt, dev=cuda, gen=g)
        M, N, K = S * S, 256, 9 * C
        kw = dict(conv=dict(in_h=S, in_w=S, in_c=C, k=3, stride=1, pad=1, out_h=S, out_w=S), relu_a=True,
                  R1=rnd(M, N, dt=dt, dev=cuda, gen=g), ldr1=N, R2=rnd(M, N, dt=dt, dev=cuda, gen=g), ldr2=N)
    else:
        M, N, K = {"dense_bias": (20195, 3072, 1024), "gelu_ragged": (4999, 1536, 512),
                   "acc_f32": (3001, 1024, 2048), "rowgroup": (35 * 576, 1024, 768)}[case]
        A = rnd(M, K, dt=dt, dev=cuda, gen=g)
    B = rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    bias = torch.randn(N, generator=g).to(cuda)
    kw.update(bias=bias)
    if case == "gelu_ragged":
        kw.update(act=DP_ACT_GELU)
    rows = M
    if case == "rowgroup":   # patch-embed remap: 576 rows per window -> 577 with a cls row in front
        kw.update(row_group=576, row_group_out=577, row_off=1)
        rows = 35 * 577
    if case == "acc_f32":
        kw.update(gamma=torch.rand(N, generator=g).to(cuda), accumulate=True)
        C0 = torch.randn(rows, N, generator=g).to(cuda)
        C1, C2 = C0.clone(), C0.clone()
    else:
        cdt = torch.float32 if case == "rowgroup" else dt
        C1 = torch.full((rows, N), 7.0, dtype=cdt, device=cuda)
        C2 = C1.clone()
    ops.gemm(A, B, C1, M=M, N=N, K=K, tile=tp, **kw)
    ops.gemm(A, B, C2, M=M, N=N, K=K, tile=tb, **kw)
    torch.cuda.synchronize()
    assert torch.equal(C1, C2), (C1.float() - C2.float()).abs().max().item()


@pytest.mark.parametrize("dt", DTYPES)
def test_conv3x3_border_corrected_composition(cuda, dt):
    """dp_gemm DP_STORE_ROWS with head_corr (the decoder out_conv composed into head.0,
    engine.compose_head0): equals the reference 1x1 conv then zero-padded 3x3 conv in fp32, at
    96 x 96 x 256 -> 128 (the 768^2 shape's engine family), every border pixel included."""
    from depth_pro.engine import compose_head0

    g = torch.Generator().manual_seed(41)
    S, c, o = 96, 256, 128
    y = torch.randn(1, c, S, S, generator=g)
    wo = torch.randn(c, c, generator=g) * c ** -0.5
    bo = torch.randn(c, generator=g)
    w0 = torch.randn(o, c, 3, 3, generator=g) * (9 * c) ** -0.5
    b0 = torch.randn(o, generator=g)
    yq = y.to(dt).float()
    ref = F.conv2d(F.conv2d(yq, wo[:, :, None, None], bo), w0, b0, padding=1)[0].permute(1, 2, 0).reshape(S * S, o)
    P = {k: v.to(cuda) for k, v in compose_head0(w0, b0, wo, bo, dt).items()}
    x = yq[0].permute(1, 2, 0).reshape(S * S, c).contiguous().to(dt).to(cuda)
    out = torch.full((S * S, o), float("nan"), dtype=dt, device=cuda)
    ops.gemm(x, P["head.0c.w"], out, M=S * S, N=o, K=9 * c,
             conv=dict(in_h=S, in_w=S, in_c=c, k=3, stride=1, pad=1, out_h=S, out_w=S),
             bias=P["head.0c.b"], border_corr=P["head.0c.corr"], tile=DP_TILE_BIG_512x128)
    close(out, ref, dt, "border-corrected composed conv")


def test_border_correction_rejects_relu_prologue(cuda):
    """head_corr (composed-conv border correction) exists only in the non-ReLU 512x128 conv
    instantiation: a ReLU-on-load request must be refused on the host, not run uncorrected."""
    from depth_pro._lib import DPError

    S, c, o = 32, 128, 128
    x = torch.zeros(S * S, c, dtype=torch.float16, device=cuda)
    w = torch.zeros(o, 9 * c, dtype=torch.float16, device=cuda)
    out = torch.empty(S * S, o, dtype=torch.float16, device=cuda)
    corr = torch.zeros(9 * o, device=cuda)
    kw = dict(M=S * S, N=o, K=9 * c, conv=dict(in_h=S, in_w=S, in_c=c, k=3, stride=1, pad=1, out_h=S, out_w=S),
              border_corr=corr, tile=DP_TILE_BIG_512x128)
    ops.gemm(x, w, out, **kw)                              # accepted without the ReLU prologue
    with pytest.raises(DPError, match="DP_ERR_ARG"):
        ops.gemm(x, w, out, relu_a=True, **kw)


@pytest.mark.parametrize("dt", DTYPES)
def test_fov_tail_vs_conv2d(cuda, dt):
    """dp_fov_tail (fov.py:46, head[4]: Conv2d(32, 1, 6) + bias on the 6x6x32 map) vs F.conv2d."""
    g = torch.Generator().manual_seed(46)
    x = torch.randn(1, 32, 6, 6, generator=g).to(dt)
    w = torch.randn(1, 32, 6, 6, generator=g) * 0.1
    b = 0.37
    x6 = x[0].permute(1, 2, 0).contiguous().to(cuda)      # NHWC 6x6x32
    out = torch.empty(1, 1, 1, 1, device=cuda)
    ops.fov_tail(x6, w.reshape(-1).contiguous().to(cuda), b, out)
    ref = F.conv2d(x.float(), w, torch.tensor([b]))
    assert abs(out.item() - ref.item()) <= 1e-5 * max(1.0, abs(ref.item())), (out.item(), ref.item())


def test_infer_epilogue_counts_nonfinite_and_keeps_nan(cuda):
    """dp_infer_epilogue's health word: NaN / inf depth values are counted (and a NaN stays NaN,
    as torch.clamp does), a finite map counts nothing; a NaN FOV (hence f_px) counts too."""
    canon = torch.rand(1, 1, 1536, 1536, device=cuda) + 0.5
    fov = torch.full((1, 1, 1, 1), 60.0, device=cuda)
    bad = torch.zeros(1, dtype=torch.int32, device=cuda)
    depth = torch.empty(1536, 1536, device=cuda)
    fpx = torch.empty((), device=cuda)
    ops.infer_epilogue(canon, fov, None, 1536, 1536, depth, fpx, bad)
    assert int(bad) == 0
    canon[0, 0, 5, 7] = float("nan")
    canon[0, 0, 900, 11] = float("nan")
    ops.infer_epilogue(canon, fov, None, 1536, 1536, depth, fpx, bad)
    assert int(bad) == 2 and torch.isnan(depth[5, 7]) and torch.isnan(depth[900, 11])
    ref = 1.0 / torch.clamp(canon * (1536 / fpx), 1e-4, 1e4)
    assert torch.equal(torch.isnan(depth), torch.isnan(ref[0, 0]))
    bad.zero_()
    canon[0, 0, 5, 7] = 1.0
    canon[0, 0, 900, 11] = 1.0
    ops.infer_epilogue(canon, torch.full_like(fov, float("nan")), None, 1536, 1536, depth, fpx, bad)
    assert int(bad) == 1 + 1536 * 1536       # f_px and every depth value


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("case", ["fc1_gelu", "qkv_gamma", "ragged_few_tiles", "k128_many_tiles", "relu_a_n256"])
def test_persistent_8phase_bit_identical_to_8phase(cuda, dt, case):
    """The persistent 8-phase engine (DP_TILE_P8PH_256x256: the workgroup's tiles as one stream of
    K steps, the next tile's loads in flight under each epilogue, column constants by LDS-DMA,
    counted buffer stores) computes every tile exactly as the 8-phase engine: bit-identical C,
    incl. ragged last M tiles, K = 128 (a tile boundary every other step) and > 1 tile per
    workgroup; and both match fp32 torch."""
    from depth_pro._lib import DP_TILE_P8PH_256x256

    g = torch.Generator().manual_seed(sum(map(ord, case)))
    M, N, K = {"fc1_gelu": (20195, 4096, 1024), "qkv_gamma": (20195, 3072, 1024),
               "ragged_few_tiles": (4999, 1536, 512), "k128_many_tiles": (20000, 2048, 128),
               "relu_a_n256": (9000, 256, 576)}[case]
    A = rnd(M, K, dt=dt, dev=cuda, gen=g)
    B = rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    bias = torch.randn(N, generator=g).to(cuda)
    kw = dict(M=M, N=N, K=K, bias=bias)
    ref = A.float() @ B.float().t() + bias
    if case in ("fc1_gelu", "ragged_few_tiles"):
        kw.update(act=DP_ACT_GELU)
        ref = F.gelu(ref)
    if case == "qkv_gamma":
        gamma = torch.rand(N, generator=g).to(cuda) + 0.5
        kw.update(gamma=gamma)
        ref = ref * gamma
    if case == "relu_a_n256":
        kw.update(relu_a=True)
        ref = F.relu(A.float()) @ B.float().t() + bias
    C1 = torch.full((M, N), 7.0, dtype=dt, device=cuda)
    C2 = C1.clone()
    ops.gemm(A, B, C1, tile=DP_TILE_P8PH_256x256, **kw)
    ops.gemm(A, B, C2, tile=DP_TILE_8PH_256x256, **kw)
    torch.cuda.synchronize()
    assert torch.equal(C1, C2), (C1.float() - C2.float()).abs().max().item()
    close(C1, ref, dt, f"p8ph {case}")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("case", ["qkv_gamma", "proj_acc", "fc2_acc", "ragged_k192", "k64", "k128_gelu"])
def test_8phase_320_bit_identical_to_320(cuda, dt, case):
    """The 8-phase 320 x 256 engine (DP_TILE_8PH_320x256: 4 x 2 waves, one 32-column quarter per
    phase, counted waits every phase) computes every tile exactly as the 320 x 256 big engine:
    bit-identical C for the load-free (bias / gamma / GELU, 16-bit C) and the fp32 residual
    accumulate epilogues, incl. a ragged last row tile and K = 64 / 128 / 192 (the loop's
    tail issue counts); both match fp32 torch."""
    from depth_pro._lib import DP_TILE_8PH_320x256

    g = torch.Generator().manual_seed(sum(map(ord, case)) + 3)
    M, N, K = {"qkv_gamma": (20195, 3072, 1024), "proj_acc": (20195, 1024, 1024), "fc2_acc": (20195, 1024, 4096),
               "ragged_k192": (1000, 512, 192), "k64": (700, 256, 64), "k128_gelu": (3001, 768, 128)}[case]
    A = rnd(M, K, dt=dt, dev=cuda, gen=g)
    B = rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    bias = torch.randn(N, generator=g).to(cuda)
    kw = dict(M=M, N=N, K=K, bias=bias)
    ref = A.float() @ B.float().t() + bias
    if case in ("qkv_gamma", "proj_acc", "fc2_acc"):
        gamma = torch.rand(N, generator=g).to(cuda) + 0.5
        kw.update(gamma=gamma)
        ref = ref * gamma
    if case == "k128_gelu":
        kw.update(act=DP_ACT_GELU)
        ref = F.gelu(ref)
    if case.endswith("_acc"):
        kw.update(accumulate=True)
        X = torch.randn(M, N, generator=g).to(cuda)
        C1, C2 = X.clone(), X.clone()
        ref = ref + X
        cdt = torch.float32 if dt == torch.float16 else dt
    else:
        C1 = torch.full((M, N), 7.0, dtype=dt, device=cuda)
        C2 = C1.clone()
        cdt = dt
    ops.gemm(A, B, C1, tile=DP_TILE_8PH_320x256, **kw)
    ops.gemm(A, B, C2, tile=DP_TILE_BIG_320x256, **kw)
    torch.cuda.synchronize()
    assert torch.equal(C1, C2), (C1.float() - C2.float()).abs().max().item()
    close(C1, ref, cdt, f"8ph320 {case}")


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("th", [16, 12])
@pytest.mark.parametrize("case", ["relu_bias_relu", "residual2", "cin128_n512",
                                  "big_relu_bias_relu", "big_residual2_cin192", "big_cin128_n512"])
def test_patch_conv3x3_bit_identical(cuda, dt, case, th):
    """The 3x3 patch-conv engine (DP_TILE_CV3_256x256: 16 x 16 pixel tiles, the input patch of a
    channel block in LDS, the 9 taps read from it) gives exactly the 256 x 256 big engine's result
    -- same K order, same zero padding, same epilogue -- for the decoder ResidualBlock convs (ReLU
    on load + bias + ReLU; bias + two residuals), 2 images, a wider N; and matches F.conv2d.
    big_*: more tiles than CUs (576 tiles; 2 x 256 tiles with 3 channel blocks = an odd K-step count
    per tile; 2 column tiles of 144).  th = 12: the 12 x 16-pixel tiles (DP_TILE_CV3_192x256), maps
    whose side is a multiple of 48."""
    from depth_pro._lib import DP_TILE_CV3_192x256, DP_TILE_CV3_256x256

    g = torch.Generator().manual_seed(sum(map(ord, case)))
    S, Ci, Co, nb = {"relu_bias_relu": (96, 256, 256, 1), "residual2": (64, 256, 256, 2),
                     "cin128_n512": (48, 128, 512, 1), "big_relu_bias_relu": (384, 256, 256, 1),
                     "big_residual2_cin192": (256, 192, 256, 2), "big_cin128_n512": (192, 128, 512, 1)}[case]
    if th == 12 and S % 48:
        if case == "residual2":
            S = 48          # the residual epilogue on 12-row tiles too
        else:
            pytest.skip("12-row tiles need a side divisible by 48")
    tile = DP_TILE_CV3_256x256 if th == 16 else DP_TILE_CV3_192x256
    x = rnd(nb, Ci, S, S, dt=dt, dev=cuda, gen=g)
    w = rnd(Co, Ci, 3, 3, dt=dt, dev=cuda, gen=g, scale=(9 * Ci) ** -0.5)
    b = torch.randn(Co, generator=g).to(cuda)
    xh = x.permute(0, 2, 3, 1).reshape(nb * S * S, Ci).contiguous()
    kw = dict(M=nb * S * S, N=Co, K=9 * Ci, conv=dict(in_h=S, in_w=S, in_c=Ci, k=3, stride=1, pad=1, out_h=S, out_w=S),
              bias=b)
    ref = F.conv2d(x.float(), w.float(), b, padding=1)
    if case.endswith("relu_bias_relu"):
        kw.update(relu_a=True, act=DP_ACT_RELU)
        ref = F.relu(F.conv2d(F.relu(x.float()), w.float(), b, padding=1))
    elif "residual2" in case:
        r1 = rnd(nb * S * S, Co, dt=dt, dev=cuda, gen=g)
        r2 = rnd(nb * S * S, Co, dt=dt, dev=cuda, gen=g)
        kw.update(R1=r1, ldr1=Co, R2=r2, ldr2=Co)
        ref = ref + (r1.float() + r2.float()).reshape(nb, S, S, Co).permute(0, 3, 1, 2)
    out1 = torch.full((nb * S * S, Co), 7.0, dtype=dt, device=cuda)
    out2 = out1.clone()
    ops.gemm(xh, ops.conv_weight(w), out1, tile=tile, **kw)
    ops.gemm(xh, ops.conv_weight(w), out2, tile=DP_TILE_BIG_256x256, **kw)
    torch.cuda.synchronize()
    assert torch.equal(out1, out2), (out1.float() - out2.float()).abs().max().item()
    close(out1.reshape(nb, S, S, Co).permute(0, 3, 1, 2), ref, dt, f"cv3 {case} th {th}")


def test_patch_conv3x3_planner_tiles(cuda):
    """The planner's patch-conv tiles for the decoder ResidualBlock shapes: 16 x 16 at 768^2 (2304
    tiles = whole rounds), 12 x 16 at 384^2 (768 = 3 rounds; 16 x 16 would make 2.25) and at 192^2
    (one round of 192 workgroups)."""
    from depth_pro._lib import DP_TILE_CV3_192x256, DP_TILE_CV3_256x256

    A = torch.empty(8, dtype=torch.float16, device=cuda)
    want = {768: DP_TILE_CV3_256x256}
    if torch.cuda.get_device_properties(cuda).multi_processor_count == 256:
        want[384] = DP_TILE_CV3_192x256
        want[192] = DP_TILE_CV3_192x256     # a single round of 192 workgroups instead of 144
    for S, t in want.items():
        conv = dict(in_h=S, in_w=S, in_c=256, k=3, stride=1, pad=1, out_h=S, out_w=S)
        tile, _ = ops.gemm(A, A, A, M=S * S, N=256, K=2304, conv=conv, relu_a=True, act=DP_ACT_RELU, plan_only=True)
        assert tile == t, (S, tile)


@pytest.mark.parametrize("dt", DTYPES)
def test_patch_conv3x3_head_epilogues(cuda, dt):
    """The patch-conv engine's head convs (128 output channels per tile): the border-corrected
    composed conv (out_conv∘head.0) bit-identical to the 512 x 128 engine on 16 x 16- and 24 x 16-pixel
    tiles (DP_TILE_CV3_384x128, 4 x 6 tiles of a 96^2 map), and the composed depth
    head (HEAD_PS: deconv∘3x3∘ReLU∘1x1∘ReLU, one parity per wave) equal to it up to the order of
    the 32-channel dot product; both against the reference layer order in fp32."""
    from depth_pro._lib import DP_TILE_CV3_256x256, DP_TILE_CV3_384x128
    from depth_pro.engine import compose_head, compose_head0

    g = torch.Generator().manual_seed(43)
    S, c, o = 96, 256, 128
    y = torch.randn(1, c, S, S, generator=g)
    wo = torch.randn(c, c, generator=g) * c ** -0.5
    bo = torch.randn(c, generator=g)
    w0 = torch.randn(o, c, 3, 3, generator=g) * (9 * c) ** -0.5
    b0 = torch.randn(o, generator=g)
    yq = y.to(dt).float()
    ref = F.conv2d(F.conv2d(yq, wo[:, :, None, None], bo), w0, b0, padding=1)[0].permute(1, 2, 0).reshape(S * S, o)
    P = {k: v.to(cuda) for k, v in compose_head0(w0, b0, wo, bo, dt).items()}
    x = yq[0].permute(1, 2, 0).reshape(S * S, c).contiguous().to(dt).to(cuda)
    kw = dict(M=S * S, N=o, K=9 * c, conv=dict(in_h=S, in_w=S, in_c=c, k=3, stride=1, pad=1, out_h=S, out_w=S),
              bias=P["head.0c.b"], border_corr=P["head.0c.corr"])
    out1 = torch.full((S * S, o), float("nan"), dtype=dt, device=cuda)
    out2 = out1.clone()
    ops.gemm(x, P["head.0c.w"], out1, tile=DP_TILE_CV3_256x256, **kw)
    ops.gemm(x, P["head.0c.w"], out2, tile=DP_TILE_BIG_512x128, **kw)
    out3 = torch.full_like(out1, float("nan"))
    ops.gemm(x, P["head.0c.w"], out3, tile=DP_TILE_CV3_384x128, **kw)
    torch.cuda.synchronize()
    assert torch.equal(out1, out2), (out1.float() - out2.float()).abs().max().item()
    assert torch.equal(out3, out2), (out3.float() - out2.float()).abs().max().item()
    close(out1, ref, dt, "cv3 border-corrected composed conv")

    ci, H = 128, 48
    h0 = torch.randn(1, ci, H, H, generator=g).to(dt).float()
    wd = torch.randn(ci, ci, 2, 2, generator=g) * ci ** -0.5
    bd = torch.randn(ci, generator=g)
    w2 = torch.randn(32, ci, 3, 3, generator=g) * (9 * ci) ** -0.5
    b2 = torch.randn(32, generator=g)
    w4 = torch.randn(32, generator=g) * 32 ** -0.5
    Q = {k: (v.to(cuda) if torch.is_tensor(v) else v) for k, v in compose_head(wd, bd, w2, b2, dt).items()}
    xh = h0[0].permute(1, 2, 0).reshape(H * H, ci).contiguous().to(dt).to(cuda)
    kh = dict(M=H * H, N=128, K=9 * ci, conv=dict(in_h=H, in_w=H, in_c=ci, k=3, stride=1, pad=1, out_h=H, out_w=H),
              bias=Q["head.ps.b"], head_w=w4.to(cuda), head_b=0.25, head_corr=Q["head.ps.corr"])
    d1 = torch.full((2 * H, 2 * H), float("nan"), device=cuda)
    d2 = d1.clone()
    ops.gemm(xh, Q["head.ps.w"], d1, tile=DP_TILE_CV3_256x256, **kh)
    ops.gemm(xh, Q["head.ps.w"], d2, tile=DP_TILE_BIG_512x128, **kh)
    d3 = torch.full_like(d1, float("nan"))
    ops.gemm(xh, Q["head.ps.w"], d3, tile=DP_TILE_CV3_384x128, **kh)
    torch.cuda.synchronize()
    assert not torch.isnan(d1).any()
    assert (d1 - d2).abs().max().item() <= 1e-5 * (d2.abs().max().item() + 1e-6)
    assert torch.equal(d3, d1)      # 24- and 16-row tiles: the same lanes sum the same products
    r = F.conv_transpose2d(h0, wd, bd, stride=2)
    r = F.relu(F.conv2d(F.relu(F.conv2d(r, w2, b2, padding=1)), w4.reshape(1, 32, 1, 1), torch.tensor([0.25])))
    close(d1, r[0, 0], dt, "cv3 head HEAD_PS")


def _chunk_stats(x):
    """(mean, M2) of each 128-column chunk of fp32 rows x, in fp64 (the folded-LN statistics)."""
    c = x.double().reshape(x.shape[0], -1, 128)
    mu = c.mean(-1)
    return torch.stack((mu, ((c - mu[..., None]) ** 2).sum(-1)), -1)


@pytest.mark.parametrize("dt", DTYPES)
def test_layernorm_stats(cuda, dt):
    """dp_layernorm_stats: x in 16 bits (exactly x.to(dt)) + per-128-column (mean, M2)."""
    g = torch.Generator().manual_seed(11)
    rows = 1155
    x = torch.randn(rows, 1024, generator=g) * 3 + torch.randn(rows, 1, generator=g) * 2
    xb = torch.empty(rows, 1024, dtype=dt, device=cuda)
    part = torch.empty(rows, 8, 2, device=cuda)
    ops.layernorm_stats(x.to(cuda), xb, part, rows, 1024)
    assert torch.equal(xb.cpu(), x.to(dt))
    ref = _chunk_stats(x)
    np.testing.assert_allclose(part.cpu().double().numpy(), ref.numpy(), rtol=2e-5, atol=1e-4)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M,K", [(20195, 1024), (577, 4096)])
def test_gemm_8ph320_ln_producer(cuda, dt, M, K):
    """Folded-LN producer (the ViT proj / fc2 with ln_out): C is bit-identical to the plain
    residual launch, xb == the new C rows in 16 bits, part == their 128-column chunk stats."""
    g = torch.Generator().manual_seed(M + K)
    N = 1024
    A = rnd(M, K, dt=dt, dev=cuda, gen=g)
    B = rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    bias = torch.randn(N, generator=g).to(cuda)
    gamma = (0.1 + 0.02 * torch.randn(N, generator=g)).to(cuda)
    C0 = (torch.randn(M, N, generator=g) * 2 + 0.5).to(cuda)
    C1, C2 = C0.clone(), C0.clone()
    xb = torch.empty(M, N, dtype=dt, device=cuda)
    part = torch.empty(M, N // 128, 2, device=cuda)
    from depth_pro._lib import DP_TILE_8PH_320x256

    kw = dict(M=M, N=N, K=K, bias=bias, gamma=gamma, accumulate=True)
    ops.gemm(A, B, C1, tile=DP_TILE_8PH_320x256, **kw)
    ops.gemm(A, B, C2, ln_out=(xb, part), **kw)
    torch.cuda.synchronize()
    assert torch.equal(C1, C2)
    assert torch.equal(xb, C2.to(dt))
    np.testing.assert_allclose(part.cpu().double().numpy(), _chunk_stats(C2.cpu()).numpy(), rtol=5e-5, atol=2e-4)


@pytest.mark.parametrize("dt", DTYPES)
def test_layernorm_stats_split_residual(cuda, dt):
    """dp_layernorm_stats with xl (ABI 12): xb == x in 16 bits and xl == the int8 low part, exactly
    the host restatement ops.split_residual; xb + xl carries x to ~16 significant bits (the split
    residual's entry into ViT block 0)."""
    g = torch.Generator().manual_seed(12)
    rows = 1155
    x = torch.randn(rows, 1024, generator=g) * 3 + torch.randn(rows, 1, generator=g) * 2
    x[0, :8] = torch.tensor([0.0, 1e-30, -1e-7, 3e-5, 65000.0, -2.0, 0.5, 1.0 + 2 ** -9])   # edges
    xb = torch.empty(rows, 1024, dtype=dt, device=cuda)
    xl = torch.empty(rows, 1024, dtype=torch.int8, device=cuda)
    part = torch.empty(rows, 8, 2, device=cuda)
    ops.layernorm_stats(x.to(cuda), xb, part, rows, 1024, xl=xl)
    hi, q = ops.split_residual(x, dt)
    assert torch.equal(xb.cpu(), hi)
    assert torch.equal(xl.cpu(), q)
    err = (ops.merge_residual(xb.cpu(), xl.cpu()) - x).abs()
    bound = 4e-5 * x.abs() + (1e-36 if dt == torch.bfloat16 else 6e-8)
    assert torch.all(err <= bound), (err - bound).max().item()
    np.testing.assert_allclose(part.cpu().double().numpy(), _chunk_stats(x).numpy(), rtol=2e-5, atol=1e-4)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M,K,fp32_out,with_part,dbg", [(20195, 1024, False, True, 0), (577, 4096, True, True, 0),
                                                         (20195, 4096, True, False, 0), (20195, 1024, True, True, 1 << 27)])
def test_gemm_8ph320_split_residual_producer(cuda, dt, M, K, fp32_out, with_part, dbg):
    """Folded-LN producer on the split residual (ABI 12, dp_gemm ln_xl; the ViT proj / fc2): with the
    stream given as (hi, int8 lo), the new rows are bit-identical to the fp32 producer's on C =
    merge(hi, lo) (exact in fp32; same per-element operation order): C (when asked for) equal, hi ==
    C in 16 bits, lo == the host encoding of C (ops.split_residual), part equal; rows past M untouched
    (M = 20195: a 35-row last tile)."""
    g = torch.Generator().manual_seed(M + K + 7)
    N = 1024
    A = rnd(M, K, dt=dt, dev=cuda, gen=g)
    B = rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    bias = torch.randn(N, generator=g).to(cuda)
    gamma = (0.1 + 0.02 * torch.randn(N, generator=g)).to(cuda)
    x = torch.randn(M, N, generator=g) * 2 + 0.5
    hi0, lo0 = ops.split_residual(x, dt)
    C1 = ops.merge_residual(hi0, lo0).to(cuda)          # the fp32 producer's input: exactly hi + lo
    xb1 = torch.empty(M, N, dtype=dt, device=cuda)
    part1 = torch.empty(M, N // 128, 2, device=cuda)
    kw = dict(M=M, N=N, K=K, bias=bias, gamma=gamma, accumulate=True)
    ops.gemm(A, B, C1, ln_out=(xb1, part1), **kw)
    # split: hi / lo with a guard row past M on each (must stay untouched)
    hi = torch.empty(M + 1, N, dtype=dt, device=cuda)
    lo = torch.empty(M + 1, N, dtype=torch.int8, device=cuda)
    hi[:M], lo[:M] = hi0.to(cuda), lo0.to(cuda)
    hi[M], lo[M] = 7.0, -3
    part = torch.full((M, N // 128, 2), 123.0, device=cuda) if with_part else None
    C2 = torch.full((M, N), 5.0, device=cuda) if fp32_out else None
    tile, _ = ops.gemm(A, B, C2, plan_only=True, ln_out=(hi, part), ln_xl=lo, **kw)
    from depth_pro import _lib
    from depth_pro._lib import DP_TILE_8PH_320x256

    assert tile == DP_TILE_8PH_320x256
    _lib.load().dp_gemm_debug_flags(dbg)      # 1 << 27: the one-chunk-ahead epilogue (A/B variant)
    try:
        ops.gemm(A, B, C2, ln_out=(hi, part), ln_xl=lo, **kw)
        torch.cuda.synchronize()
    finally:
        _lib.load().dp_gemm_debug_flags(0)
    c1 = C1.cpu()
    assert torch.equal(hi[:M], xb1)
    assert torch.equal(lo[:M].cpu(), ops.split_residual(c1, dt)[1])
    assert torch.all(hi[M] == 7.0) and torch.all(lo[M] == -3)
    if fp32_out:
        assert torch.equal(C2, C1)
    if with_part:
        assert torch.equal(part, part1)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M", [20195, 577])
def test_split_producer_merged_row_stats(cuda, dt, M):
    """ABI 13: the split producer's last workgroup per row tile merges the tile's chunk statistics
    into (rstd, -rstd * mean) per row (dp_gemm ln_rs_out); a persistent-engine consumer reading them
    (ln_rs_in) is bit-identical to the one that merges `part` in its pre-pass launch.  Two producer
    launches in a row: the row-tile counters reset themselves (the second launch's statistics are
    right too); rows past M untouched."""
    g = torch.Generator().manual_seed(M + 31)
    N, K, N2 = 1024, 1024, 4096
    A = rnd(M, K, dt=dt, dev=cuda, gen=g)
    B = rnd(N, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    bias = torch.randn(N, generator=g).to(cuda)
    gamma = (0.1 + 0.02 * torch.randn(N, generator=g)).to(cuda)
    x = torch.randn(M, N, generator=g) * 2 + 0.5
    x[:, 3] += 30.0
    hi0, lo0 = ops.split_residual(x, dt)
    W2 = rnd(N2, K, dt=dt, dev=cuda, gen=g, scale=K ** -0.5)
    colsum = W2.float().sum(1).contiguous()
    b2 = torch.randn(N2, generator=g).to(cuda)
    ws = ops.gemm_workspace(cuda)
    from depth_pro._lib import DP_TILE_P8PH_256x256

    for rep in range(2):
        hi, lo = hi0.to(cuda), lo0.to(cuda)
        if rep:      # another stream state: the counters must have been reset by the first launch
            hi, lo = (hi.float() * 0.5).to(dt), lo // 2
        part = torch.empty(M, N // 128, 2, device=cuda)
        rs = torch.full((M + 1, 2), 9.0, device=cuda)
        kw = dict(M=M, N=N, K=K, bias=bias, gamma=gamma, accumulate=True, workspace=ws)
        ops.gemm(A, B, None, ln_out=(hi, part), ln_xl=lo, ln_rs_out=rs, **kw)
        C1 = torch.empty(M, N2, dtype=dt, device=cuda)
        C2 = torch.empty(M, N2, dtype=dt, device=cuda)
        kc = dict(M=M, N=N2, K=K, bias=b2, act=DP_ACT_GELU, tile=DP_TILE_P8PH_256x256, workspace=ws)
        ops.gemm(hi, W2, C1, ln_in=(part, colsum), **kc)          # pre-pass merge (ln_merge_kernel)
        ops.gemm(hi, W2, C2, ln_in=(None, colsum), ln_rs_in=rs, **kc)
        torch.cuda.synchronize()
        assert torch.equal(C1, C2), (C1.float() - C2.float()).abs().max().item()
        assert torch.all(rs[M] == 9.0)
        # and the statistics themselves vs fp64 from the producer's own rows (hi + lo)
        xr = ops.merge_residual(hi.cpu(), lo.cpu()).double()
        mean, var = xr.mean(1), xr.var(1, unbiased=False)
        r = rs[:M].cpu().double()
        assert torch.allclose(r[:, 0], (var + 1e-6).rsqrt(), rtol=2e-5)
        assert torch.allclose(r[:, 1], -(var + 1e-6).rsqrt() * mean, rtol=2e-4, atol=2e-5)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("act,col_scale,engine", [(0, True, "8ph320"), (DP_ACT_GELU, False, "8ph320"),
                                                  (DP_ACT_GELU, False, "p8ph")])
def test_gemm_8ph320_ln_consumer(cuda, dt, act, col_scale, engine):
    """Folded-LN consumer (the ViT qkv / fc1 with ln_in): GEMM over the un-normalised 16-bit rows
    with ops.fold_layernorm's weights == LN(x) W^T + b (then * the per-column scale, or GELU) in
    fp32; its error vs that reference is no larger than the unfolded LN -> 16-bit -> GEMM path's."""
    g = torch.Generator().manual_seed(5 + act)
    M, K, N = 20195, 1024, 3072 if col_scale else 4096
    x = torch.randn(M, K, generator=g) * 2 + torch.randn(M, 1, generator=g)
    x[:, 7] += 40.0                                          # an outlier channel, as DINOv2's
    w = torch.randn(N, K, generator=g) * K ** -0.5
    b = torch.randn(N, generator=g) * 0.02
    lw = 1.0 + 0.1 * torch.randn(K, generator=g)
    lb = 0.02 * torch.randn(K, generator=g)
    cs = ops.log2q_gamma(16, 64, "cpu") if col_scale else None
    xd = x.to(cuda)
    xb = torch.empty(M, K, dtype=dt, device=cuda)
    part = torch.empty(M, K // 128, 2, device=cuda)
    ops.layernorm_stats(xd, xb, part, M, K)
    wf, bf, sf = ops.fold_layernorm(w.to(cuda), b.to(cuda), lw.to(cuda), lb.to(cuda), dt,
                                    None if cs is None else cs.to(cuda))
    from depth_pro._lib import DP_TILE_8PH_320x256, DP_TILE_P8PH_256x256

    out = torch.empty(M, N, dtype=dt, device=cuda)
    ws = ops.gemm_workspace(cuda) if engine == "p8ph" else None
    kw = dict(M=M, N=N, K=K, bias=bf, act=act, ln_in=(part, sf), workspace=ws)
    tile, _ = ops.gemm(xb, wf, out, plan_only=True, **kw)
    assert tile == (DP_TILE_P8PH_256x256 if engine == "p8ph" else DP_TILE_8PH_320x256)
    ops.gemm(xb, wf, out, **kw)
    # unfolded: LN kernel -> 16-bit -> GEMM with bias (and gamma)
    h = torch.empty(M, K, dtype=dt, device=cuda)
    ops.layernorm(xd, lw.to(cuda), lb.to(cuda), h, M, K)
    out2 = torch.empty(M, N, dtype=dt, device=cuda)
    ops.gemm(h, w.to(dt).to(cuda), out2, M=M, N=N, K=K, bias=b.to(cuda), act=act,
             gamma=None if cs is None else cs.to(cuda))
    torch.cuda.synchronize()
    ref = F.linear(F.layer_norm(x, (K,), lw, lb, 1e-6), w, b)
    if act == DP_ACT_GELU:
        ref = F.gelu(ref)
    if cs is not None:
        ref = ref * cs
    e1 = ((out.float().cpu() - ref).abs().mean() / ref.abs().mean()).item()
    e2 = ((out2.float().cpu() - ref).abs().mean() / ref.abs().mean()).item()
    print(f"\nLN fold {dt} act={act} {engine}: folded rel-L1 {e1:.3e}, unfolded {e2:.3e}")
    assert e1 < (8e-3 if dt == torch.bfloat16 else 1.5e-3)
    assert e1 < 1.25 * e2 + 1e-5
