"""CPU check of the depth-head composition (engine.compose_head) against the reference layer order.

Reference (depth_pro.py:182-207): h1 = ConvTranspose2d(k2, s2)(h0); z = Conv2d(3x3, pad 1)(h1);
out = ReLU(Conv1x1(ReLU(z))).  The engine instead runs ONE 3x3 conv over h0 with 4 x 32 columns
(parity, channel) and fixes the zero-padded border taps with a per-tap bias correction; this test
evaluates exactly that arithmetic in fp32 (the dp_gemm DP_STORE_HEAD_PS epilogue, in torch).
"""

import torch
import torch.nn.functional as F

from depth_pro.engine import compose_head


def composed_head(h0, P, w4, b4):
    """What the HEAD_PS GEMM computes, evaluated with torch ops (fp32)."""
    n, ci, H, W = h0.shape
    wc = P["head.ps.w"].float().reshape(128, ci // 64, 3, 3, 64).permute(0, 1, 4, 2, 3).reshape(128, ci, 3, 3)
    v = F.conv2d(h0, wc, padding=1) + P["head.ps.b"].reshape(1, 128, 1, 1)  # [n, (q,o), H, W]
    corr = P["head.ps.corr"].reshape(3, 3, 32)
    out = torch.empty(n, 1, 2 * H, 2 * W)
    for q in range(4):
        dy, dx = q >> 1, q & 1
        z = v[:, q * 32:(q + 1) * 32].clone()
        for a in range(3):
            for c in range(3):
                m = torch.zeros(H, W, dtype=torch.bool)
                if a == 0 and dy == 0:
                    m[0, :] = True
                if a == 2 and dy == 1:
                    m[H - 1, :] = True
                if c == 0 and dx == 0:
                    m[:, 0] = True
                if c == 2 and dx == 1:
                    m[:, W - 1] = True
                z -= corr[a, c].reshape(1, 32, 1, 1) * m.reshape(1, 1, H, W)
        hs = (F.relu(z) * w4.reshape(1, 32, 1, 1)).sum(1, keepdim=True) + b4
        out[:, :, dy::2, dx::2] = F.relu(hs)
    return out


def test_compose_head_matches_reference_layer_order():
    g = torch.Generator().manual_seed(0)
    ci, H, W = 128, 7, 9
    h0 = torch.randn(1, ci, H, W, generator=g)
    wd = torch.randn(ci, ci, 2, 2, generator=g) * ci ** -0.5
    bd = torch.randn(ci, generator=g)
    w2 = torch.randn(32, ci, 3, 3, generator=g) * (9 * ci) ** -0.5
    b2 = torch.randn(32, generator=g)
    w4 = torch.randn(32, generator=g) * 32 ** -0.5
    b4 = 0.3
    ref = F.conv_transpose2d(h0, wd, bd, stride=2)
    ref = F.relu(F.conv2d(F.relu(F.conv2d(ref, w2, b2, padding=1)), w4.reshape(1, 32, 1, 1), torch.tensor([b4])))
    P = compose_head(wd, bd, w2, b2, torch.float32)
    got = composed_head(h0, P, w4, b4)
    assert got.shape == ref.shape
    err = (got - ref).abs().max().item()
    assert err < 1e-4 * (ref.abs().max().item() + 1), err


def test_compose_head0_matches_out_conv_then_head0():
    """engine.compose_head0: the decoder's 1x1 out_conv (decoder.py:184) followed by head.0's
    3x3 zero-padded conv (depth_pro.py:182-207) == ONE 3x3 conv with the composed weights and
    bias, minus the 1x1 bias's share of every tap that falls in the zero padding (what the
    dp_gemm DP_STORE_ROWS border correction subtracts), evaluated in fp32 with torch ops."""
    from depth_pro.engine import compose_head0

    g = torch.Generator().manual_seed(3)
    c, m, o, H, W = 64, 64, 128, 7, 9
    y = torch.randn(1, c, H, W, generator=g)
    wo = torch.randn(m, c, generator=g) * c ** -0.5
    bo = torch.randn(m, generator=g)
    w0 = torch.randn(o, m, 3, 3, generator=g) * (9 * m) ** -0.5
    b0 = torch.randn(o, generator=g)
    ref = F.conv2d(F.conv2d(y, wo[:, :, None, None], bo), w0, b0, padding=1)
    P = compose_head0(w0, b0, wo, bo, torch.float32)
    wc = P["head.0c.w"].float().reshape(o, c // 64, 3, 3, 64).permute(0, 1, 4, 2, 3).reshape(o, c, 3, 3)
    got = F.conv2d(y, wc, padding=1) + P["head.0c.b"].reshape(1, o, 1, 1)
    corr = P["head.0c.corr"].reshape(3, 3, o)
    for a in range(3):
        for b in range(3):
            msk = torch.zeros(H, W, dtype=torch.bool)
            if a == 0:
                msk[0, :] = True
            if a == 2:
                msk[H - 1, :] = True
            if b == 0:
                msk[:, 0] = True
            if b == 2:
                msk[:, W - 1] = True
            got = got - msk.float()[None, None] * corr[a, b].reshape(1, o, 1, 1)
    assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4), (got - ref).abs().max()
