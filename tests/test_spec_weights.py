"""Host-side logic: parameter inventory, synthetic weights, weight packing algebra."""

import torch
import torch.nn.functional as F

from depth_pro.spec import num_params, param_spec
from depth_pro.weights import synthetic_tensor


def test_param_inventory_matches_reference_counts():
    s = param_spec()
    assert len(s) == 1119                # 1,119 state-dict keys
    assert num_params(s) == 951_991_330  # 951,991,330 params
    assert len(param_spec(use_fov_head=False)) == 1119 - 342 - 2 - 8


def test_synthetic_weights_are_deterministic_and_key_dependent():
    a = synthetic_tensor("decoder.convs.1.weight", (256, 256, 3, 3), 0)
    b = synthetic_tensor("decoder.convs.1.weight", (256, 256, 3, 3), 0)
    c = synthetic_tensor("decoder.convs.1.weight", (256, 256, 3, 3), 1)
    assert torch.equal(a, b) and not torch.equal(a, c)
    assert abs(a.std().item() - (1 / 2304) ** 0.5) < 2e-3
    assert synthetic_tensor("fov.head.4.bias", (1,)).item() == 60.0


def test_composed_deconv_out_conv_equals_sequential():
    """engine.pack_weights folds fusion deconv + 1x1 out_conv into one deconv (decoder.py:180-184)."""
    from depth_pro.engine import _deconv_w

    g = torch.Generator().manual_seed(0)
    x = torch.randn(1, 256, 6, 6, generator=g, dtype=torch.float64)
    wd = torch.randn(256, 256, 2, 2, generator=g, dtype=torch.float64) / 16
    wo = torch.randn(256, 256, 1, 1, generator=g, dtype=torch.float64) / 16
    bo = torch.randn(256, generator=g, dtype=torch.float64)
    ref = F.conv2d(F.conv_transpose2d(x, wd, stride=2), wo, bo)
    wc = torch.einsum("icyx,oc->ioyx", wd, wo[:, :, 0, 0])
    got = F.conv_transpose2d(x, wc, bo, stride=2)
    assert (got - ref).abs().max() < 1e-10
    # packed layout: B[(dy,dx,co)][ci] -> GEMM over NHWC rows, pixel-shuffle store
    B = _deconv_w(wc, torch.float64)
    xr = x[0].permute(1, 2, 0).reshape(36, 256)
    y = (xr @ B.t()).reshape(6, 6, 2, 2, 256)  # (y, x, dy, dx, co)
    y = y.permute(4, 0, 2, 1, 3).reshape(256, 12, 12) + bo[:, None, None]
    assert (y - got[0]).abs().max() < 1e-10


def test_conv_pack_layout_is_implicit_gemm_order():
    from depth_pro.engine import _conv_w

    g = torch.Generator().manual_seed(1)
    x = torch.randn(1, 64, 5, 5, generator=g, dtype=torch.float64)
    w = torch.randn(32, 64, 3, 3, generator=g, dtype=torch.float64)
    ref = F.conv2d(x, w, padding=1)
    x = torch.cat([x, torch.randn(1, 64, 5, 5, generator=g, dtype=torch.float64)], 1)   # 128 channels
    w = torch.randn(32, 128, 3, 3, generator=g, dtype=torch.float64)
    ref = F.conv2d(x, w, padding=1)
    B = _conv_w(w, torch.float64)  # [co][(ci/64, ky, kx, ci%64)]
    xp = F.pad(x, (1, 1, 1, 1))[0].permute(1, 2, 0)  # (7,7,128) NHWC padded
    cols = torch.stack([xp[y:y + 3, xx:xx + 3, :].reshape(3, 3, 2, 64).permute(2, 0, 1, 3).reshape(-1)
                        for y in range(5) for xx in range(5)])
    got = (cols @ B.t()).t().reshape(32, 5, 5)
    assert (got - ref[0]).abs().max() < 1e-10
