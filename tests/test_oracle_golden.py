"""Pin the CPU oracle (oracle/depth_pro_oracle.py) to the reference's outputs.

The fixtures in tests/golden were produced by running the reference's own
modules (tests/golden/make_golden.py) on the synthetic weights; here the
oracle must reproduce them.  Both sides are fp32 CPU, so the tolerances are
fp32 re-association level.
"""

import numpy as np
import pytest
import torch

from oracle import depth_pro_oracle as O


def _load(golden_dir, name):
    return np.load(f"{golden_dir}/{name}", allow_pickle=False)


def frame(seed, h=1536, w=1536):
    return np.random.default_rng(seed=seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def test_vit_block_matches_reference(golden_dir, synth_sd):
    g = _load(golden_dir, "golden_vit_block.npz")
    x = torch.randn(1, 577, 1024, generator=torch.Generator().manual_seed(int(g["seed"])))
    with torch.no_grad():
        y = O.vit_block(synth_sd, "encoder.patch_encoder.blocks.0.", x)
    np.testing.assert_allclose(y[0, :64].numpy(), g["out_rows"], rtol=1e-5, atol=1e-5)


def test_fusion_head_fov_tail_match_reference(golden_dir, synth_sd):
    g = _load(golden_dir, "golden_blocks.npz")
    gen = torch.Generator().manual_seed(int(g["seed"]))
    x0 = torch.randn(1, 256, 8, 8, generator=gen)
    x1 = torch.randn(1, 256, 8, 8, generator=gen)
    hin = torch.randn(1, 256, 16, 16, generator=gen)
    lo = torch.randn(1, 256, 48, 48, generator=gen)
    with torch.no_grad():
        fo = O.fusion_block(synth_sd, 1, x0, x1)
        ho = O.head_forward(synth_sd, hin)
        sd = synth_sd
        d = torch.relu(torch.nn.functional.conv2d(lo, sd["fov.downsample.0.weight"], sd["fov.downsample.0.bias"],
                                                  stride=2, padding=1))
        x = torch.relu(torch.nn.functional.conv2d(d, sd["fov.head.0.weight"], sd["fov.head.0.bias"], stride=2, padding=1))
        x = torch.relu(torch.nn.functional.conv2d(x, sd["fov.head.2.weight"], sd["fov.head.2.bias"], stride=2, padding=1))
        fh = torch.nn.functional.conv2d(x, sd["fov.head.4.weight"], sd["fov.head.4.bias"])
    np.testing.assert_allclose(fo.numpy(), g["fusion1"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(ho.numpy(), g["head"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(fh.numpy(), g["fov_tail"], rtol=1e-4, atol=1e-4)


def test_pyramid_split_merge_match_reference(golden_dir):
    g = _load(golden_dir, "golden_pyramid.npz")
    xs = torch.randn(1, 3, 1536, 1536, generator=torch.Generator().manual_seed(int(g["seed"])))
    x0, x1, x2 = O.pyramid(xs)
    np.testing.assert_allclose(x2[..., ::8, ::8].numpy(), g["x2"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(x1[..., ::16, ::16].numpy(), g["x1"], rtol=0, atol=1e-6)
    # exact 2x2 / {4d+1,4d+2} box-filter equivalence used by dp_patchify_pyramid
    box1 = 0.25 * (xs[..., 0::2, 0::2] + xs[..., 0::2, 1::2] + xs[..., 1::2, 0::2] + xs[..., 1::2, 1::2])
    box2 = 0.25 * (xs[..., 1::4, 1::4] + xs[..., 1::4, 2::4] + xs[..., 2::4, 1::4] + xs[..., 2::4, 2::4])
    assert (box1 - x1).abs().max() < 1e-6 and (box2 - x2).abs().max() < 1e-6
    s0, s1 = O.split(x0, 0.25), O.split(x1, 0.5)
    assert tuple(s0.shape) == tuple(g["s0_shape"]) and tuple(s1.shape) == tuple(g["s1_shape"])
    np.testing.assert_allclose([s0.double().sum().item(), (s0.double() ** 2).sum().item()], g["s0_sum"], rtol=1e-9)
    np.testing.assert_allclose([s1.double().sum().item(), (s1.double() ** 2).sum().item()], g["s1_sum"], rtol=1e-9)
    ids = torch.arange(35 * 24 * 24, dtype=torch.float64).reshape(35, 1, 24, 24)
    assert np.array_equal(O.merge(ids[:25], 1, 3)[0, 0].numpy().astype(np.int32), g["merge0"])
    assert np.array_equal(O.merge(ids[25:34], 1, 6)[0, 0].numpy().astype(np.int32), g["merge1"])


@pytest.mark.slow
def test_full_forward_frame0_matches_reference(golden_dir, synth_sd):
    g = _load(golden_dir, "golden_forward_frame0.npz")
    x = O.transform(frame(0)).unsqueeze(0)
    with torch.no_grad():
        canonical, fov = O.forward(synth_sd, x)
    np.testing.assert_allclose(fov.numpy().reshape(-1), g["fov_deg"], rtol=1e-5)
    np.testing.assert_allclose(canonical[0, 0, ::8, ::8].numpy(), g["canonical_sub8"], rtol=1e-4, atol=1e-5)


@pytest.mark.slow
def test_infer_frame1_matches_reference(golden_dir, synth_sd):
    g = _load(golden_dir, "golden_infer_frame1.npz")
    x = O.transform(frame(1, int(g["H"]), int(g["W"])))
    with torch.no_grad():
        p = O.infer(synth_sd, x, f_px=None)
    np.testing.assert_allclose(float(p["focallength_px"]), float(g["f_px"]), rtol=1e-5)
    np.testing.assert_allclose(p["depth"][::8, ::8].numpy(), g["depth_sub8"], rtol=1e-4, atol=1e-6)
