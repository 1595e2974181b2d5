"""End-to-end parity of the MI355X engine against the reference's golden outputs.

Fixtures: tests/golden/golden_forward_frame0.npz / golden_infer_frame1.npz,
produced by the reference modules on the synthetic weights (seed 0).
Metric: relative L1 = mean|x - x_ref| / mean|x_ref| over the stored grid
(canonical inverse depth sub-sampled 8x; depth sub-sampled 8x).
"""

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# BASELINE.json target: depth L1 vs reference < 1e-3 (relative).  bf16 carries
# 8 mantissa bits through 3 x 24 ViT-L blocks; the measured values are printed
# and bounded here (see DESIGN.md "Parity").
# Measured (round 1): bf16 canonical 2.0e-3 / depth 1.4e-3, f16 2.6e-4 / 1.7e-4 -- bounds at ~2x.
# The f16 mode meets BASELINE's < 1e-3 depth L1; bf16 does not (8 mantissa bits).
TOL = {torch.bfloat16: dict(canon=4e-3, depth=3e-3, fov=1e-3, fpx=2e-3),
       torch.float16: dict(canon=6e-4, depth=5e-4, fov=3e-4, fpx=5e-4)}


def frame(seed, h=1536, w=1536):
    return np.random.default_rng(seed=seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def rel_l1(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).mean() / np.abs(b).mean())


@pytest.fixture(scope="module", params=[torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def model(request, cuda):
    import depth_pro
    from depth_pro.depth_pro import DepthProConfig

    cfg = DepthProConfig(patch_encoder_preset="dinov2l16_384", image_encoder_preset="dinov2l16_384",
                         checkpoint_uri=None, decoder_features=256, use_fov_head=True,
                         fov_encoder_preset="dinov2l16_384")
    os.environ["DEPTH_PRO_COMPUTE_DTYPE"] = "bf16" if request.param == torch.bfloat16 else "fp16"
    try:
        m, t = depth_pro.create_model_and_transforms(cfg, device=cuda, precision=torch.float32)
    finally:
        os.environ.pop("DEPTH_PRO_COMPUTE_DTYPE", None)
    m.tol = TOL[request.param]
    m.tag = str(request.param)
    yield m, t
    del m
    torch.cuda.empty_cache()


def test_forward_frame0_vs_reference(model, golden_dir):
    m, transform = model
    g = np.load(f"{golden_dir}/golden_forward_frame0.npz")
    x = transform(frame(0)).unsqueeze(0)
    with torch.no_grad():
        canonical, fov = m.forward(x)
    c = canonical[0, 0, ::8, ::8].float().cpu().numpy()
    e_c = rel_l1(c, g["canonical_sub8"])
    e_f = abs(fov.item() - float(g["fov_deg"][0])) / abs(float(g["fov_deg"][0]))
    print(f"\n[{m.tag}] canonical rel-L1 {e_c:.3e}  max|d| {np.abs(c - g['canonical_sub8']).max():.3e}  "
          f"fov {fov.item():.4f} vs {float(g['fov_deg'][0]):.4f} (rel {e_f:.2e})")
    assert np.isfinite(c).all()
    assert e_c < m.tol["canon"]
    assert e_f < m.tol["fov"]


def test_infer_frame1_resize_path_vs_reference(model, golden_dir):
    m, transform = model
    g = np.load(f"{golden_dir}/golden_infer_frame1.npz")
    x = transform(frame(1, int(g["H"]), int(g["W"])))
    p = m.infer(x, f_px=None)
    d = p["depth"][::8, ::8].cpu().numpy()
    assert p["depth"].shape == (int(g["H"]), int(g["W"]))
    e_d = rel_l1(d, g["depth_sub8"])
    e_f = abs(float(p["focallength_px"]) - float(g["f_px"])) / float(g["f_px"])
    print(f"\n[{m.tag}] infer depth rel-L1 {e_d:.3e}  f_px {float(p['focallength_px']):.3f} vs {float(g['f_px']):.3f}")
    assert e_d < m.tol["depth"] and e_f < m.tol["fpx"]
    p2 = m.infer(x, f_px=np.float64(1400.0))
    d2 = p2["depth"][::8, ::8].cpu().numpy()
    e_d2 = rel_l1(d2, g["depth_given_sub8"])
    print(f"[{m.tag}] infer(f_px=1400) depth rel-L1 {e_d2:.3e}")
    assert e_d2 < m.tol["depth"]
    assert float(p2["focallength_px"]) == 1400.0
    with pytest.raises(AttributeError):  # reference behaviour: float has no .squeeze()
        m.infer(x, f_px=1400.0)


def test_graph_replay_matches_eager(model):
    m, transform = model
    x = transform(frame(2))
    p_eager = m.infer(x)["depth"].clone()
    m.use_hip_graph(True)
    try:
        p_graph = m.infer(x)["depth"]
        p_graph2 = m.infer(x)["depth"]
    finally:
        m.use_hip_graph(False)
    assert torch.equal(p_eager, p_graph) and torch.equal(p_graph, p_graph2)
