#!/usr/bin/env python3
"""CPU numerics study (no GPU) for the split residual stream (dp_gemm ln_xl, ABI 12): the patch
encoder's residual x held as hi + lo (two 16-bit arrays, hi = r16(x), lo = r16(x - hi)) instead of
fp32, emulated on the folded-LN ViT of tools/ln_fold_emul.py (bf16 operands) over three windows of
synthetic frame 0; rel-L1 after the final norm vs the fp32 reference, for the fp32 stream, the
split one and a plain bf16 stream (benign and stressed weights).  Measured:
    benign   | f32 2.3788e-03 | hilo 2.3789e-03 | bf16 1.0589e-02
    stressed | f32 2.2778e-03 | hilo 2.2718e-03 | bf16 7.1611e-03
"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ml-depth-pro-video_amd"))
import ln_fold_emul as L
import torch, numpy as np
import torch.nn.functional as F
from depth_pro.weights import stressed_state_dict, synthetic_state_dict
from oracle import depth_pro_oracle as O

def hilo(x, mode):
    if mode == "f32": return x
    hi = x.to(torch.bfloat16).float()
    if mode == "bf16": return hi
    lo = (x - hi).to(torch.bfloat16).float()
    return hi + lo

def block(sd, p, x, dt, mode):
    C = x.shape[-1]
    def lin_ln(x, ln, w, b):
        g, be = sd[p + ln + ".weight"], sd[p + ln + ".bias"]
        mu = x.mean(-1, keepdim=True)
        rstd = torch.rsqrt(x.var(-1, unbiased=False, keepdim=True) + L.EPS)
        wg = L.r16(w * g[None, :], dt)
        S = wg.sum(1)
        B = b + w @ be
        return rstd * (L.r16(x, dt) @ wg.t() - mu * S) + B
    qkv = lin_ln(x, "norm1", sd[p + "attn.qkv.weight"], sd[p + "attn.qkv.bias"])
    a = L.r16(L.attn16(L.r16(qkv, dt), dt), dt)
    x = hilo(x + sd[p + "ls1.gamma"] * (a @ L.r16(sd[p + "attn.proj.weight"], dt).t() + sd[p + "attn.proj.bias"]), mode)
    h = lin_ln(x, "norm2", sd[p + "mlp.fc1.weight"], sd[p + "mlp.fc1.bias"])
    m = L.r16(F.gelu(h), dt)
    return hilo(x + sd[p + "ls2.gamma"] * (m @ L.r16(sd[p + "mlp.fc2.weight"], dt).t() + sd[p + "mlp.fc2.bias"]), mode)

def run(sd, x0, dt, mode, pre="encoder.patch_encoder."):
    x = hilo(x0.clone(), mode)
    for i in range(24):
        x = block(sd, f"{pre}blocks.{i}.", x, dt, mode)
    return F.layer_norm(x, (1024,), sd[pre + "norm.weight"], sd[pre + "norm.bias"], L.EPS)

def main():
    torch.set_num_threads(8)
    img = np.random.default_rng(0).integers(0, 256, (1536, 1536, 3), dtype=np.uint8)
    xin = O.transform(img)[None]
    x0, x1, x2 = O.pyramid(xin)
    wins = torch.cat((O.split(x0, 0.25), O.split(x1, 0.5), x2), dim=0)
    pick = wins[[0, 12, 34]]
    for name, sd in (("benign", synthetic_state_dict(0)), ("stressed", stressed_state_dict(0))):
        with torch.no_grad():
            e0 = O.vit_embed(sd, "encoder.patch_encoder.", pick)
            ref, _ = L.run(sd, e0, torch.float32, False)
            line = [name]
            for mode in ("f32", "hilo", "bf16"):
                out = run(sd, e0, torch.bfloat16, mode)
                e = ((out - ref).abs().mean() / ref.abs().mean()).item()
                line.append(f"{mode} {e:.4e}")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
