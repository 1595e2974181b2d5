#!/usr/bin/env python3
"""CPU numerics study (no GPU): what folding each ViT LayerNorm into the GEMM that consumes it
does to the patch encoder's error against the fp32 reference.

    LN(x) W^T = rstd * (x (W o gamma)^T - mu * S) + (b + W beta),   S[c] = sum_k (W o gamma)[c, k]

lets the producer (proj / fc2 epilogue) write x in 16 bits and the consumer (qkv / fc1) take
x -- not LN(x) -- as its A operand, with the per-row (mu, rstd) applied in its epilogue.  The
catch is precision: the 16-bit rounding then hits x instead of the normalised LN(x).

Emulates the engine's mixed-mode ViT (16-bit operands, fp32 accumulate and residual stream,
16-bit P in attention) both ways on a few windows of synthetic frame 0 and reports each one's
rel-L1 vs the fp32 oracle after the final norm, for the benign and the stressed weight sets.
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ml-depth-pro-video_amd"))
from depth_pro.weights import stressed_state_dict, synthetic_state_dict  # noqa: E402
from oracle import depth_pro_oracle as O  # noqa: E402

EPS = 1e-6


def r16(t, dt):
    return t.to(dt).float()


def attn16(qkv, dt, H=16):
    B, N, C3 = qkv.shape
    C = C3 // 3
    q, k, v = qkv.reshape(B, N, 3, H, C // H).permute(2, 0, 3, 1, 4).unbind(0)
    s = (r16(q, dt) @ r16(k, dt).transpose(-1, -2)) * (C // H) ** -0.5
    m = s.amax(-1, keepdim=True)
    p = torch.exp(s - m)
    o = (r16(p, dt) @ r16(v, dt)) / p.sum(-1, keepdim=True)
    return o.transpose(1, 2).reshape(B, N, C)


def block(sd, p, x, dt, fold):
    C = x.shape[-1]

    def lin_ln(x, ln, w, b):
        g, be = sd[p + ln + ".weight"], sd[p + ln + ".bias"]
        if not fold:
            h = r16(F.layer_norm(x, (C,), g, be, EPS), dt)
            return h @ r16(w, dt).t() + b
        mu = x.mean(-1, keepdim=True)
        rstd = torch.rsqrt(x.var(-1, unbiased=False, keepdim=True) + EPS)
        wg = r16(w * g[None, :], dt)
        S = wg.sum(1)
        B = b + w @ be
        return rstd * (r16(x, dt) @ wg.t() - mu * S) + B

    qkv = lin_ln(x, "norm1", sd[p + "attn.qkv.weight"], sd[p + "attn.qkv.bias"])
    a = r16(attn16(r16(qkv, dt), dt), dt)
    x = x + sd[p + "ls1.gamma"] * (a @ r16(sd[p + "attn.proj.weight"], dt).t() + sd[p + "attn.proj.bias"])
    h = lin_ln(x, "norm2", sd[p + "mlp.fc1.weight"], sd[p + "mlp.fc1.bias"])
    m = r16(F.gelu(h), dt)
    return x + sd[p + "ls2.gamma"] * (m @ r16(sd[p + "mlp.fc2.weight"], dt).t() + sd[p + "mlp.fc2.bias"])


def run(sd, x0, dt, fold, pre="encoder.patch_encoder."):
    x = x0.clone()
    for i in range(24):
        x = block(sd, f"{pre}blocks.{i}.", x, dt, fold)
    return F.layer_norm(x, (1024,), sd[pre + "norm.weight"], sd[pre + "norm.bias"], EPS), x


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    img = np.random.default_rng(0).integers(0, 256, (1536, 1536, 3), dtype=np.uint8)
    xin = O.transform(img)[None]
    x0, x1, x2 = O.pyramid(xin)
    wins = torch.cat((O.split(x0, 0.25), O.split(x1, 0.5), x2), dim=0)   # encoder.py:245-263
    pick = wins[[0, 12, 34]]
    for name, sd in (("benign", synthetic_state_dict(0)), ("stressed", stressed_state_dict(0))):
        with torch.no_grad():
            x0 = O.vit_embed(sd, "encoder.patch_encoder.", pick)
            ref, xr = run(sd, x0, torch.float32, False)
            line = [name, f"residual |max| {xr.abs().max():.1f}, row |mean|/std max "
                          f"{(xr.mean(-1).abs() / xr.std(-1)).max():.3f}"]
            for dt in (torch.bfloat16, torch.float16):
                for fold in (False, True):
                    out, _ = run(sd, x0, dt, fold)
                    e = ((out - ref).abs().mean() / ref.abs().mean()).item()
                    line.append(f"{str(dt)[6:]} {'fold' if fold else 'LN  '} {e:.3e}")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
