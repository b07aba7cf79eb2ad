"""Functional fp32 restatement of the reference prompt-audio encoder — TEST INFRASTRUCTURE
(tests and the fixture generator use it; nothing in the product path imports oracle/).

Follows tts/core/codec/encoder.py:58-128 (forward, quantize, encode), encoder_modules.py
(ResidualUnit 20-42, EncoderBlock 45-68, SemanticEncoder 71-127, AcousticEncoder 130-187),
activations.py (SnakeBeta 45-86, Activation1d 89-110) and filters.py (UpSample1d 88-113,
DownSample1d / LowPassFilter1d 50-85, 116-135), with the quantizer of vector_quantize_pytorch
1.17.8 as oracle/shims restates it.  The w2v-bert-2.0 layer-16 features are an input here
(transformers' Wav2Vec2BertModel computes them in the fixture generator).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def wn_weight(w: dict, pre: str) -> torch.Tensor:
    """Legacy torch.nn.utils.weight_norm(dim=0): g * v / ||v|| over (in, k) per output."""
    v, g = w[pre + "weight_v"], w[pre + "weight_g"]
    return v * (g / v.flatten(1).norm(dim=1).view(-1, 1, 1))


def snake_aa(x: torch.Tensor, alpha: torch.Tensor, beta: torch.Tensor, filt: torch.Tensor) -> torch.Tensor:
    """Activation1d(SnakeBeta(alpha_logscale=True)) on [C, T]: 2x up (replicate pad 5,
    conv_transpose stride 2, x2, crop 15 / 15), SnakeBeta, 2x down (replicate pad 5 / 6,
    low-pass stride 2)."""
    C = x.shape[0]
    k = filt.numel()
    fw = filt.view(1, 1, k).expand(C, -1, -1)
    xp = F.pad(x[None], (5, 5), mode="replicate")
    u = 2 * F.conv_transpose1d(xp, fw, stride=2, groups=C)
    u = u[..., 15:-15]
    a, b = alpha.exp().view(1, -1, 1), beta.exp().view(1, -1, 1)
    u = u + (1.0 / (b + 1e-9)) * torch.pow(torch.sin(u * a), 2)
    up = F.pad(u, (5, 6), mode="replicate")
    return F.conv1d(up, fw, stride=2, groups=C)[0]


def acoustic(w: dict, wav: torch.Tensor, filt: torch.Tensor, up_ratios=(2, 2, 4, 4, 5), dilations=(1, 3, 9)):
    """AcousticEncoder.forward on one waveform [N] -> [T, 1024]."""
    a = "acoustic_encoder."
    x = F.conv1d(wav.view(1, 1, -1), wn_weight(w, a + "conv_blocks.0."), w[a + "conv_blocks.0.bias"], padding=3)[0]
    for i, s in enumerate(up_ratios, start=1):
        for r, d in enumerate(dilations):
            p = f"{a}conv_blocks.{i}.block.{r}.block."
            y = snake_aa(x, w[p + "0.act.alpha"], w[p + "0.act.beta"], filt)
            y = F.conv1d(y[None], wn_weight(w, p + "1."), w[p + "1.bias"], dilation=d, padding=3 * d)[0]
            y = snake_aa(y, w[p + "2.act.alpha"], w[p + "2.act.beta"], filt)
            y = F.conv1d(y[None], wn_weight(w, p + "3."), w[p + "3.bias"])[0]
            x = x + y
        p = f"{a}conv_blocks.{i}.block."
        x = snake_aa(x, w[p + "3.act.alpha"], w[p + "3.act.beta"], filt)
        x = F.conv1d(x[None], wn_weight(w, p + "4."), w[p + "4.bias"], stride=s, padding=s // 2 + s % 2)[0]
    p = a + "conv_final_block."
    x = snake_aa(x, w[p + "0.act.alpha"], w[p + "0.act.beta"], filt)
    x = F.conv1d(x[None], wn_weight(w, p + "1."), w[p + "1.bias"], padding=1)[0]
    return x.t()


def semantic(w: dict, feats: torch.Tensor) -> torch.Tensor:
    """SemanticEncoder.forward on [T, 1024] -> [T, 1024].  The residual branch starts with
    ReLU(inplace=True) applied to the initial conv's output, so the skip adds relu(x0)."""
    p = "semantic_encoder."
    x0 = F.conv1d(feats.t()[None], w[p + "initial_conv.weight"], padding=1)
    x0 = torch.relu(x0)
    y = F.conv1d(x0, w[p + "residual_blocks.1.weight"], w[p + "residual_blocks.1.bias"], padding=1)
    y = F.conv1d(torch.relu(y), w[p + "residual_blocks.3.weight"], w[p + "residual_blocks.3.bias"], padding=1)
    x = y + x0
    return F.conv1d(x, w[p + "final_conv.weight"], padding=1)[0].t()


def fsq_bound(z: torch.Tensor, levels, eps: float = 1e-3) -> torch.Tensor:
    lv = torch.tensor(levels, dtype=torch.float32)
    half_l = (lv - 1) * (1 + eps) / 2
    offset = torch.where(torch.tensor(levels) % 2 == 0, 0.5, 0.0)
    shift = (offset / half_l).atanh()
    return (z + shift).tanh() * half_l - offset


def encode(w: dict, wav: torch.Tensor, w2v16: torch.Tensor, filt: torch.Tensor, levels=(4,) * 8):
    """Encoder.encode: pad to a whole hop (+320 when already whole, as the reference does),
    acoustic | semantic -> fusion -> project_in -> bound -> FSQ (bound, round) -> indices.
    Returns (codes [T] int, the pre-round values [T, 8])."""
    n = wav.numel()
    audio = F.pad(wav.view(1, -1), (0, 320 - n % 320))[0]
    ac = acoustic(w, audio, filt)
    se = semantic(w, w2v16)
    h = torch.cat([se, ac], dim=1) @ w["fusion_layer.weight"].t() + w["fusion_layer.bias"]
    z = h @ w["quantizer.project_in.weight"].t() + w["quantizer.project_in.bias"]
    pre = fsq_bound(fsq_bound(z, levels), levels)
    q = pre.round()
    half = torch.tensor([lv // 2 for lv in levels], dtype=torch.float32)
    basis = torch.cumprod(torch.tensor([1] + list(levels[:-1])), 0).float()
    idx = (((q / half) * half + half) * basis).sum(-1).to(torch.int32)
    return idx, pre
