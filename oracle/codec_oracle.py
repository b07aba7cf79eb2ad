"""CPU oracle of the codec decoder — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

Functional fp32 torch restatement of the reference ``Decoder.forward``
(tts/core/codec/decoder.py:69-89) from a state dict with the reference's key names:

* ResidualFSQ.get_output_from_indices (vector_quantize_pytorch 1.17.8, third-party;
  built at decoder_modules.py:418-420): index -> 8 base-4 digits -> (d-2)/2 -> project_out
* fc_post_a                              decoder.py:63,79
* VocosBackbone.forward                  decoder_modules.py:390-400
  - embed Conv1d(k7, p3)                 :340
  - ResnetBlock                          :162-223 (GroupNorm(32, eps 1e-6) -> swish -> conv3 x2, + x)
  - TransformerBlock x depth             :293-314 (RMSNorm 226-236, Attention 254-290 with
    torchtune RotaryPositionalEmbeddings 0.6.1 applied to [b,h,t,d] => position = head index,
    interleaved pairs; non-causal SDPA; MLP 239-251 with SiLU)
  - final LayerNorm(eps 1e-6)            :373,399
* UpSamplerBlock.forward                 upsampler.py:62-69 (weight-normed ConvTranspose1d,
  ResnetBlock, out_proj + swish)
* ISTFTHead.forward + ISTFT('same')      decoder_modules.py:118-148, 64-93

Pinning: oracle/make_golden.py runs the reference Decoder itself (with restated third-party
pieces, oracle/shims) and checks this restatement against it; the waveforms it produced are
committed under tests/golden/.
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def swish(x):
    return x * torch.sigmoid(x)


def fsq_codes(idx: torch.Tensor) -> torch.Tensor:
    """[T] int -> [T, 8] float in {-1, -0.5, 0, 0.5}."""
    digits = torch.stack([(idx // (4 ** j)) % 4 for j in range(8)], dim=-1)
    return (digits.float() - 2.0) / 2.0


def resnet(x: torch.Tensor, w: dict, pre: str) -> torch.Tensor:
    """x: [1, C, T] channels-first like the reference."""
    h = F.group_norm(x, 32, w[pre + "norm1.weight"], w[pre + "norm1.bias"], eps=1e-6)
    h = swish(h)
    h = F.conv1d(h, w[pre + "conv1.weight"], w[pre + "conv1.bias"], padding=1)
    h = F.group_norm(h, 32, w[pre + "norm2.weight"], w[pre + "norm2.bias"], eps=1e-6)
    h = swish(h)
    h = F.conv1d(h, w[pre + "conv2.weight"], w[pre + "conv2.bias"], padding=1)
    return x + h


def rope_by_head(x: torch.Tensor) -> torch.Tensor:
    """torchtune RoPE (dim 64, base 10000) on x [b, h, t, d] treating h as the sequence."""
    b, h, t, d = x.shape
    theta = 1.0 / (10000 ** (torch.arange(0, d, 2)[: d // 2].float() / d))
    seq = torch.arange(h, dtype=theta.dtype)
    ang = torch.einsum("i,j->ij", seq, theta).float()          # [h, d/2]
    cos, sin = torch.cos(ang), torch.sin(ang)
    xs = x.float().reshape(b, h, t, d // 2, 2)
    c = cos.view(1, h, 1, d // 2)
    s = sin.view(1, h, 1, d // 2)
    out = torch.stack([xs[..., 0] * c - xs[..., 1] * s, xs[..., 1] * c + xs[..., 0] * s], -1)
    return out.flatten(3).type_as(x)


def rmsnorm(x, wt, eps=1e-6):
    return x * torch.rsqrt(torch.mean(x ** 2, dim=-1, keepdim=True) + eps) * wt


def transformer(x: torch.Tensor, w: dict, pre: str, heads: int = 16) -> torch.Tensor:
    """x: [1, T, D]."""
    b, t, dm = x.shape
    h = rmsnorm(x, w[pre + "att_norm.weight"])
    qkv = h @ w[pre + "att.c_attn.weight"].t()
    q, k, v = qkv.view(b, t, 3, heads, dm // heads).permute(2, 0, 3, 1, 4)
    q, k = rope_by_head(q), rope_by_head(k)
    y = F.scaled_dot_product_attention(q, k, v, attn_mask=None, dropout_p=0.0, is_causal=False)
    y = y.transpose(1, 2).reshape(b, t, dm)
    x = x + y @ w[pre + "att.c_proj.weight"].t()
    h = rmsnorm(x, w[pre + "ffn_norm.weight"])
    h = F.silu(h @ w[pre + "mlp.fc1.weight"].t()) @ w[pre + "mlp.fc2.weight"].t()
    return x + h


def weight_norm_fold(g: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """legacy torch.nn.utils.weight_norm(dim=0): w = g * v / ||v|| (norm over dims 1..)."""
    return v * (g / torch.linalg.vector_norm(v, dim=tuple(range(1, v.dim())), keepdim=True))


def istft_same(spec: torch.Tensor, n_fft: int, hop: int, window: torch.Tensor) -> torch.Tensor:
    """spec: [B, N//2+1, F] complex -> [B, F*hop]."""
    pad = (n_fft - hop) // 2
    B, N, T = spec.shape
    ifft = torch.fft.irfft(spec, n_fft, dim=1, norm="backward") * window[None, :, None]
    out_size = (T - 1) * hop + n_fft
    y = F.fold(ifft, output_size=(1, out_size), kernel_size=(1, n_fft), stride=(1, hop))[:, 0, 0, pad:-pad]
    wsq = window.square().expand(1, T, -1).transpose(1, 2)
    env = F.fold(wsq, output_size=(1, out_size), kernel_size=(1, n_fft), stride=(1, hop)).squeeze()[pad:-pad]
    assert (env > 1e-11).all()
    return y / env


@torch.no_grad()
def decode(w: dict, codes: torch.Tensor, hop_length: int, upsample_factors=(), kernel_sizes=(),
           depth: int = 12) -> torch.Tensor:
    """codes [T] int -> wav [1, T*hop*prod(ups)] float32 (reference AudioDecoder.decode)."""
    w = {k: v.float() for k, v in w.items()}
    z = fsq_codes(codes.long())[None]                                              # [1, T, 8]
    emb = z @ w["decoder.quantizer.project_out.weight"].t() + w["decoder.quantizer.project_out.bias"]
    x = emb @ w["fc_post_a.weight"].t() + w["fc_post_a.bias"]                      # [1, T, 1024]
    x = x.transpose(1, 2)
    x = F.conv1d(x, w["decoder.backbone.embed.weight"], w["decoder.backbone.embed.bias"], padding=3)
    for i in range(2):
        x = resnet(x, w, f"decoder.backbone.prior_net.{i}.")
    x = x.transpose(1, 2)
    for i in range(depth):
        x = transformer(x, w, f"decoder.backbone.transformers.{i}.")
    x = x.transpose(1, 2)
    for i in range(2):
        x = resnet(x, w, f"decoder.backbone.post_net.{i}.")
    x = x.transpose(1, 2)
    x = F.layer_norm(x, (x.shape[-1],), w["decoder.backbone.final_layer_norm.weight"],
                     w["decoder.backbone.final_layer_norm.bias"], eps=1e-6)
    if upsample_factors:
        h = x.transpose(1, 2)
        for i, (u, k) in enumerate(zip(upsample_factors, kernel_sizes)):
            p = f"upsampler.upsample_layers.{i}."
            wt = w[p + "weight"] if (p + "weight") in w else weight_norm_fold(w[p + "weight_g"], w[p + "weight_v"])
            h = F.conv_transpose1d(h, wt, w[p + "bias"], stride=u, padding=(k - u) // 2)
            h = resnet(h, w, f"upsampler.resnet_blocks.{i}.")
        x = swish(h.transpose(1, 2) @ w["upsampler.out_proj.weight"].t() + w["upsampler.out_proj.bias"])
    n_fft = 4 * hop_length
    xp = (x @ w["decoder.head.out.weight"].t() + w["decoder.head.out.bias"]).transpose(1, 2)
    mag, p = xp.chunk(2, dim=1)
    mag = torch.clip(torch.exp(mag), max=1e2)
    spec = mag * (torch.cos(p) + 1j * torch.sin(p))
    window = w.get("decoder.head.istft.window", torch.hann_window(n_fft))
    return istft_same(spec, n_fft, hop_length, window)
