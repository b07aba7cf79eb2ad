"""Deterministic synthetic weights and inputs (no checkpoints are reachable offline).

``synth_values`` is bit-identical to the device generator ``tts_synth_fill``
(csrc/lm_ops.hip): value_i = (2*u_i - 1) * scale with u_i the top 24 bits of
splitmix64(seed + (i+1)*0x9E3779B97F4A7C15) / 2^24.  The GPU box can therefore rebuild,
on the device and in milliseconds, exactly the weights the golden fixtures were produced
with on the CPU.

Weight names are the reference state-dict keys: HF Llama keys for the SpeechLM and the
``Decoder`` keys of tts/core/codec/decoder.py for the codec.
"""

from __future__ import annotations

import dataclasses
import math
import zlib

import numpy as np
import torch

from . import configs

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def tensor_seed(base_seed: int, name: str) -> int:
    return (base_seed * 0x100000001B3 + zlib.crc32(name.encode())) & 0xFFFFFFFFFFFFFFFF


def synth_values(seed: int, n: int, scale: float, chunk: int = 1 << 24) -> np.ndarray:
    """float32 array of n synthetic values (see module docstring)."""
    out = np.empty(n, dtype=np.float32)
    s = np.uint64(seed)
    sc = np.float32(scale)
    with np.errstate(over="ignore"):
        for a in range(0, n, chunk):
            b = min(n, a + chunk)
            z = s + (np.arange(a + 1, b + 1, dtype=np.uint64) * _GOLD)
            z = (z ^ (z >> np.uint64(30))) * _M1
            z = (z ^ (z >> np.uint64(27))) * _M2
            z = z ^ (z >> np.uint64(31))
            u = (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
            out[a:b] = (u * np.float32(2.0) - np.float32(1.0)) * sc
    return out


# ------------------------------------------------------------------ SpeechLM weights ---

def lm_tensor_specs(arch: configs.LmArch) -> list[tuple[str, tuple[int, ...], float, float]]:
    """(name, shape, scale, offset) for every LlamaForCausalLM tensor.  value = offset + synth.

    Linear weights: uniform with std 0.02 (scale 0.02*sqrt(3)); norm weights 1 +- 0.2 so the
    bf16 `weight * x` step is exercised; the (tied) embedding uses std 0.08 which widens the
    greedy argmax margins ("lm_head scaled x4")."""
    H, KVH, D, HID, FF = arch.num_heads, arch.num_kv_heads, arch.head_dim, arch.hidden_size, arch.intermediate_size
    lin = 0.02 * math.sqrt(3.0)
    specs = [("model.embed_tokens.weight", (arch.vocab_size, HID), 0.08 * math.sqrt(3.0), 0.0)]
    for i in range(arch.num_layers):
        p = f"model.layers.{i}."
        specs += [
            (p + "input_layernorm.weight", (HID,), 0.2, 1.0),
            (p + "self_attn.q_proj.weight", (H * D, HID), lin, 0.0),
            (p + "self_attn.k_proj.weight", (KVH * D, HID), lin, 0.0),
            (p + "self_attn.v_proj.weight", (KVH * D, HID), lin, 0.0),
            (p + "self_attn.o_proj.weight", (HID, H * D), lin, 0.0),
            (p + "post_attention_layernorm.weight", (HID,), 0.2, 1.0),
            (p + "mlp.gate_proj.weight", (FF, HID), lin, 0.0),
            (p + "mlp.up_proj.weight", (FF, HID), lin, 0.0),
            (p + "mlp.down_proj.weight", (HID, FF), lin, 0.0),
        ]
    specs.append(("model.norm.weight", (HID,), 0.2, 1.0))
    if not arch.tie_word_embeddings:
        specs.append(("lm_head.weight", (arch.vocab_size, HID), 0.08 * math.sqrt(3.0), 0.0))
    return specs


def lm_weights_cpu(arch: configs.LmArch, seed: int) -> dict[str, torch.Tensor]:
    """bf16 CPU tensors (numpy generator)."""
    out = {}
    for name, shape, scale, off in lm_tensor_specs(arch):
        n = int(np.prod(shape))
        v = synth_values(tensor_seed(seed, name), n, scale)
        t = torch.from_numpy(v).reshape(shape)
        if off:
            t = t + off  # fp32 add, then one RNE rounding to bf16 (same on device)
        out[name] = t.to(torch.bfloat16)
    return out


def lm_weights_device(arch: configs.LmArch, seed: int, device) -> dict[str, torch.Tensor]:
    """Same values generated on the GPU by tts_synth_fill (bit-identical to lm_weights_cpu)."""
    from . import _lib

    lib = _lib.load_library()
    out = {}
    for name, shape, scale, off in lm_tensor_specs(arch):
        n = int(np.prod(shape))
        if off:
            t = torch.empty(shape, dtype=torch.float32, device=device)
            _lib.check(lib.tts_synth_fill(t.data_ptr(), _lib.DT_F32, n, tensor_seed(seed, name), scale,
                                          _lib.stream_ptr()))
            out[name] = (t + off).to(torch.bfloat16)
        else:
            t = torch.empty(shape, dtype=torch.bfloat16, device=device)
            _lib.check(lib.tts_synth_fill(t.data_ptr(), _lib.DT_BF16, n, tensor_seed(seed, name), scale,
                                          _lib.stream_ptr()))
            out[name] = t
    torch.cuda.synchronize()
    return out


# ------------------------------------------------- decisive greedy-parity model ("chain") ---
#
# With random weights the bf16 dataflow is chaotic at the ulp level: two valid
# implementations (transformers on CPU, the engine) differ by ~0.5 % of the hidden state per
# layer, so over hundreds of free-running steps some top-1/top-2 margin always falls inside
# that noise and "bit-exact ids" cannot be shown on random weights alone.  The chain model
# keeps every random tensor (the same numerics everywhere) and overwrites a few rows with
# exact values so that each step's argmax is decided by a margin far above the noise AND by
# the greedy head's semantics (repetition penalty over prompt + generated ids, the
# min-new-tokens EOS mask, EOS stop):
#
# * chain tokens c_0..c_{U-1} (distinct <|s_N|> ids) and EOS get embedding rows s*H_r, r a
#   Sylvester-Hadamard row (exactly orthogonal, exact in bf16), and so do their lm_head rows
#   (the same tensor when tied, written separately when not);
# * MLP unit j of layer 0 detects c_j (gate = up = 2^g H_{r(j)}) and writes
#   2^q (H_{r(j+1)} + w_seen H_{r(j-lag)}) into the residual: the already-generated
#   c_{j-lag} has the larger raw logit (x w_seen = 1.046875) but, penalised by
#   repetition_penalty = 1.1, loses to the fresh c_{j+1} (and wins without a penalty);
# * units j = eos_phase (mod eos_period) write 2^q (H_{r(j+1)} + 2 H_eos) instead: EOS wins
#   unless min_new_tokens masks it.
#
# Every value is a signed power of two or a sum of two such values, so the construction is
# bit-identical with numpy on the CPU and torch on the device.

@dataclasses.dataclass(frozen=True)
class ChainSpec:
    seed: int = 0xC4A1
    units: int = 2040            # chain tokens (Hadamard rows 1..units), EOS uses row `eos_row`
    eos_row: int = 2047
    emb_exp: int = -3            # embedding rows s*H, s = 2^emb_exp
    gate_exp: int = -7           # gate/up rows 2^gate_exp * H
    down_exp: int = -1           # down columns 2^down_exp * (H_next + w H_seen)
    lag: int = 7
    w_seen: float = 1.046875     # 1 + 3/64 (exact in bf16)
    eos_period: int = 150
    eos_phase: int = 40


def hadamard_rows(rows, n: int) -> np.ndarray:
    """Rows of the n x n Sylvester-Hadamard matrix: H[r][k] = (-1)^popcount(r & k)."""
    r = np.asarray(rows, dtype=np.int64)[:, None]
    k = np.arange(n, dtype=np.int64)[None, :]
    x = r & k
    par = np.zeros_like(x)
    while np.any(x):
        par ^= x & 1
        x >>= 1
    return (1 - 2 * par).astype(np.float32)


def chain_tokens(vocab, spec: ChainSpec) -> list[int]:
    rng = np.random.default_rng(spec.seed)
    codes = rng.permutation(vocab.codebook_size)[: spec.units]
    return [int(vocab.code_to_id(int(c))) for c in codes]


def chain_overrides(arch: configs.LmArch, spec: ChainSpec) -> dict[str, tuple[np.ndarray, np.ndarray]]:
    """{tensor name: (index, rows)} — rows (float32, bf16-exact) that replace tensor[index]
    (rows of the embedding / gate / up; columns of down, given transposed)."""
    if arch.hidden_size & (arch.hidden_size - 1) or spec.units + 1 > arch.hidden_size or \
            spec.units > arch.intermediate_size:
        raise ValueError("chain model needs a power-of-two hidden size >= units + 1")
    d = arch.hidden_size
    vocab = configs.vocab_for(arch)
    toks = chain_tokens(vocab, spec)
    eos = vocab.speech_end_id
    U = spec.units
    H = hadamard_rows(list(range(1, U + 1)) + [spec.eos_row], d)  # chain rows, then EOS
    s = np.float32(2.0 ** spec.emb_exp)
    emb_idx = np.asarray(toks + [eos], dtype=np.int64)
    emb_rows = H * s
    gate = H[:U] * np.float32(2.0 ** spec.gate_exp)
    down = np.zeros((U, d), dtype=np.float32)  # transposed: down[:, j] = down_t[j]
    q = np.float32(2.0 ** spec.down_exp)
    for j in range(U - 1):
        if j % spec.eos_period == spec.eos_phase:
            down[j] = q * (H[j + 1] + np.float32(2.0) * H[U])
        elif j >= spec.lag:
            down[j] = q * (H[j + 1] + np.float32(spec.w_seen) * H[j - spec.lag])
        else:
            down[j] = q * H[j + 1]
    p = "model.layers.0."
    unit_idx = np.arange(U, dtype=np.int64)
    out = {
        "model.embed_tokens.weight": (emb_idx, emb_rows),
        p + "mlp.gate_proj.weight": (unit_idx, gate),
        p + "mlp.up_proj.weight": (unit_idx, gate),
        p + "mlp.down_proj.weight.T": (unit_idx, down),
    }
    if not arch.tie_word_embeddings:  # untied (TTS-1-Max): the same rows in the lm_head
        out["lm_head.weight"] = (emb_idx, emb_rows)
    return out


def apply_chain(weights: dict[str, torch.Tensor], arch: configs.LmArch, spec: ChainSpec) -> None:
    """Overwrites the chain rows in place (CPU or device tensors; bit-identical results)."""
    for name, (idx, rows) in chain_overrides(arch, spec).items():
        transposed = name.endswith(".T")
        t = weights[name[:-2] if transposed else name]
        ix = torch.from_numpy(idx).to(t.device)
        v = torch.from_numpy(rows).to(device=t.device, dtype=t.dtype)
        if transposed:
            t[:, ix] = v.t()
        else:
            t[ix] = v


def chain_prompt(vocab, spec: ChainSpec, utt: int, start: int, n_text_tokens: int, n_prompt_codes: int) -> list[int]:
    """A synthetic prompt whose speech part ends with c_{start-lag-1} .. c_start, so that
    decoding follows the chain from c_{start+1} and every lagged id is already seen."""
    toks = chain_tokens(vocab, spec)
    if start < spec.lag + 1 or start >= spec.units - 1:
        raise ValueError("chain start out of range")
    base = synthetic_prompt(vocab, utt, n_text_tokens, n_prompt_codes)
    chain = set(toks)
    base = [t for t in base if t not in chain]  # (random prompt codes never hit the chain)
    return base + toks[start - spec.lag - 1: start + 1]


# -------------------------------------------------------------------- encoder weights ---

def encoder_tensor_specs(cfg: configs.EncoderArch) -> list[tuple[str, tuple[int, ...], float, float]]:
    """(name, shape, scale, offset) for the reference Encoder's own modules (encoder.py:20-46:
    semantic_encoder, acoustic_encoder with legacy weight_norm g / v, fusion_layer,
    quantizer.project_in / project_out).  Weight-norm directions v are uniform, magnitudes g
    near 1 (a conv keeps its input's scale), SnakeBeta log-scale alpha / beta near 0."""
    specs = []

    def wn(pre, co, ci, k):
        specs.extend([(pre + "weight_g", (co, 1, 1), 0.2, 1.0), (pre + "weight_v", (co, ci, k), 1.0, 0.0),
                      (pre + "bias", (co,), 0.01, 0.0)])

    def snake(pre, c):
        specs.extend([(pre + "act.alpha", (c,), 0.3, 0.0), (pre + "act.beta", (c,), 0.3, 0.0)])

    a = "acoustic_encoder."
    d = cfg.ngf
    wn(a + "conv_blocks.0.", d, 1, 7)
    for i, stride in enumerate(cfg.up_ratios, start=1):
        half, d = d, d * 2
        for r, _ in enumerate(cfg.dilations):
            pre = f"{a}conv_blocks.{i}.block.{r}.block."
            snake(pre + "0.", half)
            wn(pre + "1.", half, half, 7)
            snake(pre + "2.", half)
            wn(pre + "3.", half, half, 1)
        snake(f"{a}conv_blocks.{i}.block.3.", half)
        wn(f"{a}conv_blocks.{i}.block.4.", d, half, 2 * stride)
    snake(a + "conv_final_block.0.", d)
    wn(a + "conv_final_block.1.", cfg.acoustic_dim, d, 3)
    S = cfg.semantic_dim
    sc = math.sqrt(3.0 / (3 * S))
    specs += [("semantic_encoder.initial_conv.weight", (S, S, 3), sc, 0.0),
              ("semantic_encoder.residual_blocks.1.weight", (S, S, 3), sc, 0.0),
              ("semantic_encoder.residual_blocks.1.bias", (S,), 0.01, 0.0),
              ("semantic_encoder.residual_blocks.3.weight", (S, S, 3), sc, 0.0),
              ("semantic_encoder.residual_blocks.3.bias", (S,), 0.01, 0.0),
              ("semantic_encoder.final_conv.weight", (S, S, 3), sc, 0.0)]
    F = S + cfg.acoustic_dim
    fs = math.sqrt(3.0 / F)
    specs += [("fusion_layer.weight", (F, F), fs, 0.0), ("fusion_layer.bias", (F,), 0.01, 0.0),
              ("quantizer.project_in.weight", (len(cfg.levels), F), 2 * fs, 0.0),
              ("quantizer.project_in.bias", (len(cfg.levels),), 0.1, 0.0),
              ("quantizer.project_out.weight", (F, len(cfg.levels)), 0.2, 0.0),
              ("quantizer.project_out.bias", (F,), 0.01, 0.0)]
    return specs


def w2v_tensor_specs(cfg: configs.EncoderArch) -> list[tuple[str, tuple[int, ...], float, float]]:
    """(name, shape, scale, offset) for transformers' Wav2Vec2BertModel with
    `cfg.w2v_hf_config()` (the names of its state dict; layer norms near 1, linear weights of
    std 0.02 like its initializer)."""
    H, FF, Fi, hd = cfg.w2v_hidden, cfg.w2v_ffn, cfg.w2v_feat_in, cfg.w2v_hidden // cfg.w2v_heads
    lin = 0.02 * math.sqrt(3.0)

    def ln(pre, n):
        return [(pre + "weight", (n,), 0.1, 1.0), (pre + "bias", (n,), 0.02, 0.0)]

    specs = [("masked_spec_embed", (H,), 0.1, 0.0)]
    specs += ln("feature_projection.layer_norm.", Fi)
    specs += [("feature_projection.projection.weight", (H, Fi), math.sqrt(3.0 / Fi), 0.0),
              ("feature_projection.projection.bias", (H,), 0.01, 0.0)]
    for i in range(cfg.w2v_layers):
        p = f"encoder.layers.{i}."
        for f in ("ffn1", "ffn2"):
            specs += ln(p + f + "_layer_norm.", H)
            specs += [(p + f + ".intermediate_dense.weight", (FF, H), lin, 0.0),
                      (p + f + ".intermediate_dense.bias", (FF,), 0.01, 0.0),
                      (p + f + ".output_dense.weight", (H, FF), lin, 0.0),
                      (p + f + ".output_dense.bias", (H,), 0.01, 0.0)]
        specs += ln(p + "self_attn_layer_norm.", H)
        for n in ("q", "k", "v", "out"):
            specs += [(p + f"self_attn.linear_{n}.weight", (H, H), lin, 0.0),
                      (p + f"self_attn.linear_{n}.bias", (H,), 0.01, 0.0)]
        specs.append((p + "self_attn.distance_embedding.weight", (cfg.w2v_left + cfg.w2v_right + 1, hd), 0.5, 0.0))
        specs += ln(p + "conv_module.layer_norm.", H)
        specs += [(p + "conv_module.pointwise_conv1.weight", (2 * H, H, 1), lin, 0.0),
                  (p + "conv_module.depthwise_conv.weight", (H, 1, cfg.w2v_conv_k), 0.3, 0.0)]
        specs += ln(p + "conv_module.depthwise_layer_norm.", H)
        specs.append((p + "conv_module.pointwise_conv2.weight", (H, H, 1), lin, 0.0))
        specs += ln(p + "final_layer_norm.", H)
    return specs


def weights_from_specs_cpu(specs, seed: int) -> dict[str, torch.Tensor]:
    """fp32 CPU tensors of a spec list (the counter generator of this module)."""
    out = {}
    for name, shape, scale, off in specs:
        v = synth_values(tensor_seed(seed, name), int(np.prod(shape)), scale)
        t = torch.from_numpy(v).reshape(shape)
        out[name] = t + off if off else t
    return out


def weights_from_specs_device(specs, seed: int, device) -> dict[str, torch.Tensor]:
    """The same fp32 values generated on the GPU (tts_synth_fill) and returned on the host
    (bit-identical to weights_from_specs_cpu, a few seconds instead of minutes for w2v-bert)."""
    from . import _lib

    lib = _lib.load_library()
    out = {}
    for name, shape, scale, off in specs:
        t = torch.empty(shape, dtype=torch.float32, device=device)
        _lib.check(lib.tts_synth_fill(t.data_ptr(), _lib.DT_F32, int(np.prod(shape)), tensor_seed(seed, name), scale,
                                      _lib.stream_ptr()))
        out[name] = t + off if off else t
    torch.cuda.synchronize()
    return {k: v.cpu() for k, v in out.items()}


def kaiser_sinc_filter(cutoff: float, half_width: float, kernel_size: int) -> torch.Tensor:
    """The anti-aliasing filter of the encoder's Activation1d (filters.py:17-46, the julius /
    alias-free-torch Kaiser-windowed sinc), computed with the same torch CPU ops in fp32."""
    even = kernel_size % 2 == 0
    half_size = kernel_size // 2
    delta_f = 4 * half_width
    A = 2.285 * (half_size - 1) * math.pi * delta_f + 7.95
    if A > 50.0:
        beta = 0.1102 * (A - 8.7)
    elif A >= 21.0:
        beta = 0.5842 * (A - 21) ** 0.4 + 0.07886 * (A - 21.0)
    else:
        beta = 0.0
    window = torch.kaiser_window(kernel_size, beta=beta, periodic=False)
    time = (torch.arange(-half_size, half_size) + 0.5) if even else (torch.arange(kernel_size) - half_size)
    f = 2 * cutoff * window * torch.sinc(2 * cutoff * time)
    return (f / f.sum()).float()


def synthetic_wav(seed: int, n: int, sample_rate: int = 16000) -> np.ndarray:
    """A deterministic speech-like test signal: three drifting partials + noise, peak ~0.5."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / sample_rate
    f0 = 120 + 40 * rng.random()
    x = sum((0.3 / (h + 1)) * np.sin(2 * np.pi * f0 * (h + 1) * t * (1 + 0.05 * np.sin(2 * np.pi * 3 * t)) + rng.random())
            for h in range(3))
    x = x + 0.02 * rng.standard_normal(n)
    return x.astype(np.float32)


# ---------------------------------------------------------------------- codec weights ---

def codec_tensor_specs(cfg: configs.CodecArch) -> list[tuple[str, tuple[int, ...], float, float]]:
    """(name, shape, scale, offset) for the reference Decoder state dict (decoder.py:14-67)."""
    D, VQ = cfg.hidden_dim, cfg.vq_dim
    w = 0.02 * math.sqrt(3.0)
    b = 0.01
    specs = [
        ("decoder.quantizer.project_out.weight", (VQ, 8), 1.0 / math.sqrt(8), 0.0),
        ("decoder.quantizer.project_out.bias", (VQ,), b, 0.0),
        ("fc_post_a.weight", (D, VQ), 1.0 / math.sqrt(VQ), 0.0),
        ("fc_post_a.bias", (D,), b, 0.0),
        ("decoder.backbone.embed.weight", (D, D, 7), w, 0.0),
        ("decoder.backbone.embed.bias", (D,), b, 0.0),
    ]

    def resblock(pre, C, temb=False):
        s = [
            (pre + "norm1.weight", (C,), 0.1, 1.0), (pre + "norm1.bias", (C,), 0.05, 0.0),
            (pre + "conv1.weight", (C, C, 3), w, 0.0), (pre + "conv1.bias", (C,), b, 0.0),
        ]
        if temb:  # exists in upsampler blocks (temb_channels=512) but unused at inference
            s += [(pre + "temb_proj.weight", (C, 512), w, 0.0), (pre + "temb_proj.bias", (C,), b, 0.0)]
        s += [
            (pre + "norm2.weight", (C,), 0.1, 1.0), (pre + "norm2.bias", (C,), 0.05, 0.0),
            (pre + "conv2.weight", (C, C, 3), w, 0.0), (pre + "conv2.bias", (C,), b, 0.0),
        ]
        return s

    for i in range(2):
        specs += resblock(f"decoder.backbone.prior_net.{i}.", D)
    for i in range(cfg.depth):
        p = f"decoder.backbone.transformers.{i}."
        specs += [
            (p + "att_norm.weight", (D,), 0.1, 1.0),
            (p + "ffn_norm.weight", (D,), 0.1, 1.0),
            (p + "att.c_attn.weight", (3 * D, D), w, 0.0),
            (p + "att.c_proj.weight", (D, D), w, 0.0),
            (p + "mlp.fc1.weight", (4 * D, D), w, 0.0),
            (p + "mlp.fc2.weight", (D, 4 * D), w, 0.0),
        ]
    for i in range(2):
        specs += resblock(f"decoder.backbone.post_net.{i}.", D)
    specs += [
        ("decoder.backbone.final_layer_norm.weight", (D,), 0.1, 1.0),
        ("decoder.backbone.final_layer_norm.bias", (D,), 0.05, 0.0),
    ]
    C = D
    for i, (u, k) in enumerate(zip(cfg.upsample_factors, cfg.kernel_sizes)):
        p = f"upsampler.upsample_layers.{i}."
        specs += [
            (p + "weight_g", (C, 1, 1), 0.2, 1.0),
            (p + "weight_v", (C, C // 2, k), w, 0.0),
            (p + "bias", (C // 2,), b, 0.0),
        ]
        specs += resblock(f"upsampler.resnet_blocks.{i}.", C // 2, temb=True)
        C //= 2
    if cfg.upsample_factors:
        specs += [("upsampler.out_proj.weight", (D, C), w, 0.0), ("upsampler.out_proj.bias", (D,), b, 0.0)]
    nfft = 4 * cfg.hop_length
    specs += [
        ("decoder.head.out.weight", (nfft + 2, D), w, 0.0),
        ("decoder.head.out.bias", (nfft + 2,), b, 0.0),
    ]
    return specs


def codec_weights_cpu(cfg: configs.CodecArch, seed: int) -> dict[str, torch.Tensor]:
    out = {}
    for name, shape, scale, off in codec_tensor_specs(cfg):
        n = int(np.prod(shape))
        t = torch.from_numpy(synth_values(tensor_seed(seed, name), n, scale)).reshape(shape)
        out[name] = t + off if off else t
    # non-learned buffers that the reference state dict also carries
    nfft = 4 * cfg.hop_length
    out["decoder.head.istft.window"] = torch.hann_window(nfft)
    D = cfg.vq_dim
    out["decoder.quantizer.project_in.weight"] = torch.zeros(8, D)
    out["decoder.quantizer.project_in.bias"] = torch.zeros(8)
    return out


# ------------------------------------------------------------------------ inputs -------

def synthetic_prompt(vocab: configs.SpeechVocab, utt: int, n_text_tokens: int, n_prompt_codes: int,
                     rng_base: int = 1234) -> list[int]:
    """Prompt ids shaped like InferencePromptCompiler output (tts/core/prompting.py:124-154):
    BOS + instruction + <|text_prompt_start|> text <|text_prompt_end|> '\\n' <|speech_start|>
    + prompt speech codes."""
    rng = np.random.default_rng(rng_base + utt)
    text_hi = vocab.text_vocab
    ids = [vocab.bos_id]
    ids += rng.integers(0, text_hi, size=8).tolist()  # "Convert the text to speech:"
    ids += [vocab.text_prompt_start_id]
    ids += rng.integers(0, text_hi, size=n_text_tokens).tolist()
    ids += [vocab.text_prompt_end_id, vocab.newline_id, vocab.speech_start_id]
    codes = rng.integers(0, vocab.codebook_size, size=n_prompt_codes)
    ids += [vocab.code_to_id(int(c)) for c in codes]
    return [int(x) for x in ids]
