"""CPU oracle of the SpeechLM hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker / CPU baseline; the product path (tts-max_amd) never does.

A plain-torch restatement of what the reference executes for
``_generate_speech_tokens`` (tts/inference/inferencing.py:94-107): transformers
``LlamaForCausalLM`` (pinned 4.53.2 by uv.lock:4610-4611; third-party, so the arithmetic is
restated from its source) driven by ``GenerationMixin._sample`` in greedy mode:

* LlamaRMSNorm            modeling_llama.py:53-67   fp32 mean(x^2) -> rsqrt -> bf16 -> *w (bf16)
* LlamaRotaryEmbedding    modeling_llama.py:70-127, modeling_rope_utils.py:580-660 (llama3)
* apply_rotary_pos_emb    modeling_llama.py:138-160 (rotate_half; bf16 ops)
* LlamaAttention (sdpa)   modeling_llama.py:217-281 (GQA, scale D^-0.5, fp32 softmax; the
  probabilities enter P.V rounded to bf16, unnormalised, as torch's flash kernels do)
* LlamaMLP                modeling_llama.py:163-176 down(silu(gate) * up)
* LlamaDecoderLayer       modeling_llama.py:284-326 (bf16 residual adds)
* lm_head + _sample       generation/utils.py:2894-2925: bf16 logits -> .float() ->
  RepetitionPenaltyLogitsProcessor (logits_process.py:306-413, set of ids, x<0 ? x*p : x/p)
  -> MinNewTokensLengthLogitsProcessor (:164-236) -> argmax (first index on ties)

Pinning: tests/test_oracle_golden.py checks this restatement against fixtures produced by
running transformers' LlamaForCausalLM.generate itself (oracle/make_golden.py).
"""

from __future__ import annotations

import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tts-max_amd"))
from tts_amd import configs  # noqa: E402
from tts_amd.speechlm import hf_rope_table  # noqa: E402  (the table itself is pinned vs HF in tests)

BF16 = torch.bfloat16


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    xf = xf * torch.rsqrt(var + eps)
    return w * xf.to(x.dtype)


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """bf16 nn.Linear: fp32 accumulation, one rounding of the output."""
    return (x.float() @ w.float().t()).to(x.dtype)


def rotate_half(x):
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), dim=-1)


class LlamaOracle:
    """Greedy HF-semantics SpeechLM on CPU with a growing KV cache."""

    def __init__(self, arch: configs.LmArch, weights: dict[str, torch.Tensor], max_seq_len: int = 4096,
                 dtype=BF16):
        self.a = arch
        self.dtype = dtype
        self.w = {k: v.to(dtype) for k, v in weights.items()}
        if arch.tie_word_embeddings:
            self.w["lm_head.weight"] = self.w["model.embed_tokens.weight"]
        cos, sin = hf_rope_table(arch, max_seq_len)
        self.cos, self.sin = cos.to(dtype), sin.to(dtype)

    def forward(self, ids: list[int], start: int, cache: list) -> torch.Tensor:
        """Runs positions [start, start+len(ids)); returns the final hidden rows (pre-norm)."""
        a, w = self.a, self.w
        H, KVH, D = a.num_heads, a.num_kv_heads, a.head_dim
        n = len(ids)
        x = w["model.embed_tokens.weight"][torch.tensor(ids)]
        pos = torch.arange(start, start + n)
        cos, sin = self.cos[pos][:, None, :], self.sin[pos][:, None, :]
        for li in range(a.num_layers):
            p = f"model.layers.{li}."
            h = rmsnorm(x, w[p + "input_layernorm.weight"], a.rms_norm_eps)
            q = linear(h, w[p + "self_attn.q_proj.weight"]).view(n, H, D)
            k = linear(h, w[p + "self_attn.k_proj.weight"]).view(n, KVH, D)
            v = linear(h, w[p + "self_attn.v_proj.weight"]).view(n, KVH, D)
            q = (q * cos) + (rotate_half(q) * sin)
            k = (k * cos) + (rotate_half(k) * sin)
            if len(cache) <= li:
                cache.append([k, v])
            else:
                cache[li][0] = torch.cat([cache[li][0], k], 0)
                cache[li][1] = torch.cat([cache[li][1], v], 0)
            K, V = cache[li]
            ctx = K.shape[0]
            rep = H // KVH
            Kf = K.float().repeat_interleave(rep, dim=1).transpose(0, 1)  # [H, ctx, D]
            Vf = V.float().repeat_interleave(rep, dim=1).transpose(0, 1)
            qf = q.float().transpose(0, 1)                                 # [H, n, D]
            s = (qf @ Kf.transpose(1, 2)) * (1.0 / math.sqrt(D))
            qpos = pos[:, None]
            kpos = torch.arange(ctx)[None, :]
            s = s.masked_fill((kpos > qpos)[None], float("-inf"))
            # flash-attention numerics (torch's CPU flash kernel for bf16 and FA2 on GPU alike):
            # unnormalised p = exp(s - max) in fp32, p rounded to bf16 for the P.V product,
            # normaliser = fp32 sum of the unrounded p.
            pu = torch.exp(s - s.amax(-1, keepdim=True))
            lsum = pu.sum(-1, keepdim=True)
            o = ((pu.to(self.dtype).float() @ Vf) / lsum).transpose(0, 1).reshape(n, H * D).to(self.dtype)
            x = x + linear(o, w[p + "self_attn.o_proj.weight"])
            h = rmsnorm(x, w[p + "post_attention_layernorm.weight"], a.rms_norm_eps)
            g = linear(h, w[p + "mlp.gate_proj.weight"])
            u = linear(h, w[p + "mlp.up_proj.weight"])
            x = x + linear(torch.nn.functional.silu(g) * u, w[p + "mlp.down_proj.weight"])
        return x

    def logits(self, x_last: torch.Tensor) -> torch.Tensor:
        h = rmsnorm(x_last, self.w["model.norm.weight"], self.a.rms_norm_eps)
        return linear(h, self.w["lm_head.weight"]).float()

    def score(self, ids: list[int], n_last: int) -> torch.Tensor:
        """Teacher-forced bf16 logits (as fp32) of the last n_last positions."""
        x = self.forward(ids, 0, [])
        return self.logits(x[-n_last:])

    @staticmethod
    def process(scores: torch.Tensor, seen: list[int], penalty: float, new_len: int, min_new: int,
                eos: int) -> torch.Tensor:
        s = scores.clone()
        if penalty != 1.0:
            idx = torch.tensor(sorted(set(seen)), dtype=torch.long)
            g = s[idx]
            s[idx] = torch.where(g < 0, g * penalty, g / penalty)
        if eos >= 0 and new_len < min_new:
            s[eos] = float("-inf")
        return s

    def generate(self, prompt: list[int], max_length: int, min_new_tokens: int = 0, eos_token_id: int = -1,
                 repetition_penalty: float = 1.0):
        """Returns (new_tokens, margins): margins[i] = top1 - top2 of the processed scores."""
        if len(prompt) >= max_length:
            raise ValueError("input length >= max_length")
        cache: list = []
        x = self.forward(prompt, 0, cache)
        seq = list(prompt)
        new, margins = [], []
        while True:
            sc = self.process(self.logits(x[-1:])[0], seq, repetition_penalty, len(seq) - len(prompt),
                              min_new_tokens, eos_token_id)
            top = torch.topk(sc, 2)
            tok = int(torch.argmax(sc))
            margins.append(float(top.values[0] - top.values[1]))
            new.append(tok)
            seq.append(tok)
            if tok == eos_token_id or len(seq) >= max_length:
                break
            x = self.forward([tok], len(seq) - 1, cache)
        return new, margins


def sample_probs(scores: torch.Tensor, temperature: float, top_k: int, top_p: float) -> torch.Tensor:
    """The distribution GenerationMixin._sample draws from (generation/utils.py:2918-2923,
    `probs = softmax(next_token_scores)`) after the sampling warpers, in the order
    _get_logits_processor appends them (generation/utils.py, `if generation_config.do_sample`):

    * TemperatureLogitsWarper (logits_process.py:238-300): scores / T, only when T != 1.0
    * TopKLogitsWarper (logits_process.py:542-580): k = min(top_k, V); remove
      `scores < topk(scores, k).values[..., -1]` (ties with the k-th value are kept)
    * TopPLogitsWarper (logits_process.py:473-540), only when top_p < 1.0: ascending sort,
      softmax, cumsum; remove `cum <= 1 - top_p`, except the largest (min_tokens_to_keep=1)

    `scores` is one row of processed fp32 logits (after repetition penalty / EOS mask).
    Pinned against transformers' own warper classes in tests/test_oracle_golden.py."""
    s = scores.float().clone()
    if temperature != 1.0:
        s = s / temperature
    if top_k and top_k > 0:
        k = min(top_k, s.numel())
        kth = torch.topk(s, k).values[-1]
        s = s.masked_fill(s < kth, float("-inf"))
    if top_p < 1.0:
        sv, si = torch.sort(s, descending=False)
        cum = sv.softmax(dim=-1).cumsum(dim=-1)
        rm = cum <= (1 - top_p)
        rm[-1:] = False
        s = s.masked_fill(rm.scatter(0, si, rm), float("-inf"))
    return torch.softmax(s, dim=-1)


def vllm_process(scores: torch.Tensor, prompt: list[int], output: list[int], repetition_penalty: float,
                 frequency_penalty: float, min_tokens: int, stop_id: int) -> torch.Tensor:
    """vLLM's penalties for the vLLM form of the reference call (inferencing.py:75-92:
    repetition_penalty, frequency_penalty, min_tokens, stop_token_ids), restated from vLLM's
    `apply_penalties` (vllm/model_executor/layers/utils.py; vLLM is not installed here and
    the reference pins no version of it, so this restatement is PARITY UNPINNED):
    repetition over ids in prompt | output (logits > 0 ? /p : *p), then
    `logits -= frequency_penalty * count(id in output)`, and the stop id masked while
    len(output) < min_tokens (MinTokensLogitsProcessor)."""
    s = scores.float().clone()
    seen = sorted(set(prompt) | set(output))
    if repetition_penalty != 1.0 and seen:
        idx = torch.tensor(seen, dtype=torch.long)
        g = s[idx]
        s[idx] = torch.where(g > 0, g / repetition_penalty, g * repetition_penalty)
    if frequency_penalty != 0.0 and output:
        cnt = torch.bincount(torch.tensor(output, dtype=torch.long), minlength=s.numel()).float()
        s = s - frequency_penalty * cnt
    if stop_id >= 0 and len(output) < min_tokens:
        s[stop_id] = float("-inf")
    return s
