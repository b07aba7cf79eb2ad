"""HF-compatible SpeechLM surface backed by the MI355X engine.

``MI355XSpeechLM.generate`` is a drop-in for the call the reference makes in
tts/inference/inferencing.py:94-107::

    model.generate(input_ids=[1, P] LongTensor, max_length=, min_new_tokens=,
                   eos_token_id=, do_sample=, repetition_penalty=, top_p=, temperature=)
    -> LongTensor [1, P + N]   (prompt + new tokens, EOS included when produced)

and ``generate(prompt_token_ids=list, sampling_params=...)`` mirrors the vLLM form of
inferencing.py:75-92 (completion ids only, ``max_tokens`` counts new tokens).  Arithmetic
follows transformers LlamaForCausalLM + GenerationMixin._sample (pinned 4.53.2 by the
reference's uv.lock:4610); see DESIGN.md for the exact rounding points.
"""

from __future__ import annotations

import ctypes
import dataclasses
import json
import math
import os
import threading
from typing import Any, Sequence

import numpy as np
import torch

from . import _lib, configs, synth


def hf_rope_table(arch: configs.LmArch, max_seq_len: int) -> tuple[torch.Tensor, torch.Tensor]:
    """cos/sin [max_seq_len, head_dim] bf16 exactly as LlamaRotaryEmbedding computes them
    (transformers modeling_llama.py LlamaRotaryEmbedding.forward and
    modeling_rope_utils.py:580-660 `_compute_llama3_parameters`): fp32 inv_freq, fp32
    `inv_freq @ position`, cat(freqs, freqs), fp32 cos/sin, then cast to bf16."""
    dim = arch.head_dim
    inv_freq = 1.0 / (arch.rope_theta ** (torch.arange(0, dim, 2, dtype=torch.int64).to(dtype=torch.float) / dim))
    if arch.rope_llama3:
        factor, lo, hi = arch.rope_factor, arch.rope_low_freq_factor, arch.rope_high_freq_factor
        old = arch.rope_original_max_position
        low_freq_wavelen = old / lo
        high_freq_wavelen = old / hi
        wavelen = 2 * math.pi / inv_freq
        inv_freq_llama = torch.where(wavelen > low_freq_wavelen, inv_freq / factor, inv_freq)
        smooth = (old / wavelen - lo) / (hi - lo)
        smoothed = (1 - smooth) * inv_freq_llama / factor + smooth * inv_freq_llama
        is_medium = ~(wavelen < high_freq_wavelen) * ~(wavelen > low_freq_wavelen)
        inv_freq = torch.where(is_medium, smoothed, inv_freq_llama)
    pos = torch.arange(max_seq_len)[None, :]
    inv_e = inv_freq[None, :, None].float()
    pos_e = pos[:, None, :].float()
    freqs = (inv_e @ pos_e).transpose(1, 2)
    emb = torch.cat((freqs, freqs), dim=-1)
    cos = (emb.cos() * 1.0).to(torch.bfloat16)[0]
    sin = (emb.sin() * 1.0).to(torch.bfloat16)[0]
    return cos.contiguous(), sin.contiguous()


@dataclasses.dataclass
class CompletionOutput:
    token_ids: list[int]


@dataclasses.dataclass
class RequestOutput:
    prompt_token_ids: list[int]
    outputs: list[CompletionOutput]


def lm_config(arch: configs.LmArch, max_batch: int = 1, max_seq_len: int = 2048) -> "_lib.LmConfig":
    """The C ABI's tts_lm_config of an architecture."""
    return _lib.LmConfig(
        hidden_size=arch.hidden_size, num_layers=arch.num_layers, num_heads=arch.num_heads,
        num_kv_heads=arch.num_kv_heads, head_dim=arch.head_dim, intermediate_size=arch.intermediate_size,
        vocab_size=arch.vocab_size, tie_word_embeddings=int(arch.tie_word_embeddings),
        rms_norm_eps=arch.rms_norm_eps, rope_theta=arch.rope_theta, rope_llama3=int(arch.rope_llama3),
        rope_factor=arch.rope_factor, rope_low_freq_factor=arch.rope_low_freq_factor,
        rope_high_freq_factor=arch.rope_high_freq_factor,
        rope_original_max_position=arch.rope_original_max_position, max_batch=max_batch,
        max_seq_len=max_seq_len)


def step_plan(arch: configs.LmArch, rows: int, num_cu: int = 256) -> list[str]:
    """The kernels one decode step over `rows` rows launches (tts_debug_step_plan: the
    engine's step code in dry-run mode; no GPU needed): unique, in first-seen order."""
    lib = _lib.load_library()
    cfg = lm_config(arch, max_batch=max(rows, 1), max_seq_len=2048)
    buf = ctypes.create_string_buffer(1 << 16)
    _lib.check(lib.tts_debug_step_plan(ctypes.byref(cfg), rows, num_cu, buf, len(buf)))
    return [ln for ln in buf.value.decode().splitlines() if ln]


class MI355XSpeechLM:
    """One SpeechLM resident on one MI355X (one engine, one stream)."""

    def __init__(self, arch: configs.LmArch, weights: dict[str, torch.Tensor], device: int = 0,
                 max_batch: int = 1, max_seq_len: int = 2048, id_to_code: np.ndarray | None = None):
        self.arch = arch
        self.device = torch.device("cuda", device)
        self.max_batch = max_batch
        self.max_seq_len = max_seq_len
        self._lib = _lib.load_library()
        # one engine = one caller at a time (C ABI: not re-entrant); the continuous batcher
        # that holds the engine's slot batch, if any (serving.ContinuousBatcher)
        self.lock = threading.RLock()
        self._slot_batcher = None
        h = ctypes.c_void_p()
        _lib.check(self._lib.tts_engine_create(device, ctypes.byref(h)))
        self._h = h
        cfg = lm_config(arch, max_batch, max_seq_len)
        cos, sin = hf_rope_table(arch, max_seq_len)
        tensors = dict(weights)
        tensors["rope.cos"] = cos
        tensors["rope.sin"] = sin
        if id_to_code is not None:
            tensors["vocab.id_to_code"] = torch.from_numpy(np.ascontiguousarray(id_to_code, dtype=np.int32))
        descs, keep = _lib.make_descs(tensors)
        torch.cuda.synchronize()
        _lib.check(self._lib.tts_lm_load(self._h, ctypes.byref(cfg), descs, len(tensors)))
        del keep
        self.generation_config = type("GenerationConfig", (), {"eos_token_id": None, "top_k": 50})()

    # ------------------------------------------------------------------ constructors ---
    @classmethod
    def synthetic(cls, arch: configs.LmArch, seed: int = 0x5EED, device: int = 0,
                  chain: "synth.ChainSpec | None" = None, **kw) -> "MI355XSpeechLM":
        """Random-init weights of `arch`, generated on the device (bit-identical to the
        CPU generator the golden fixtures were made with); `chain` overwrites the rows of
        the decisive-parity model (synth.apply_chain)."""
        w = synth.lm_weights_device(arch, seed, torch.device("cuda", device))
        if chain is not None:
            synth.apply_chain(w, arch, chain)
        vocab = configs.vocab_for(arch)
        m = cls(arch, w, device=device, id_to_code=vocab.id_to_code(), **kw)
        del w
        torch.cuda.empty_cache()
        return m

    @classmethod
    def from_pretrained(cls, model_dir: str, device: int = 0, **kw) -> "MI355XSpeechLM":
        """Loads a serving directory written by tools/serving/convert_checkpoint.py
        (config.json + *.safetensors + tokenizer files + generation_config.json)."""
        from safetensors.torch import load_file

        arch = configs.LmArch.from_hf_config(os.path.join(model_dir, "config.json"), name=os.path.basename(model_dir))
        weights: dict[str, torch.Tensor] = {}
        for f in sorted(os.listdir(model_dir)):
            if f.endswith(".safetensors"):
                weights.update(load_file(os.path.join(model_dir, f)))
        weights = {k: v for k, v in weights.items() if k.startswith(("model.", "lm_head."))}
        lut = None
        tok_path = os.path.join(model_dir, "tokenizer.json")
        if os.path.exists(tok_path):
            lut = id_to_code_from_tokenizer_json(tok_path, arch.vocab_size)
        m = cls(arch, weights, device=device, id_to_code=lut, **kw)
        gc = os.path.join(model_dir, "generation_config.json")
        if os.path.exists(gc):
            with open(gc) as f:
                g = json.load(f)
            m.generation_config.eos_token_id = g.get("eos_token_id")
        return m

    # ------------------------------------------------------------------ generation -----
    def generate(self, input_ids: torch.Tensor | None = None, max_length: int | None = None,
                 min_new_tokens: int = 0, eos_token_id: int | None = None, do_sample: bool = False,
                 repetition_penalty: float = 1.0, top_p: float = 1.0, temperature: float = 1.0,
                 top_k: int | None = None, max_new_tokens: int | None = None,
                 prompt_token_ids: Sequence[int] | None = None, sampling_params: Any = None, **unused):
        if prompt_token_ids is not None:
            return self._generate_vllm_form(prompt_token_ids, sampling_params)
        if input_ids is None:
            raise ValueError("input_ids is required")
        ids = input_ids if input_ids.dim() == 2 else input_ids[None]
        P = ids.shape[1]
        if max_length is None:
            max_length = P + (max_new_tokens if max_new_tokens is not None else 20)
        if eos_token_id is None:
            eos_token_id = self.generation_config.eos_token_id
        if isinstance(eos_token_id, (list, tuple)):
            if len(eos_token_id) != 1:
                raise NotImplementedError("a single eos_token_id is supported")
            eos_token_id = eos_token_id[0]
        if P >= max_length:
            raise ValueError(f"Input length of input_ids is {P}, but `max_length` is set to {max_length}.")
        prompts = [row.tolist() for row in ids.cpu()]
        new = self.generate_batch(prompts, max_length=max_length, min_new_tokens=min_new_tokens,
                                  eos_token_id=-1 if eos_token_id is None else int(eos_token_id),
                                  do_sample=do_sample, repetition_penalty=repetition_penalty, top_p=top_p,
                                  temperature=temperature, top_k=top_k)
        if len(new) == 1:
            out = torch.tensor([prompts[0] + new[0]], dtype=torch.long)
        else:  # HF pads finished rows with pad = eos; keep that shape convention
            L = max(len(p) + len(n) for p, n in zip(prompts, new))
            pad = eos_token_id if eos_token_id is not None else 0
            out = torch.full((len(new), L), pad, dtype=torch.long)
            for i, (p, n) in enumerate(zip(prompts, new)):
                out[i, :len(p) + len(n)] = torch.tensor(p + n)
        return out.to(input_ids.device)

    def generate_batch(self, prompts: Sequence[Sequence[int]], max_length: int, min_new_tokens: int = 0,
                       eos_token_id: int = -1, do_sample: bool = False, repetition_penalty: float = 1.0,
                       top_p: float = 1.0, temperature: float = 1.0, top_k: int | None = None,
                       seed: int | None = None, frequency_penalty: float = 0.0) -> list[list[int]]:
        """Independent sequences (each as its batch-1 HF generate): returns new tokens.

        do_sample: GenerationMixin._sample's warpers (temperature, top_k — HF default 50 —,
        top_p) and a multinomial draw from the engine's counter-based RNG.  `seed=None`
        draws the seed from torch's default generator, so torch.manual_seed() makes runs
        reproducible as it does for HF (the token streams differ from HF's: only the
        distribution is shared)."""
        if do_sample and seed is None:
            seed = int(torch.randint(0, 2**62, (1,)).item())
        B = len(prompts)
        if B < 1 or B > self.max_batch:
            raise ValueError(f"batch {B} outside [1, max_batch={self.max_batch}]")
        with self.lock:
            self._take_from_batcher()
            return self._generate_batch_locked(prompts, max_length, min_new_tokens, eos_token_id, do_sample,
                                               repetition_penalty, top_p, temperature, top_k, seed,
                                               frequency_penalty)

    def _take_from_batcher(self):
        """A one-shot generation reuses the decode rows a continuous batcher holds: refuse while
        it serves requests, otherwise let it reopen its slot batch next time."""
        b = self._slot_batcher
        if b is not None:
            if b.busy():
                raise RuntimeError("the engine's continuous batcher is serving requests; "
                                   "use the batcher (or another engine) for this generation")
            self._slot_batcher = None

    def _generate_batch_locked(self, prompts, max_length, min_new_tokens, eos_token_id, do_sample,
                               repetition_penalty, top_p, temperature, top_k, seed, frequency_penalty):
        B = len(prompts)
        lens = np.array([len(p) for p in prompts], dtype=np.int32)
        for p in prompts:
            if len(p) >= max_length:
                raise ValueError(f"Input length of input_ids is {len(p)}, but `max_length` is set to {max_length}.")
        flat = np.ascontiguousarray(np.concatenate([np.asarray(p, dtype=np.int32) for p in prompts]))
        stride = max(1, max_length - int(lens.min()))
        out = np.zeros((B, stride), dtype=np.int32)
        out_lens = np.zeros(B, dtype=np.int32)
        params = _lib.GenParams(max_length=max_length, min_new_tokens=min_new_tokens, eos_token_id=eos_token_id,
                                do_sample=1 if do_sample else 0, repetition_penalty=repetition_penalty,
                                temperature=temperature, top_p=top_p, top_k=50 if top_k is None else top_k,
                                seed=0 if seed is None else seed, frequency_penalty=frequency_penalty)
        pi32 = ctypes.POINTER(ctypes.c_int32)
        _lib.check(self._lib.tts_generate(self._h, ctypes.byref(params), flat.ctypes.data_as(pi32),
                                          lens.ctypes.data_as(pi32), B, out.ctypes.data_as(pi32), stride,
                                          out_lens.ctypes.data_as(pi32), None))
        return [out[b, :out_lens[b]].tolist() for b in range(B)]

    def generate_stream(self, prompts: Sequence[Sequence[int]], max_length: int, chunk: int = 25,
                        min_new_tokens: int = 0, eos_token_id: int = -1, do_sample: bool = False,
                        repetition_penalty: float = 1.0, top_p: float = 1.0, temperature: float = 1.0,
                        top_k: int | None = None, seed: int | None = None):
        """Chunked generation (config 5): yields (new_tokens_per_row, all_done) after the first
        token and then after every `chunk` further decode steps.  The rows' final tokens are
        identical to generate_batch with the same arguments (same device loop, paused).

        The engine lock is held while the generator is alive (one open generation per
        engine): consume it to the end or close() it, in the thread that created it —
        closing (or garbage collection) releases the lock through the `with` block."""
        if do_sample and seed is None:
            seed = int(torch.randint(0, 2**62, (1,)).item())
        B = len(prompts)
        if B < 1 or B > self.max_batch:
            raise ValueError(f"batch {B} outside [1, max_batch={self.max_batch}]")
        lens = np.array([len(p) for p in prompts], dtype=np.int32)
        if int(lens.max()) >= max_length:
            raise ValueError(f"Input length of input_ids is {int(lens.max())}, but `max_length` is set to {max_length}.")
        flat = np.ascontiguousarray(np.concatenate([np.asarray(p, dtype=np.int32) for p in prompts]))
        params = _lib.GenParams(max_length=max_length, min_new_tokens=min_new_tokens, eos_token_id=eos_token_id,
                                do_sample=1 if do_sample else 0, repetition_penalty=repetition_penalty,
                                temperature=temperature, top_p=top_p, top_k=50 if top_k is None else top_k,
                                seed=0 if seed is None else seed)
        with self.lock:
            self._take_from_batcher()
            yield from self._stream_locked(B, flat, lens, params, max_length, chunk)

    def _stream_locked(self, B, flat, lens, params, max_length, chunk):
        pi32 = ctypes.POINTER(ctypes.c_int32)
        _lib.check(self._lib.tts_generate_begin(self._h, ctypes.byref(params), flat.ctypes.data_as(pi32),
                                                lens.ctypes.data_as(pi32), B, None))
        stride = max(1, max_length - int(lens.min()))
        out = np.zeros((B, stride), dtype=np.int32)
        out_lens = np.zeros(B, dtype=np.int32)
        done = ctypes.c_int32(0)
        steps = 0
        while True:
            _lib.check(self._lib.tts_generate_read(self._h, out.ctypes.data_as(pi32), stride,
                                                   out_lens.ctypes.data_as(pi32)))
            yield [out[b, :out_lens[b]].tolist() for b in range(B)], bool(done.value)
            if done.value:
                return
            _lib.check(self._lib.tts_generate_continue(self._h, chunk, ctypes.byref(done)))
            steps += 1

    def _generate_vllm_form(self, prompt_token_ids, sampling_params):
        sp = sampling_params
        temperature = float(getattr(sp, "temperature", 1.0) or 0.0)
        if float(getattr(sp, "presence_penalty", 0.0) or 0.0) != 0.0:
            raise NotImplementedError("vLLM presence_penalty is not implemented")
        top_k = int(getattr(sp, "top_k", -1) or -1)
        if temperature > 0 and top_k <= 0:
            raise NotImplementedError("full-vocabulary sampling (vLLM top_k=-1) is not built; pass top_k")
        max_tokens = int(getattr(sp, "max_tokens", 16))
        stop = list(getattr(sp, "stop_token_ids", None) or [])
        prompt = list(prompt_token_ids)
        new = self.generate_batch([prompt], max_length=len(prompt) + max_tokens,
                                  min_new_tokens=int(getattr(sp, "min_tokens", 0)),
                                  eos_token_id=stop[0] if stop else -1,
                                  repetition_penalty=float(getattr(sp, "repetition_penalty", 1.0)),
                                  do_sample=temperature > 0, temperature=temperature or 1.0,
                                  top_p=float(getattr(sp, "top_p", 1.0)),
                                  top_k=top_k if top_k > 0 else None,
                                  seed=getattr(sp, "seed", None),
                                  frequency_penalty=float(getattr(sp, "frequency_penalty", 0.0) or 0.0))[0]
        return [RequestOutput(prompt_token_ids=prompt, outputs=[CompletionOutput(token_ids=new)])]

    # ------------------------------------------------------------------ utilities ------
    def score(self, sequences: Sequence[Sequence[int]], n_last: int) -> torch.Tensor:
        """Teacher-forced bf16 logits (as fp32) of the last n_last positions: [B, n_last, V]."""
        with self.lock:
            self._take_from_batcher()
            return self._score_locked(sequences, n_last)

    def _score_locked(self, sequences, n_last):
        B = len(sequences)
        lens = np.array([len(s) for s in sequences], dtype=np.int32)
        flat = np.ascontiguousarray(np.concatenate([np.asarray(s, dtype=np.int32) for s in sequences]))
        out = np.zeros((B, n_last, self.arch.vocab_size), dtype=np.float32)
        pi32 = ctypes.POINTER(ctypes.c_int32)
        _lib.check(self._lib.tts_lm_score(self._h, flat.ctypes.data_as(pi32), lens.ctypes.data_as(pi32), B, n_last,
                                          out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), None))
        return torch.from_numpy(out)

    def score_decode(self, sequences: Sequence[Sequence[int]], n_last: int,
                     gather_idx: np.ndarray | None = None) -> torch.Tensor:
        """Teacher-forced bf16 logits (as fp32) of the last n_last positions computed by the
        DECODE step (prefill of the prefixes, then one decode step per position, all sequences
        as one batch): [B, n_last, V], or [B, n_last, k] at gather_idx [B, n_last, k]."""
        with self.lock:
            self._take_from_batcher()
            B = len(sequences)
            lens = np.array([len(s) for s in sequences], dtype=np.int32)
            flat = np.ascontiguousarray(np.concatenate([np.asarray(s, dtype=np.int32) for s in sequences]))
            pi32 = ctypes.POINTER(ctypes.c_int32)
            if gather_idx is not None:
                gi = np.ascontiguousarray(np.asarray(gather_idx, dtype=np.int32))
                if gi.ndim != 3 or gi.shape[:2] != (B, n_last):
                    raise ValueError("gather_idx must be [batch, n_last, k]")
                k = gi.shape[2]
                gptr = gi.ctypes.data_as(pi32)
            else:
                k, gptr = self.arch.vocab_size, None
            out = np.zeros((B, n_last, k), dtype=np.float32)
            _lib.check(self._lib.tts_lm_score_decode(self._h, flat.ctypes.data_as(pi32), lens.ctypes.data_as(pi32), B,
                                                     n_last, gptr, k,
                                                     out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), None))
            return torch.from_numpy(out)

    def last_timing(self) -> tuple[float, float, int]:
        a, b, n = ctypes.c_float(), ctypes.c_float(), ctypes.c_int32()
        _lib.check(self._lib.tts_lm_last_timing(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(n)))
        return a.value, b.value, n.value

    KERNELS = ("qkv", "o_proj", "gate_up", "down", "lm_head", "attention")

    def bench_kernel(self, which: str, rows: int = 1, ctx: int = 450, iters: int = 50) -> tuple[float, float]:
        """(avg ms per launch, algorithmic bytes per launch) of one decode-step kernel."""
        ms, b = ctypes.c_float(), ctypes.c_double()
        # qkv_attn: QKV with the decode attention fused in (the one-row step's form);
        # qkv_attn_oproj: the same launch also carrying o_proj (the default 1..16-row step)
        sel = {"qkv_attn": 6, "qkv_attn_oproj": 7, "head_screened": 8, "head_screen": 9}.get(which)
        sel = self.KERNELS.index(which) if sel is None else sel
        _lib.check(self._lib.tts_lm_bench_kernel(self._h, sel, rows, ctx, iters,
                                                 ctypes.byref(ms), ctypes.byref(b)))
        return ms.value, b.value

    def ids_to_codes(self, ids: Sequence[int]) -> list[int]:
        arr = np.ascontiguousarray(np.asarray(ids, dtype=np.int32))
        out = np.zeros_like(arr)
        pi32 = ctypes.POINTER(ctypes.c_int32)
        _lib.check(self._lib.tts_lm_id_to_code(self._h, arr.ctypes.data_as(pi32), len(arr), out.ctypes.data_as(pi32)))
        return out.tolist()

    def close(self):
        if getattr(self, "_h", None):
            self._lib.tts_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def id_to_code_from_tokenizer_json(path: str, vocab_size: int) -> np.ndarray:
    """Token id -> speech code LUT from a tokenizer.json's added tokens (<|s_N|> -> N),
    replacing the per-token string parse of inferencing.py:53-63 + batch_decode."""
    with open(path) as f:
        tj = json.load(f)
    lut = np.full(vocab_size, -1, dtype=np.int32)
    entries = list(tj.get("added_tokens", []))
    vocab = tj.get("model", {}).get("vocab", {})
    items = [(e["content"], e["id"]) for e in entries] + list(vocab.items() if isinstance(vocab, dict) else [])
    for content, i in items:
        if isinstance(content, str) and content.startswith("<|s_") and content.endswith("|>") and 0 <= i < vocab_size:
            try:
                lut[i] = int(content[4:-2])
            except ValueError:
                pass
    return lut
