#!/usr/bin/env python
"""Generates the golden fixtures under tests/golden/ — RUN IN THE BUILD CONTAINER ONLY.

It executes the reference implementations themselves on CPU:

* SpeechLM: transformers ``LlamaForCausalLM.generate`` (the third-party arithmetic behind
  tts/inference/inferencing.py:94-107), called with the reference's greedy settings
  (do_sample=False, repetition_penalty, min_new_tokens, eos_token_id=<|speech_end|>,
  max_length = total length).
* Codec: the reference ``tts.core.codec.decoder.Decoder`` imported from /root/reference with
  the absent third-party modules restated under oracle/shims (see shims/README.md).

Weights and inputs are synthetic and deterministic (tts_amd.synth), so the GPU box can
rebuild them bit-identically without shipping weights.  The script also checks the CPU
restatements (oracle/lm_oracle.py, oracle/codec_oracle.py) against the reference outputs
and records the agreement in tests/golden/manifest.json.

    python oracle/make_golden.py            # all fixtures
    python oracle/make_golden.py --only lm_tiny
"""

from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))
sys.path.insert(0, ROOT)
from tts_amd import configs, synth  # noqa: E402
from oracle import codec_oracle, lm_oracle  # noqa: E402
from oracle.hf_ref import hf_generate, hf_model  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")

# (fixture, arch, weight seed, [(utt, n_text, n_prompt_codes)], settings)
LM_CASES = {
    "lm_tiny": ("tiny", 11, [(0, 5, 0), (1, 12, 20), (2, 30, 64)],
                [dict(new=40, min_new=10, rep=1.1), dict(new=24, min_new=0, rep=1.4), dict(new=48, min_new=48, rep=1.0)]),
    "lm_small": ("small", 12, [(0, 20, 50), (1, 7, 3)], [dict(new=64, min_new=10, rep=1.1), dict(new=32, min_new=5, rep=1.3)]),
    "lm_tiny128": ("tiny128", 13, [(0, 9, 16)], [dict(new=32, min_new=8, rep=1.1)]),
    "lm_tts1": ("tts1", 0x5EED, [(0, 40, 150), (1, 25, 60)],
                [dict(new=48, min_new=48, rep=1.1), dict(new=32, min_new=10, rep=1.4)]),
}

CODEC_CASES = {
    "codec_24k": ("codec-24k", 0xC0DEC, [60, 1, 7]),
    "codec_16k": ("xcodec2-16k", 0xC0DEC + 1, [40]),
    "codec_48k": ("codec-48k", 0xC0DEC + 2, [30]),
    "codec_24k_d2": ("codec-24k-d2", 0xC0DEC + 3, [50, 3]),
    # the bench's codec leg (650 codes = 150 prompt + 500 generated; 11 key chunks of 64 in
    # the codec attention) and three lengths between
    "codec_24k_long": ("codec-24k", 0xC0DEC, [650, 300, 130, 65]),
}


def lm_fixture(name: str, manifest: dict) -> None:
    arch_name, seed, prompts, settings = LM_CASES[name]
    arch = configs.LM_ARCHS[arch_name]
    vocab = configs.vocab_for(arch)
    t0 = time.time()
    w = synth.lm_weights_cpu(arch, seed)
    model = hf_model(arch, w)
    orc = lm_oracle.LlamaOracle(arch, w, max_seq_len=4096)
    eos = vocab.speech_end_id
    rec = dict(prompt_ids=[], prompt_lens=[], hf_new=[], hf_new_lens=[], oracle_new=[], oracle_lens=[],
               oracle_margins=[], max_length=[], min_new=[], rep=[], eos=[])
    stats = []
    for (utt, n_text, n_codes), st in zip(prompts, settings):
        prompt = synth.synthetic_prompt(vocab, utt, n_text, n_codes)
        P = len(prompt)
        max_length = P + st["new"]
        hf_new, hf_margins, _ = hf_generate(model, prompt, max_length, st["min_new"], eos, st["rep"])
        rec.setdefault("hf_margins", []).extend(hf_margins)
        o_new, margins = orc.generate(prompt, max_length, st["min_new"], eos, st["rep"])
        agree = 0
        while agree < min(len(hf_new), len(o_new)) and hf_new[agree] == o_new[agree]:
            agree += 1
        # teacher-forced logits on the HF sequence: HF forward vs oracle
        seq = prompt + hf_new
        with torch.no_grad():
            hf_logits = model(torch.tensor([seq])).logits[0, -8:].float()
        o_logits = orc.score(seq, 8)
        diff = (hf_logits - o_logits).abs().max().item()
        if arch.vocab_size > 100000:  # engine-vs-transformers logits: top-32 + 32 fixed indices per step
            n_tf = len(hf_new)
            with torch.no_grad():
                tf = model(torch.tensor([seq[:-1]])).logits[0, -n_tf:].float()
            gen = torch.Generator().manual_seed(utt)
            idx = torch.cat([torch.topk(tf, 32, dim=-1).indices,
                             torch.randint(0, arch.vocab_size, (n_tf, 32), generator=gen)], dim=1)
            rec.setdefault("tf_idx", []).append(idx.numpy().astype(np.int32))
            rec.setdefault("tf_val", []).append(torch.gather(tf, 1, idx).numpy().astype(np.float32))
            o_tf = orc.score(seq[:-1], n_tf)
            tf_oracle_dev = (torch.gather(o_tf, 1, idx) - torch.gather(tf, 1, idx)).abs()
        stats.append(dict(P=P, n_new=len(hf_new), agree_prefix=agree, identical=hf_new == o_new,
                          min_margin=min(margins), hf_min_margin=min(hf_margins),
                          first_hf_near_tie=next((i for i, m in enumerate(hf_margins) if m < 0.25), None),
                          max_abs_logit_diff=diff,
                          logit_scale=hf_logits.abs().max().item()))
        if arch.vocab_size > 100000:
            stats[-1].update(tf_oracle_max=float(tf_oracle_dev.max()), tf_oracle_mean=float(tf_oracle_dev.mean()))
        rec["prompt_ids"] += prompt
        rec["prompt_lens"].append(P)
        rec["hf_new"] += hf_new
        rec["hf_new_lens"].append(len(hf_new))
        rec["oracle_new"] += o_new
        rec["oracle_lens"].append(len(o_new))
        rec["oracle_margins"] += margins
        rec["max_length"].append(max_length)
        rec["min_new"].append(st["min_new"])
        rec["rep"].append(st["rep"])
        rec["eos"].append(eos)
    for k in ("tf_idx", "tf_val"):
        if k in rec:
            rec[k] = np.concatenate(rec[k])
    np.savez_compressed(os.path.join(GOLDEN, f"{name}.npz"), arch=arch_name, seed=seed,
                        **{k: np.asarray(v) for k, v in rec.items()})
    manifest[name] = dict(kind="lm", arch=arch_name, seed=seed, generator="transformers.LlamaForCausalLM.generate "
                          f"(transformers {__import__('transformers').__version__}, bf16, CPU, sdpa)",
                          cases=stats, seconds=round(time.time() - t0, 1))
    print(name, json.dumps(stats))


# decisive greedy parity at the real vocabulary (synth.ChainSpec): TTS-1 dims, 16 layers,
# V = 193,856.  (utt, chain start, settings, group): "single" cases exercise the penalty /
# min-new / EOS / no-penalty paths at batch 1; the "batch" group shares settings so the
# GPU test can run its prompts (and copies of them) as 8..48 rows of one batch.
CHAIN_CASES = {
    "lm_chain": ("tts1", 0x5EED, [
        (0, 300, dict(new=500, min_new=500, rep=1.1), "single"),  # bench shape: 500 codes, EOS masked
        (1, 200, dict(new=300, min_new=100, rep=1.1), "single"),  # EOS unit 340 -> stops with EOS
        (2, 60, dict(new=120, min_new=120, rep=1.0), "single"),   # no penalty: lagged ids win
        (3, 700, dict(new=200, min_new=200, rep=1.4), "single"),  # CLI penalty
    ] + [(10 + r, 10 + 190 * r, dict(new=500, min_new=500, rep=1.1), "batch") for r in range(8)]),
    # TTS-1-Max (configs[3]'s model: 4096 wide, 32 layers, untied lm_head, head dim 128) at
    # full depth; the chain rows also go into the untied lm_head (synth.chain_overrides)
    "lm_chain_max": ("tts1-max", 0x5EED, [
        (0, 300, dict(new=200, min_new=200, rep=1.1), "single"),
        (1, 200, dict(new=200, min_new=100, rep=1.1), "single"),  # EOS unit 340 -> stops with EOS
        (2, 60, dict(new=120, min_new=120, rep=1.0), "single"),
        (3, 700, dict(new=200, min_new=200, rep=1.4), "single"),
    ] + [(10 + r, 10 + 190 * r, dict(new=200, min_new=200, rep=1.1), "batch") for r in range(8)]),
    # configs[3]'s length at full depth: 500 codes, EOS masked (the bench shape, rep 1.1)
    "lm_chain_max500": ("tts1-max", 0x5EED, [
        (0, 300, dict(new=500, min_new=500, rep=1.1), "single"),
    ]),
}


def chain_fixture(name: str, manifest: dict) -> None:
    arch_name, seed, cases = CHAIN_CASES[name]
    arch = configs.LM_ARCHS[arch_name]
    vocab = configs.vocab_for(arch)
    spec = synth.ChainSpec()
    t0 = time.time()
    w = synth.lm_weights_cpu(arch, seed)
    synth.apply_chain(w, arch, spec)
    model = hf_model(arch, w)  # (the oracle below shares w's bf16 storage: 2 copies in all)
    orc = lm_oracle.LlamaOracle(arch, w, max_seq_len=4096)
    eos = vocab.speech_end_id
    rec = dict(prompt_ids=[], prompt_lens=[], hf_new=[], hf_new_lens=[], hf_margins=[], hf_top2=[], max_length=[],
               min_new=[], rep=[], eos=[], group=[], start=[])
    stats = []
    for utt, start, st, group in cases:
        prompt = synth.chain_prompt(vocab, spec, utt, start, 30 + utt % 7, 120 + 3 * utt)
        P = len(prompt)
        new, margins, tops = hf_generate(model, prompt, P + st["new"], st["min_new"], eos, st["rep"])
        # the decision noise: HF vs the oracle, teacher-forced, on each step's top-2 logits
        seq = prompt + new
        n_tf = min(len(new), 24)
        with torch.no_grad():
            tf = model(torch.tensor([seq[:-1]])).logits[0, -n_tf:].float()
        o_tf = orc.score(seq[:-1], n_tf)
        top2 = torch.tensor(tops[-n_tf:])
        dev = (torch.gather(tf, 1, top2) - torch.gather(o_tf, 1, top2)).abs()
        stats.append(dict(utt=utt, start=start, group=group, P=P, n_new=len(new), ends_with_eos=new[-1] == eos,
                          hf_min_margin=min(margins), top2_dev_vs_oracle_max=float(dev.max()), **st))
        rec["prompt_ids"] += prompt
        rec["prompt_lens"].append(P)
        rec["hf_new"] += new
        rec["hf_new_lens"].append(len(new))
        rec["hf_margins"] += margins
        rec["hf_top2"] += tops
        rec["max_length"].append(P + st["new"])
        rec["min_new"].append(st["min_new"])
        rec["rep"].append(st["rep"])
        rec["eos"].append(eos)
        rec["group"].append(group)
        rec["start"].append(start)
        print(name, json.dumps(stats[-1]), flush=True)
    np.savez_compressed(os.path.join(GOLDEN, f"{name}.npz"), arch=arch_name, seed=seed,
                        chain=json.dumps(dataclasses.asdict(spec)), **{k: np.asarray(v) for k, v in rec.items()})
    manifest[name] = dict(kind="lm_chain", arch=arch_name, seed=seed, chain=dataclasses.asdict(spec),
                          generator="transformers.LlamaForCausalLM.generate "
                          f"(transformers {__import__('transformers').__version__}, bf16, CPU, sdpa) on the chain "
                          "model (synth.apply_chain)", cases=stats, seconds=round(time.time() - t0, 1))


# Teacher-forced logits through transformers' own DECODE path (prefill of a prefix, then one
# cached forward per token with DynamicCache: what GenerationMixin._sample runs,
# generation/utils.py:2783-2950) at the contexts the configs and the reference's defaults
# reach: TTS-1 up to max_tokens = 1,792 total positions (inferencing.py:21,
# tools/serving/inference.py:142), crossing the decode attention's 1,024-position pass at
# head dim 64; TTS-1-Max's dims (2 layers) at configs[3]'s ~700 positions, crossing the
# 512-position pass at head dim 128.  Sequences = a synthetic prompt + random speech ids
# (teacher forcing needs no greedy continuation).  Stored per decode step: HF's top-16 ids
# and 16 fixed random ids with their logits.
# (arch, seed, [(utt, total length)], n_last)
LONG_CASES = {
    "lm_tts1_long": ("tts1", 0x5EED, [(0, 1792), (1, 1664), (2, 1536), (3, 1408)], 1200),
    "lm_max2l_long": ("tts1-max-2l", 77, [(r, 760 - 20 * r) for r in range(8)], 560),
}


def hf_decode_logits(model, seq, n_last):
    """transformers' cached decode over the last n_last tokens of seq (fp32 copies of the
    bf16 logits, as _sample's `.float()`): [n_last, V]."""
    p0 = len(seq) - n_last
    out = []
    with torch.no_grad():
        r = model(torch.tensor([seq[:p0]]), use_cache=True, logits_to_keep=1)
        pkv = r.past_key_values
        for t in range(p0, len(seq)):
            r = model(torch.tensor([[seq[t]]]), past_key_values=pkv, use_cache=True)
            pkv = r.past_key_values
            out.append(r.logits[0, -1].float())
    return torch.stack(out)


def long_fixture(name: str, manifest: dict) -> None:
    arch_name, seed, seqs, n_last = LONG_CASES[name]
    arch = configs.LM_ARCHS[arch_name]
    vocab = configs.vocab_for(arch)
    t0 = time.time()
    w = synth.lm_weights_cpu(arch, seed)
    model = hf_model(arch, w)
    orc = lm_oracle.LlamaOracle(arch, w, max_seq_len=2048)
    rec = dict(ids=[], lens=[], tf_idx=[], tf_val=[])
    stats = []
    for utt, L in seqs:
        prompt = synth.synthetic_prompt(vocab, utt, 40, 150)
        rng = np.random.default_rng(4321 + utt)
        seq = prompt + [vocab.code_to_id(int(c)) for c in rng.integers(0, vocab.codebook_size, L - len(prompt))]
        tf = hf_decode_logits(model, seq, n_last)
        gen = torch.Generator().manual_seed(1000 + utt)
        idx = torch.cat([torch.topk(tf, 16, dim=-1).indices,
                         torch.randint(0, arch.vocab_size, (n_last, 16), generator=gen)], dim=1)
        val = torch.gather(tf, 1, idx)
        st = dict(utt=utt, L=L, n_last=n_last, first_pos=L - n_last, logit_absmax=float(tf.abs().max()))
        if utt == seqs[0][0]:  # the CPU oracle (prefill form) on the first sequence
            o = orc.score(seq, n_last)
            dev = (torch.gather(o, 1, idx) - val).abs()
            st.update(oracle_prefill_vs_hf_decode_max=float(dev.max()), oracle_prefill_vs_hf_decode_mean=float(dev.mean()))
        stats.append(st)
        rec["ids"] += seq
        rec["lens"].append(L)
        rec["tf_idx"].append(idx.numpy().astype(np.int32))
        rec["tf_val"].append(val.numpy().astype(np.float32))
        print(name, json.dumps(st), round(time.time() - t0), flush=True)
    np.savez_compressed(os.path.join(GOLDEN, f"{name}.npz"), arch=arch_name, seed=seed, n_last=n_last,
                        ids=np.asarray(rec["ids"], np.int32), lens=np.asarray(rec["lens"], np.int32),
                        tf_idx=np.stack(rec["tf_idx"]), tf_val=np.stack(rec["tf_val"]))
    manifest[name] = dict(kind="lm_decode_tf", arch=arch_name, seed=seed,
                          generator="transformers.LlamaForCausalLM cached decode (DynamicCache, one token per "
                          f"forward; transformers {__import__('transformers').__version__}, bf16, CPU, sdpa)",
                          cases=stats, seconds=round(time.time() - t0, 1))


# The synthesis composition (inferencing.py:110-159) executed by the reference's own
# `_synthesize_audio`: transformers' generate on the tiny LM, the reference codec loaded by
# its own `decoding.create` from a {"model": ...} checkpoint, a duck-typed tokenizer that
# hands over the prompt ids and names ids like the real one (<|s_N|>, other added tokens).
# (utt, n_text, n_prompt_codes, max_new, min_new, rep)
SYNTH_CASES = {"synth_tiny": ("tiny", 11, "codec-24k", 0xC0DEC,
                                 [(0, 12, 20, 40, 10, 1.1), (1, 5, 4, 24, 0, 1.4), (2, 30, 50, 48, 48, 1.0)])}


class _IdTokenizer:
    """The three tokenizer calls _synthesize_audio makes (inferencing.py:122,126,149)."""

    def __init__(self, vocab, prompt_ids):
        self.vocab, self.prompt_ids = vocab, prompt_ids

    def __call__(self, prompt, add_special_tokens=True, return_tensors="pt"):
        return {"input_ids": torch.tensor([self.prompt_ids])}

    def convert_tokens_to_ids(self, tok):
        assert tok == "<|speech_end|>"
        return self.vocab.speech_end_id

    def batch_decode(self, ids, skip_special_tokens=True):
        lut = self.vocab.id_to_code()
        return [f"<|s_{lut[int(i)]}|>" if lut[int(i)] >= 0 else f"<|tok_{int(i)}|>" for i in ids]


def synth_fixture(name: str, manifest: dict) -> None:
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "oracle", "shims"))
    sys.path.insert(0, "/root/reference")
    from tts.core.codec import decoding as ref_decoding
    from tts.inference import inferencing as ref_inferencing

    lm_arch_name, lm_seed, codec_name, codec_seed, cases = SYNTH_CASES[name]
    arch = configs.LM_ARCHS[lm_arch_name]
    carch = configs.CODEC_ARCHS[codec_name]
    vocab = configs.vocab_for(arch)
    t0 = time.time()
    model = hf_model(arch, synth.lm_weights_cpu(arch, lm_seed))
    cw = synth.codec_weights_cpu(carch, codec_seed)
    with tempfile.TemporaryDirectory() as td:
        with open(os.path.join(td, "model_config.json"), "w") as f:
            json.dump(carch.to_json_dict(), f)
        ck = os.path.join(td, "codec.pt")
        torch.save({"model": {"generator." + k: v for k, v in cw.items()}}, ck)
        dec = ref_decoding.create(ck, device="cpu")  # (the reference's strict checkpoint load)
    rec = dict(prompt_ids=[], prompt_lens=[], speech_ids=[], speech_lens=[], settings=[], wav=[], wav_lens=[])
    stats = []
    for utt, n_text, n_codes, new, min_new, rep in cases:
        prompt = synth.synthetic_prompt(vocab, utt, n_text, n_codes)
        lut = vocab.id_to_code()
        speech_ids = [int(lut[i]) for i in prompt[len(prompt) - n_codes:]] if n_codes else []
        st = ref_inferencing.InferenceSettings(temperature=0.0, max_tokens=len(prompt) + new, min_tokens=min_new,
                                               repetition_penalty=rep)
        wav, _ = ref_inferencing._synthesize_audio(model=model, tokenizer=_IdTokenizer(vocab, prompt),
                                                   audio_decoder=dec, speech_ids=speech_ids, prompt="",
                                                   model_device=torch.device("cpu"), inference_settings=st,
                                                   use_vllm=False)
        w = wav[0].numpy().astype(np.float32)
        stats.append(dict(utt=utt, P=len(prompt), n_prompt_codes=n_codes, L=int(w.size), rms=float(np.sqrt(np.mean(w ** 2)))))
        rec["prompt_ids"] += prompt
        rec["prompt_lens"].append(len(prompt))
        rec["speech_ids"] += speech_ids
        rec["speech_lens"].append(len(speech_ids))
        rec["settings"].append([new, min_new, rep])
        rec["wav"].append(w)
        rec["wav_lens"].append(int(w.size))
    rec["wav"] = np.concatenate(rec["wav"])
    np.savez_compressed(os.path.join(GOLDEN, f"{name}.npz"), lm_arch=lm_arch_name, lm_seed=lm_seed,
                        codec_arch=codec_name, codec_seed=codec_seed, **{k: np.asarray(v) for k, v in rec.items()})
    manifest[name] = dict(kind="synthesize_audio", lm_arch=lm_arch_name, codec_arch=codec_name,
                          generator="reference tts.inference.inferencing._synthesize_audio (transformers generate, "
                          "reference decoding.create + Decoder, oracle/shims incl. lightning/absl import shims)",
                          cases=stats, seconds=round(time.time() - t0, 1))
    print(name, json.dumps(stats))


# BASELINE configs[0] (tts_amd/config1.py): the 100 samples.jsonl utterances, RLHF pairing,
# each through the reference's own _synthesize_audio (tiny LM, depth-2 codec).  Stored: the
# generated ids (transformers' generate, recorded by a pass-through wrapper) and per-utterance
# waveform statistics (length, sum of squares, 64 samples at fixed positions).
CONFIG1_CASES = {"config1": ("tiny", 11, "codec-24k-d2", 0xC0DEC + 3)}


class _Recorder:
    """Passes model.generate through and keeps each call's output."""

    def __init__(self, model):
        self._m, self.calls = model, []

    def generate(self, *a, **kw):
        out = self._m.generate(*a, **kw)
        self.calls.append(out)
        return out

    def __getattr__(self, k):
        return getattr(self._m, k)


def config1_fixture(name: str, manifest: dict) -> None:
    sys.path.insert(0, os.path.join(ROOT, "oracle", "shims"))
    sys.path.insert(0, "/root/reference")
    from tts.core.codec import decoding as ref_decoding
    from tts.inference import inferencing as ref_inferencing

    from tts_amd import config1

    lm_arch_name, lm_seed, codec_name, codec_seed = CONFIG1_CASES[name]
    arch = configs.LM_ARCHS[lm_arch_name]
    carch = configs.CODEC_ARCHS[codec_name]
    vocab = configs.vocab_for(arch)
    t0 = time.time()
    model = _Recorder(hf_model(arch, synth.lm_weights_cpu(arch, lm_seed)))
    cw = synth.codec_weights_cpu(carch, codec_seed)
    # the reference's AudioDecoder (its decode() and rate properties) around the reference
    # Decoder reduced to the variant's depth (decoding.create always builds 12 blocks)
    from tts.core.codec import decoder as ref_decoder

    d = ref_decoder.Decoder(sample_rate=carch.sample_rate, hop_length=carch.hop_length,
                            upsample_factors=list(carch.upsample_factors) or None,
                            kernel_sizes=list(carch.kernel_sizes) or None)
    d.decoder.backbone.transformers = torch.nn.Sequential(*list(d.decoder.backbone.transformers)[: carch.depth])
    d.load_state_dict(cw, strict=True)
    d.eval()
    dec = ref_decoding.AudioDecoder.__new__(ref_decoding.AudioDecoder)
    dec._device, dec._decoder = "cpu", d
    dec._sample_rate, dec._token_rate = carch.sample_rate, carch.token_rate
    samples = config1.load_samples("/root/reference/example/configs/samples.jsonl")
    reqs = config1.requests(samples, vocab)
    rec = dict(new_ids=[], new_lens=[], wav_lens=[], wav_ss=[], wav_pick=[])
    for i, r in enumerate(reqs):
        P = len(r["prompt_ids"])
        st = ref_inferencing.InferenceSettings(temperature=0.0, max_tokens=P + r["n_new"], min_tokens=r["n_new"],
                                               repetition_penalty=1.1)
        wav, _ = ref_inferencing._synthesize_audio(model=model, tokenizer=_IdTokenizer(vocab, r["prompt_ids"]),
                                                   audio_decoder=dec, speech_ids=r["speech_ids"], prompt="",
                                                   model_device=torch.device("cpu"), inference_settings=st,
                                                   use_vllm=False)
        new = model.calls[-1][0, P:].tolist()
        w = wav[0].double().numpy()
        L = int(w.size)
        pick = np.linspace(0, max(L - 1, 0), 64).astype(np.int64) if L else np.zeros(64, np.int64)
        rec["new_ids"] += new
        rec["new_lens"].append(len(new))
        rec["wav_lens"].append(L)
        rec["wav_ss"].append(float((w ** 2).sum()))
        rec["wav_pick"].append(w[pick].astype(np.float32) if L else np.zeros(64, np.float32))
        if i % 10 == 0:
            print(name, i, P, len(new), L, flush=True)
    rec["wav_pick"] = np.stack(rec["wav_pick"])
    np.savez_compressed(os.path.join(GOLDEN, f"{name}.npz"), lm_arch=lm_arch_name, lm_seed=lm_seed,
                        codec_arch=codec_name, codec_seed=codec_seed, **{k: np.asarray(v) for k, v in rec.items()})
    manifest[name] = dict(kind="config1", lm_arch=lm_arch_name, codec_arch=codec_name, n=len(reqs),
                          total_new=int(sum(rec["new_lens"])), total_samples=int(sum(rec["wav_lens"])),
                          generator="reference tts.inference.inferencing._synthesize_audio per utterance "
                          "(transformers generate; the reference AudioDecoder.decode around the reference Decoder at "
                          "depth 2) on tts_amd.config1.requests (samples.jsonl, rlhf.py:56-67 pairing)",
                          seconds=round(time.time() - t0, 1))
    print(name, manifest[name])


def codec_fixture(name: str, manifest: dict) -> None:
    sys.path.insert(0, os.path.join(ROOT, "oracle", "shims"))
    sys.path.insert(0, "/root/reference")
    from tts.core.codec import decoder as ref_decoder  # the reference's own code

    arch_name, seed, lengths = CODEC_CASES[name]
    arch = configs.CODEC_ARCHS[arch_name]
    t0 = time.time()
    w = synth.codec_weights_cpu(arch, seed)
    d = ref_decoder.Decoder(sample_rate=arch.sample_rate, hop_length=arch.hop_length,
                            upsample_factors=list(arch.upsample_factors) or None,
                            kernel_sizes=list(arch.kernel_sizes) or None)
    if arch.depth != 12:  # reduced-depth test variant: same modules, fewer transformer blocks
        d.decoder.backbone.transformers = torch.nn.Sequential(*list(d.decoder.backbone.transformers)[: arch.depth])
    d.load_state_dict(w, strict=True)
    d.eval()
    rng = np.random.default_rng(seed)
    rec = dict(codes=[], lens=[], wav=[], wav_lens=[])
    stats = []
    for T in lengths:
        codes = rng.integers(0, 65536, size=T)
        with torch.no_grad():
            ref = d(torch.tensor(codes)[None, None]).squeeze(0)  # AudioDecoder.decode: [1, L]
            orc = codec_oracle.decode(w, torch.tensor(codes), arch.hop_length, arch.upsample_factors,
                                      arch.kernel_sizes, arch.depth)
        r = ref[0].numpy()
        o = orc[0].numpy()
        rel = float(np.linalg.norm(r - o) / max(np.linalg.norm(r), 1e-30))
        stats.append(dict(T=int(T), L=int(r.size), oracle_rel_l2=rel, rms=float(np.sqrt(np.mean(r ** 2)))))
        rec["codes"] += codes.tolist()
        rec["lens"].append(int(T))
        rec["wav"].append(r.astype(np.float32))
        rec["wav_lens"].append(int(r.size))
    np.savez_compressed(os.path.join(GOLDEN, f"{name}.npz"), arch=arch_name, seed=seed,
                        codes=np.asarray(rec["codes"], dtype=np.int32), lens=np.asarray(rec["lens"]),
                        wav=np.concatenate(rec["wav"]), wav_lens=np.asarray(rec["wav_lens"]))
    manifest[name] = dict(kind="codec", arch=arch_name, seed=seed,
                          generator="reference tts.core.codec.decoder.Decoder (fp32, CPU) + oracle/shims",
                          cases=stats, seconds=round(time.time() - t0, 1))
    print(name, json.dumps(stats))


# The prompt-audio encoder (§8f rank 1): the reference's own Encoder.encode
# (tts/core/codec/encoder.py:115-128) on synthetic weights.  Its __init__ loads the
# feature extractor and w2v-bert-2.0 from the hub, so the object is assembled here with the
# same modules (encoder.py:20-56) and transformers' SeamlessM4TFeatureExtractor /
# Wav2Vec2BertModel from a local config (configs.EncoderArch: the hub dimensions, parity of
# those dimensions unpinned).  (seed, [(wav seed, samples)])
ENCODER_CASES = {"encoder_16k": (0xE2C0, [(0, 8000), (1, 20800), (2, 48123)])}


def build_reference_encoder(arch, seed):
    """The reference Encoder object with synthetic weights (no hub access)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle", "shims"))
    sys.path.insert(0, "/root/reference")
    import transformers
    import vector_quantize_pytorch as vq  # the shim (vector_quantize_pytorch 1.17.8 restated)
    from tts.core.codec import encoder as ref_encoder, encoder_modules  # the reference's own code

    enc = ref_encoder.Encoder.__new__(ref_encoder.Encoder)
    torch.nn.Module.__init__(enc)
    enc.sample_rate, enc.token_rate = arch.sample_rate, arch.token_rate
    enc.semantic_encoder = encoder_modules.SemanticEncoder(input_channels=1024, output_channels=1024,
                                                           encode_channels=1024, kernel_size=3)
    enc.acoustic_encoder = encoder_modules.AcousticEncoder(
        num_generator_features=arch.ngf, initial_conv_kernel_size=7, final_conv_kernel_size=3,
        up_ratios=list(arch.up_ratios), dilations=tuple(arch.dilations), output_dim=arch.acoustic_dim)
    enc.fusion_layer = torch.nn.Linear(2048, 2048)
    enc.quantizer = vq.ResidualFSQ(dim=2048, levels=list(arch.levels), num_quantizers=1)
    w = synth.weights_from_specs_cpu(synth.encoder_tensor_specs(arch), seed)
    missing, unexpected = enc.load_state_dict(w, strict=False)
    assert not unexpected, unexpected
    assert all(m.endswith("filter") for m in missing), missing  # the anti-aliasing buffers
    enc.wav2vec_feature_extractor = transformers.SeamlessM4TFeatureExtractor(padding_value=1.0)
    cfg = transformers.Wav2Vec2BertConfig(**arch.w2v_hf_config())
    enc.wav2vec_model = transformers.Wav2Vec2BertModel(cfg)
    enc.wav2vec_model.config.output_hidden_states = True
    enc.wav2vec_model.load_state_dict(synth.weights_from_specs_cpu(synth.w2v_tensor_specs(arch), seed + 1),
                                      strict=True)
    enc.eval()
    return enc


def encoder_fixture(name: str, manifest: dict) -> None:
    arch = configs.ENCODER
    seed, cases = ENCODER_CASES[name]
    t0 = time.time()
    enc = build_reference_encoder(arch, seed)
    filt = enc.acoustic_encoder.conv_final_block[0]
    up_f, dn_f = filt.upsample.filter.flatten(), filt.downsample.lowpass.filter.flatten()
    assert torch.equal(up_f, synth.kaiser_sinc_filter(0.25, 0.3, 12))
    assert torch.equal(dn_f, synth.kaiser_sinc_filter(0.25, 0.3, 12))
    rec = dict(wav=[], wav_lens=[], feats=[], w2v=[], acoustic=[], pre_round=[], codes=[], T=[])
    stats = []
    hooks = {}
    enc.acoustic_encoder.register_forward_hook(lambda m, i, o: hooks.__setitem__("acoustic", o.detach()))
    enc.quantizer.layers[0].register_forward_hook(lambda m, i, o: hooks.__setitem__("fsq_in", i[0].detach()))
    for ws, n in cases:
        wav = torch.from_numpy(synth.synthetic_wav(ws, n))[None]
        with torch.no_grad():
            codes = enc.encode(wav)  # the reference call (encoding.py:67-72 -> encoder.py:115-128)
            # the intermediate tensors of the same call, recomputed for the fixture
            audio = torch.nn.functional.pad(wav, (0, 320 - (wav.shape[1] % 320)))
            audio_pad = torch.nn.functional.pad(audio, (160, 160))
            feat = enc.wav2vec_feature_extractor(audio_pad, sampling_rate=16000,
                                                 return_tensors="pt").data["input_features"]
            w2v = enc.wav2vec_model(feat).hidden_states[16]
        codes = codes.reshape(-1).numpy().astype(np.int32)
        T = codes.size
        fsq_in = hooks["fsq_in"].reshape(T, -1).float()  # the FSQ layer's input = bound(project_in(x))
        lv = torch.tensor(arch.levels, dtype=torch.float32)
        pre = enc.quantizer.layers[0].bound(fsq_in)  # the value torch.round sees
        stats.append(dict(samples=n, T=int(T), feats=list(feat.shape), w2v_rms=float(w2v.pow(2).mean().sqrt()),
                          acoustic_rms=float(hooks["acoustic"].pow(2).mean().sqrt()),
                          min_round_margin=float((pre - pre.round()).abs().sub(0.5).abs().min()),
                          distinct_codes=int(len(set(codes.tolist())))))
        rec["wav"].append(wav[0].numpy())
        rec["wav_lens"].append(n)
        rec["feats"].append(feat[0].numpy().astype(np.float32))
        rec["w2v"].append(w2v[0].numpy().astype(np.float32))
        rec["acoustic"].append(hooks["acoustic"][0].numpy().astype(np.float32))
        rec["pre_round"].append(pre.numpy().astype(np.float32))
        rec["codes"].append(codes)
        rec["T"].append(int(T))
        print(name, json.dumps(stats[-1]), flush=True)
        del lv
    np.savez_compressed(os.path.join(GOLDEN, f"{name}.npz"), seed=seed,
                        **{k: (np.concatenate(v) if k not in ("wav_lens", "T") else np.asarray(v))
                           for k, v in rec.items()})
    manifest[name] = dict(kind="encoder", arch=arch.name, seed=seed,
                          generator="reference tts.core.codec.encoder.Encoder.encode (fp32, CPU) + oracle/shims; "
                          f"transformers {__import__('transformers').__version__} SeamlessM4TFeatureExtractor / "
                          "Wav2Vec2BertModel from a local config (w2v-bert-2.0 dims: parity unpinned)",
                          cases=stats, seconds=round(time.time() - t0, 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    args = ap.parse_args()
    os.makedirs(GOLDEN, exist_ok=True)
    mpath = os.path.join(GOLDEN, "manifest.json")
    manifest = json.load(open(mpath)) if os.path.exists(mpath) else {}
    torch.manual_seed(0)
    names = args.only or (list(LM_CASES) + list(CHAIN_CASES) + list(LONG_CASES) + list(SYNTH_CASES) +
                          list(CONFIG1_CASES) + list(CODEC_CASES) + list(ENCODER_CASES))
    for n in names:
        fn = (lm_fixture if n in LM_CASES else chain_fixture if n in CHAIN_CASES else
              long_fixture if n in LONG_CASES else
              synth_fixture if n in SYNTH_CASES else config1_fixture if n in CONFIG1_CASES else
              encoder_fixture if n in ENCODER_CASES else codec_fixture)
        fn(n, manifest)
        with open(mpath, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
