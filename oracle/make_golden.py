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
}


def lm_fixture(name: str, manifest: dict) -> None:
    from transformers import LlamaConfig, LlamaForCausalLM

    arch_name, seed, prompts, settings = LM_CASES[name]
    arch = configs.LM_ARCHS[arch_name]
    vocab = configs.vocab_for(arch)
    t0 = time.time()
    w = synth.lm_weights_cpu(arch, seed)
    cfg = LlamaConfig(**arch.hf_config_dict())
    with torch.device("meta"):
        model = LlamaForCausalLM(cfg)
    model = model.to_empty(device="cpu").to(torch.bfloat16)
    sd = dict(w)
    if arch.tie_word_embeddings:
        sd["lm_head.weight"] = w["model.embed_tokens.weight"]
    missing, unexpected = model.load_state_dict(sd, strict=False)
    missing = [m for m in missing if "rotary_emb" not in m]
    assert not missing and not unexpected, (missing, unexpected)
    model.model.rotary_emb = type(model.model.rotary_emb)(cfg)  # buffers were on meta
    model.eval()
    orc = lm_oracle.LlamaOracle(arch, w, max_seq_len=4096)
    eos = vocab.speech_end_id
    rec = dict(prompt_ids=[], prompt_lens=[], hf_new=[], hf_new_lens=[], oracle_new=[], oracle_lens=[],
               oracle_margins=[], max_length=[], min_new=[], rep=[], eos=[])
    stats = []
    for (utt, n_text, n_codes), st in zip(prompts, settings):
        prompt = synth.synthetic_prompt(vocab, utt, n_text, n_codes)
        P = len(prompt)
        max_length = P + st["new"]
        with torch.no_grad():
            out = model.generate(input_ids=torch.tensor([prompt]), max_length=max_length,
                                 min_new_tokens=st["min_new"], eos_token_id=eos, do_sample=False,
                                 repetition_penalty=st["rep"], top_p=1.0, temperature=0.0,
                                 output_scores=True, return_dict_in_generate=True)
        hf_new = out.sequences[0, P:].tolist()
        hf_margins = []
        for sc in out.scores:  # processed scores (penalty + min-new mask) of each step
            top = torch.topk(sc[0].float(), 2).values
            hf_margins.append(float(top[0] - top[1]))
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
        stats.append(dict(P=P, n_new=len(hf_new), agree_prefix=agree, identical=hf_new == o_new,
                          min_margin=min(margins), hf_min_margin=min(hf_margins),
                          first_hf_near_tie=next((i for i, m in enumerate(hf_margins) if m < 0.25), None),
                          max_abs_logit_diff=diff,
                          logit_scale=hf_logits.abs().max().item()))
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
    np.savez_compressed(os.path.join(GOLDEN, f"{name}.npz"), arch=arch_name, seed=seed,
                        **{k: np.asarray(v) for k, v in rec.items()})
    manifest[name] = dict(kind="lm", arch=arch_name, seed=seed, generator="transformers.LlamaForCausalLM.generate "
                          f"(transformers {__import__('transformers').__version__}, bf16, CPU, sdpa)",
                          cases=stats, seconds=round(time.time() - t0, 1))
    print(name, json.dumps(stats))


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    args = ap.parse_args()
    os.makedirs(GOLDEN, exist_ok=True)
    mpath = os.path.join(GOLDEN, "manifest.json")
    manifest = json.load(open(mpath)) if os.path.exists(mpath) else {}
    torch.manual_seed(0)
    names = args.only or (list(LM_CASES) + list(CODEC_CASES))
    for n in names:
        (lm_fixture if n in LM_CASES else codec_fixture)(n, manifest)
        with open(mpath, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
