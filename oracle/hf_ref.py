"""transformers' LlamaForCausalLM holding the synthetic weights, and the reference's greedy
generate call — TEST INFRASTRUCTURE (the golden-fixture generator oracle/make_golden.py and
bench.py's cpu_baseline leg use it; nothing in the product path imports oracle/).

The SpeechLM arithmetic of the reference is transformers' LlamaForCausalLM +
GenerationMixin (the reference pins transformers 4.53.2, uv.lock:4610-4611; the
installed 5.15.0 restates the same processors); the call shape is
tts/inference/inferencing.py:94-107.
"""

from __future__ import annotations

import torch


def hf_model(arch, w):
    """transformers LlamaForCausalLM (bf16, CPU) holding the synthetic weights `w`."""
    from transformers import LlamaConfig, LlamaForCausalLM

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
    return model


def hf_generate(model, prompt, max_length, min_new, eos, rep):
    """The reference call (inferencing.py:94-107, greedy) -> (new ids, per-step top-2 margins
    of the processed scores, per-step (top1, top2) ids)."""
    with torch.no_grad():
        out = model.generate(input_ids=torch.tensor([prompt]), max_length=max_length, min_new_tokens=min_new,
                             eos_token_id=eos, do_sample=False, repetition_penalty=rep, top_p=1.0,
                             temperature=0.0, output_scores=True, return_dict_in_generate=True)
    new = out.sequences[0, len(prompt):].tolist()
    margins, tops = [], []
    for sc in out.scores:  # processed scores (penalty + min-new mask) of each step
        top = torch.topk(sc[0].float(), 2)
        margins.append(float(top.values[0] - top.values[1]))
        tops.append([int(i) for i in top.indices])
    return new, margins, tops
