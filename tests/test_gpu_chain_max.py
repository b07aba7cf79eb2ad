"""Decisive greedy-id parity for TTS-1-Max at full depth (configs[3]'s model: hidden 4096,
32 layers, head dim 128, untied lm_head, V = 193,856) against transformers.

tests/golden/lm_chain_max.npz holds transformers' own LlamaForCausalLM.generate (the call
of tts/inference/inferencing.py:94-107) on the chain model (tts_amd.synth.ChainSpec; the
chain rows also written into the untied lm_head), made in the build container by
oracle/make_golden.py --only lm_chain_max.  Each step is decided by a margin far above the
implementation noise (the manifest's hf_min_margin against top2_dev_vs_oracle_max), so a
single differing id fails.  Runs the HF-form surface at batch 1 and the graph-captured
batched decode at 8 rows (configs[3]'s per-GPU shard: 64 prompts over 8 GPUs) and 24 rows.
tests/golden/lm_chain_max500.npz (oracle/make_golden.py --only lm_chain_max500) holds one
500-id sequence, configs[3]'s length (prompt 170 + 500 codes, EOS masked, penalty 1.1).
"""

import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURE = os.path.join(GOLDEN, "lm_chain_max.npz")
FIXTURE500 = os.path.join(GOLDEN, "lm_chain_max500.npz")


def _cases(path=FIXTURE):
    z = np.load(path)
    out, po, no = [], 0, 0
    for i, P in enumerate(z["prompt_lens"]):
        n = int(z["hf_new_lens"][i])
        out.append(dict(prompt=z["prompt_ids"][po:po + P].tolist(), hf_new=z["hf_new"][no:no + n].tolist(),
                        max_length=int(z["max_length"][i]), min_new=int(z["min_new"][i]), rep=float(z["rep"][i]),
                        eos=int(z["eos"][i]), group=str(z["group"][i])))
        po += P
        no += n
    return str(z["arch"]), int(z["seed"]), json.loads(str(z["chain"])), out


_model = {}


def _lm():
    from tts_amd import configs, synth
    from tts_amd.speechlm import MI355XSpeechLM

    if "m" not in _model:
        arch_name, seed, spec, _ = _cases()
        _model["m"] = MI355XSpeechLM.synthetic(configs.LM_ARCHS[arch_name], seed=seed, chain=synth.ChainSpec(**spec),
                                               max_batch=24, max_seq_len=720)
    return _model["m"]


def test_fixture_is_decisive():
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))["lm_chain_max"]
    assert man["arch"] == "tts1-max"
    for c in man["cases"]:
        assert c["hf_min_margin"] >= 4 * max(c["top2_dev_vs_oracle_max"], 1.0), c


@pytest.mark.parametrize("idx", [0, 1, 2, 3])
def test_max_chain_single_hf_surface(idx):
    _, _, _, cases = _cases()
    c = cases[idx]
    m = _lm()
    out = m.generate(input_ids=torch.tensor([c["prompt"]]), max_length=c["max_length"],
                     min_new_tokens=c["min_new"], eos_token_id=c["eos"], do_sample=False,
                     repetition_penalty=c["rep"], top_p=1.0, temperature=0.0)
    new = out[0, len(c["prompt"]):].tolist()
    assert new == c["hf_new"], next(i for i, (a, b) in enumerate(zip(new + [-9], c["hf_new"] + [-8])) if a != b)


@pytest.mark.parametrize("rows", [8, 24])
def test_max_chain_batched_rows(rows):
    """Row r runs prompt r % 8 of the batch group; every row equals transformers' batch-1
    sequence for its prompt, all 200 ids."""
    _, _, _, cases = _cases()
    grp = [c for c in cases if c["group"] == "batch"]
    assert len(grp) == 8
    m = _lm()
    prompts = [grp[r % 8]["prompt"] for r in range(rows)]
    new_n = grp[0]["max_length"] - len(grp[0]["prompt"])
    L = max(len(p) for p in prompts) + new_n
    outs = m.generate_batch(prompts, max_length=L, min_new_tokens=new_n, eos_token_id=grp[0]["eos"],
                            repetition_penalty=grp[0]["rep"])
    for r, o in enumerate(outs):
        ref = grp[r % 8]["hf_new"]
        assert o[:new_n] == ref, (r, next(i for i, (a, b) in enumerate(zip(o, ref)) if a != b))


def test_max_chain_500_codes():
    """configs[3]'s length at full depth: transformers' 500 ids for the bench-shaped case, id
    for id, through the HF-form surface and as 8 copies in the graph-captured decode (the
    per-GPU shard's row count)."""
    arch, seed, spec, cases = _cases(FIXTURE500)
    assert (arch, seed, spec) == _cases()[:3]  # (the model of the other chain tests)
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))["lm_chain_max500"]
    c, mc = cases[0], man["cases"][0]
    assert len(c["hf_new"]) == 500 and mc["hf_min_margin"] >= 4 * max(mc["top2_dev_vs_oracle_max"], 1.0), mc
    m = _lm()
    out = m.generate(input_ids=torch.tensor([c["prompt"]]), max_length=c["max_length"],
                     min_new_tokens=c["min_new"], eos_token_id=c["eos"], do_sample=False,
                     repetition_penalty=c["rep"], top_p=1.0, temperature=0.0)
    new = out[0, len(c["prompt"]):].tolist()
    assert new == c["hf_new"], next(i for i, (a, b) in enumerate(zip(new + [-9], c["hf_new"] + [-8])) if a != b)
    outs = m.generate_batch([c["prompt"]] * 8, max_length=c["max_length"], min_new_tokens=c["min_new"],
                            eos_token_id=c["eos"], repetition_penalty=c["rep"])
    for r, o in enumerate(outs):
        assert o[:500] == c["hf_new"], (r, next(i for i, (a, b) in enumerate(zip(o, c["hf_new"])) if a != b))
