"""Decisive greedy-id parity at the real vocabulary (V = 193,856, TTS-1 dims, 16 layers).

The fixture tests/golden/lm_chain.npz holds transformers' own LlamaForCausalLM.generate
(the call of tts/inference/inferencing.py:94-107; transformers generation/utils.py
_sample) on the chain model (tts_amd.synth.ChainSpec: random TTS-1 weights with a few rows
overwritten by exact values).  On it every step is decided by a margin of >= 7.8 logits
(HF min margin, tests/golden/manifest.json) against a teacher-forced HF-vs-oracle deviation
of <= 1 logit on the top-2 tokens, and by the greedy head's semantics:

* repetition penalty over the prompt + generated ids (the lagged, already-seen chain id
  has the larger raw logit and loses only when penalised: rep 1.1 and 1.4 cases; with
  rep 1.0 it wins and the sequence cycles),
* min_new_tokens masking EOS (EOS units inside the masked range) and the EOS stop,
* max_length counting the prompt.

So the bar has no margin escape hatch: a single differing id over 500 steps fails.  Runs
through the C ABI: the HF-form generate surface at batch 1, the graph-captured batched
decode at 8 / 32 / 48 rows (copies of 8 distinct prompts at different chain offsets,
17..32-row and 33..64-row plans) and the streaming loop.
"""

import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _cases():
    z = np.load(os.path.join(GOLDEN, "lm_chain.npz"))
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
                                               max_batch=48, max_seq_len=1024)
    return _model["m"]


def test_fixture_is_decisive():
    """The fixture itself: every HF step's margin is far above the implementation noise."""
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))["lm_chain"]
    for c in man["cases"]:
        assert c["hf_min_margin"] >= 4 * max(c["top2_dev_vs_oracle_max"], 1.0), c


@pytest.mark.parametrize("idx", [0, 1, 2, 3])
def test_chain_single_hf_surface(idx):
    """HF-form generate (the reference's call shape): prompt + every new id, EOS included."""
    _, _, _, cases = _cases()
    c = cases[idx]
    m = _lm()
    out = m.generate(input_ids=torch.tensor([c["prompt"]]), max_length=c["max_length"],
                     min_new_tokens=c["min_new"], eos_token_id=c["eos"], do_sample=False,
                     repetition_penalty=c["rep"], top_p=1.0, temperature=0.0)
    new = out[0, len(c["prompt"]):].tolist()
    assert new == c["hf_new"], next(i for i, (a, b) in enumerate(zip(new + [-9], c["hf_new"] + [-8])) if a != b)


@pytest.mark.parametrize("rows", [8, 32, 48])
def test_chain_batched_rows(rows):
    """The graph-captured batched decode: row r runs prompt r % 8 of the batch group; every
    row equals transformers' batch-1 sequence for its prompt, all 500 ids."""
    _, _, _, cases = _cases()
    grp = [c for c in cases if c["group"] == "batch"]
    assert len(grp) == 8 and len({(c["rep"], c["min_new"], c["max_length"] - len(c["prompt"])) for c in grp}) == 1
    m = _lm()
    prompts = [grp[r % 8]["prompt"] for r in range(rows)]
    new_n = grp[0]["max_length"] - len(grp[0]["prompt"])
    # one max_length for the batch: each row's own limit is max_length - its prompt length,
    # so pass per-row-equal new-token counts by padding max_length to the longest prompt and
    # checking the first new_n ids (min_new = new_n keeps every row running that long)
    L = max(len(p) for p in prompts) + new_n
    outs = m.generate_batch(prompts, max_length=L, min_new_tokens=new_n, eos_token_id=grp[0]["eos"],
                            repetition_penalty=grp[0]["rep"])
    for r, o in enumerate(outs):
        ref = grp[r % 8]["hf_new"]
        assert o[:new_n] == ref, (r, next(i for i, (a, b) in enumerate(zip(o, ref)) if a != b))


def test_chain_streaming_equals_hf():
    """Config 5's chunked loop (generate_stream, chunks of 25) ends with the same ids."""
    _, _, _, cases = _cases()
    grp = [c for c in cases if c["group"] == "batch"]
    m = _lm()
    prompts = [c["prompt"] for c in grp]
    new_n = grp[0]["max_length"] - len(grp[0]["prompt"])
    L = max(len(p) for p in prompts) + new_n
    final = None
    for new, done in m.generate_stream(prompts, max_length=L, chunk=25, min_new_tokens=new_n,
                                       eos_token_id=grp[0]["eos"], repetition_penalty=grp[0]["rep"]):
        final = new
    for c, o in zip(grp, final):
        assert o[:new_n] == c["hf_new"]


def test_chain_continuous_batching_equals_hf():
    """SURVEY §8f rank 3 (vLLM LLM.generate / continuous batching, tts_slots_*): the 8 batch
    prompts go through 3 persistent decode rows (requests admitted between 16-step chunks as
    rows free up), and through the vLLM-shaped LLM facade; every request's ids equal
    transformers' for its prompt, all 500 of them."""
    from tts_amd.serving import LLM, ContinuousBatcher

    _, _, _, cases = _cases()
    grp = [c for c in cases if c["group"] == "batch"]
    m = _lm()
    new_n = grp[0]["max_length"] - len(grp[0]["prompt"])
    b = ContinuousBatcher(m, n_slots=3, eos_token_id=grp[0]["eos"], min_new_tokens=grp[0]["min_new"],
                          repetition_penalty=grp[0]["rep"], chunk=16)
    got = b.generate([c["prompt"] for c in grp], [new_n] * len(grp))
    for c, o in zip(grp, got):
        assert o[:new_n] == c["hf_new"][:new_n], next(i for i, (x, y) in enumerate(zip(o, c["hf_new"])) if x != y)

    class SP:  # vllm.SamplingParams fields the reference sets (inferencing.py:75-92)
        max_tokens = new_n
        min_tokens = grp[0]["min_new"]
        stop_token_ids = [grp[0]["eos"]]
        repetition_penalty = grp[0]["rep"]
        temperature = 0.0

    outs = LLM(m, n_slots=4, chunk=16).generate(prompt_token_ids=[c["prompt"] for c in grp[:5]], sampling_params=SP())
    for c, o in zip(grp[:5], outs):
        assert list(o.outputs[0].token_ids)[:new_n] == c["hf_new"][:new_n]
