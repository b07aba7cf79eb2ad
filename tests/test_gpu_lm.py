"""SpeechLM end-to-end parity on the GPU (through the C ABI) against:

* the golden fixtures produced by transformers' LlamaForCausalLM.generate itself
  (oracle/make_golden.py; tests/golden/lm_*.npz) — greedy token ids, bit-exact;
* the CPU oracle (oracle/lm_oracle.py) for teacher-forced logits (bf16, to a tolerance of
  a few bf16 ulps of the logit scale: different fp32 summation orders round a few
  intermediate bf16 values differently).

Exactness contract: greedy ids must equal the reference's wherever the
reference's top-1/top-2 margin exceeds the logit tolerance; every golden case in the suite
has all margins above it, so the whole sequences must match.
"""

import os

import numpy as np
import pytest
import torch

from oracle import lm_oracle

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# engine-vs-transformers bar of test_tts1_teacher_forced_logits_vs_transformers
# 1.25x the measured 0.375 / 0.0791 (profiles/r3q_tts1_tf_logit_dev.json, r4a_tts1_tf_logit_dev.json)
TF_MAX, TF_MEAN = 0.47, 0.099
# absolute, on logits of magnitude ~1-20.  The oracle (torch CPU) and the GPU sum the fp32
# dot products in different orders (split-K trees chosen per matrix by the stream plan), so
# bf16 activations differ by an ulp here and there and the difference compounds over the
# layers: measured max 0.066 (lm_small, split-K 4 gate/up) — argmax agreement is exact.
LOGIT_TOL = 0.1


def _cases(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    out, po, no = [], 0, 0
    for i, P in enumerate(z["prompt_lens"]):
        n = int(z["hf_new_lens"][i])
        out.append(dict(prompt=z["prompt_ids"][po:po + P].tolist(), hf_new=z["hf_new"][no:no + n].tolist(),
                        hf_margins=z["hf_margins"][no:no + n].tolist(),
                        max_length=int(z["max_length"][i]), min_new=int(z["min_new"][i]), rep=float(z["rep"][i]),
                        eos=int(z["eos"][i])))
        po += P
        no += n
    return str(z["arch"]), int(z["seed"]), out


_models = {}


def _model(arch_name, seed, max_batch=4):
    from tts_amd import configs
    from tts_amd.speechlm import MI355XSpeechLM

    key = (arch_name, seed, max_batch)
    if key not in _models:
        for k in list(_models):
            _models.pop(k).close()
        _models[key] = MI355XSpeechLM.synthetic(configs.LM_ARCHS[arch_name], seed=seed, max_batch=max_batch,
                                                max_seq_len=1024)
    return _models[key]


MARGIN_TOL = 0.25  # reference top1-top2 margin below which the choice is backend noise


def _margin_tol(name, case):
    """A choice is decidable when the reference's margin exceeds twice the logit deviation
    two valid implementations show on it (manifest: transformers vs the CPU oracle,
    teacher-forced), plus one bf16 ulp; never below MARGIN_TOL."""
    import json

    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))[name]
    dev = max(c["max_abs_logit_diff"] for c in man["cases"])
    return max(MARGIN_TOL, 2.0 * dev + 0.125)


def _process(logits, seen, rep, new_len, min_new, eos):
    return lm_oracle.LlamaOracle.process(logits, seen, rep, new_len, min_new, eos)


@pytest.mark.parametrize("name", ["lm_tiny", "lm_small", "lm_tiny128", "lm_tts1"])
def test_greedy_ids_match_reference(name):
    """Free-running greedy ids equal the reference's up to its first near-tie step (all of
    the sequence for every case without one), and teacher-forced on the reference's own
    sequence the engine picks the reference's token at every step whose margin clears
    MARGIN_TOL.  For the small configs that is the whole sequence.  On random TTS-1 weights
    (lm_tts1) bf16 ties and near-ties occur from step 1 (V = 193,856, logits quantised to
    bf16), so this case is NOT decisive; the decisive full-vocabulary bar (500 ids, no
    margin escape) is tests/test_gpu_chain.py, and the raw TTS-1 logits are compared with
    transformers directly in test_tts1_teacher_forced_logits_vs_transformers."""
    arch, seed, cases = _cases(name)
    m = _model(arch, seed)
    for c in cases:
        out = m.generate(input_ids=torch.tensor([c["prompt"]]), max_length=c["max_length"],
                         min_new_tokens=c["min_new"], eos_token_id=c["eos"], do_sample=False,
                         repetition_penalty=c["rep"], top_p=1.0, temperature=0.0)
        new = out[0, len(c["prompt"]):].tolist()
        ref = c["hf_new"]
        hm = c["hf_margins"]
        tol = _margin_tol(name, c)
        k = next((i for i, x in enumerate(hm) if x < tol), len(ref))
        assert new[:k] == ref[:k], (name, k, new, ref)
        if k == len(ref):
            assert new == ref
        # teacher forcing over the whole reference sequence
        seq = c["prompt"] + ref
        lg = m.score([seq], len(ref) + 1)[0]
        P = len(c["prompt"])
        for i in range(len(ref)):
            sc = _process(lg[i], seq[:P + i], c["rep"], i, c["min_new"], c["eos"])
            if hm[i] >= tol:
                assert int(torch.argmax(sc)) == ref[i], (name, i, hm[i], tol)


@pytest.mark.parametrize("name", ["lm_tiny", "lm_small", "lm_tiny128"])
def test_teacher_forced_logits_vs_oracle(name):
    from tts_amd import configs, synth

    arch, seed, cases = _cases(name)
    m = _model(arch, seed)
    orc = lm_oracle.LlamaOracle(configs.LM_ARCHS[arch], synth.lm_weights_cpu(configs.LM_ARCHS[arch], seed))
    for c in cases:
        seq = c["prompt"] + c["hf_new"]
        got = m.score([seq], 6)[0]
        ref = orc.score(seq, 6)
        assert (got - ref).abs().max().item() <= LOGIT_TOL
        assert torch.equal(got.argmax(-1), ref.argmax(-1))


def test_batch_is_independent_sequences():
    """Ragged batch: each sequence equals its batch-1 result (no padding in the arithmetic)."""
    arch, seed, cases = _cases("lm_tiny")
    m = _model(arch, seed)
    L = max(len(c["prompt"]) for c in cases) + 20
    singles = [m.generate_batch([c["prompt"]], max_length=len(c["prompt"]) + 20, min_new_tokens=5, eos_token_id=-1,
                                repetition_penalty=1.1)[0] for c in cases]
    batch = m.generate_batch([c["prompt"] for c in cases], max_length=L, min_new_tokens=5, eos_token_id=-1,
                             repetition_penalty=1.1)
    for s, b, c in zip(singles, batch, cases):
        assert b[:len(s)] == s


def test_stop_rules():
    """EOS stops (and is returned); max_length counts the prompt; min_new masks EOS."""
    arch, seed, cases = _cases("lm_tiny")
    m = _model(arch, seed)
    c = cases[1]
    ref = c["hf_new"]
    # make the 3rd generated token the EOS: generation must stop right after it
    eos = ref[2]
    first = ref.index(eos)
    new = m.generate_batch([c["prompt"]], max_length=len(c["prompt"]) + 30, min_new_tokens=0, eos_token_id=eos,
                           repetition_penalty=c["rep"])[0]
    assert new == ref[:first + 1]
    # with min_new_tokens > 3 the EOS is masked at step 3 -> sequence differs from ref there
    new2 = m.generate_batch([c["prompt"]], max_length=len(c["prompt"]) + 6, min_new_tokens=6, eos_token_id=eos,
                            repetition_penalty=c["rep"])[0]
    assert len(new2) == 6 and eos not in new2[:6]
    with pytest.raises(ValueError):
        m.generate(input_ids=torch.tensor([c["prompt"]]), max_length=len(c["prompt"]))
    # single-token prompt
    one = m.generate_batch([[c["prompt"][0]]], max_length=5, eos_token_id=-1)[0]
    assert len(one) == 4


def test_vllm_form_and_codes_lut():
    arch, seed, cases = _cases("lm_tiny")
    m = _model(arch, seed)
    c = cases[0]

    class SP:
        max_tokens = 10
        min_tokens = 10
        stop_token_ids = [c["eos"]]
        repetition_penalty = c["rep"]
        temperature = 0.0

    out = m.generate(prompt_token_ids=c["prompt"], sampling_params=SP())
    assert out[0].outputs[0].token_ids == c["hf_new"][:10]
    codes = m.ids_to_codes([256, 257, 5, 204])
    assert codes == [0, 1, -1, -1]


@pytest.mark.parametrize("rows", [24, 32, 48])
def test_batched_decode_tts1_dims(rows):
    """Batched decode at TTS-1 dims (config 3's shape class): 17..32 rows take the two-m-tile
    GEMMs with the A rows in LDS and the K-sliced down projection (fp32 chunk partials +
    combine kernel); 33..64 rows run as two 32-row launches.  Every row is a copy of a golden case, so every row must reproduce the
    reference ids up to its first near-tie step, and the copies must agree with each other
    bit for bit (rows never mix in the arithmetic)."""
    arch, seed, cases = _cases("lm_tts1")
    m = _model(arch, seed, max_batch=64)
    tol = _margin_tol("lm_tts1", cases[0])
    for c in cases:
        outs = m.generate_batch([c["prompt"]] * rows, max_length=c["max_length"], min_new_tokens=c["min_new"],
                                eos_token_id=c["eos"], repetition_penalty=c["rep"])
        ref, hm = c["hf_new"], c["hf_margins"]
        k = next((i for i, x in enumerate(hm) if x < tol), len(ref))
        for o in outs:
            assert o == outs[0]
        assert outs[0][:k] == ref[:k], (k, outs[0], ref)


def test_vllm_form_frequency_penalty():
    """vLLM-form greedy with the reference's vLLM defaults (repetition 1.1 — CLI 1.4 —,
    frequency 0.3/0.4, min_tokens): teacher-forced on the engine's own output, every pick is
    the argmax of the oracle's restatement of vLLM's penalties (parity unpinned: vLLM is
    not installed) wherever the top-2 margin clears the logit tolerance."""
    arch, seed, cases = _cases("lm_tiny")
    m = _model(arch, seed)
    c = cases[0]

    class SP:
        max_tokens = 40
        min_tokens = 12
        stop_token_ids = [c["eos"]]
        repetition_penalty = 1.4
        frequency_penalty = 0.4
        temperature = 0.0

    new = m.generate(prompt_token_ids=c["prompt"], sampling_params=SP())[0].outputs[0].token_ids
    assert 12 <= len(new) <= 40
    plain = m.generate_batch([c["prompt"]], max_length=len(c["prompt"]) + 40, min_new_tokens=12,
                             eos_token_id=c["eos"], repetition_penalty=1.4)[0]
    assert new != plain  # the frequency penalty changes the greedy path
    seq = c["prompt"] + new
    lg = m.score([seq], len(new) + 1)[0]
    P = len(c["prompt"])
    for i in range(len(new)):
        sc = lm_oracle.vllm_process(lg[i], c["prompt"], new[:i], 1.4, 0.4, 12, c["eos"])
        top = torch.topk(sc, 2).values
        if float(top[0] - top[1]) >= LOGIT_TOL:
            assert int(torch.argmax(sc)) == new[i], i


def test_rows_stop_at_different_steps():
    """A batch whose rows hit EOS at different steps: stopped rows idle inside the captured
    step (their kernels skip them) while the others continue; every row equals its batch-1
    run, EOS included, and lengths differ."""
    arch, seed, cases = _cases("lm_small")
    m = _model(arch, seed)
    prompts = [c["prompt"] for c in cases]
    L = max(len(p) for p in prompts) + 40
    free = m.generate_batch(prompts, max_length=L, min_new_tokens=0, eos_token_id=-1, repetition_penalty=1.1)
    # a token some row emits for the first time (step >= 1 where the row varies): it stops there; the
    # others stop when (if) they emit it
    r, i = next((r, k) for r in range(len(free)) for k in range(len(free[r])) if free[r][k] not in free[r][:k] and k >= (1 if len(set(free[r])) > 1 else 0))
    eos = free[r][i]
    batch = m.generate_batch(prompts, max_length=L, min_new_tokens=0, eos_token_id=eos, repetition_penalty=1.1)
    singles = [m.generate_batch([p], max_length=L, min_new_tokens=0, eos_token_id=eos, repetition_penalty=1.1)[0]
               for p in prompts]
    assert batch == singles
    assert batch[r] == free[r][:i + 1]
    assert len({len(x) for x in batch}) > 1 or len(batch) == 1


_FUSED_CHILD = r'''
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
from tts_amd import configs, synth
from tts_amd.speechlm import MI355XSpeechLM
arch = configs.TTS1
m = MI355XSpeechLM.synthetic(arch, seed=0x5EED, max_batch=1, max_seq_len=1408)
vocab = configs.vocab_for(arch)
p = synth.synthetic_prompt(vocab, 3, 39, 150)
new = m.generate_batch([p], max_length=1400, min_new_tokens=1400 - len(p), eos_token_id=-1, repetition_penalty=1.1)[0]
print(json.dumps(new))
'''


def test_fused_qkv_attention_equals_separate_launches():
    """The one-row decode step's QKV launch with the attention fused in (q/k/v handed to
    appended attention workgroups as tagged granules, lm_gemm_kernel.h fattn_consumer) and
    o_proj fused behind that attention (the attention row handed back to the projection
    workgroups as granules, fused_oproj), the same launch without o_proj
    (TTS_FUSED_OPROJ=0), and all-separate launches (TTS_FUSED_ATTN=0) produce the same greedy ids on
    TTS-1 over 1.2k generated positions: the context crosses the 1,024 positions of the
    attention's first pass (a second pass per wave) and every 64-position wave boundary."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = {}
    for fa, fo in (("1", "1"), ("1", "0"), ("0", "0")):
        env = dict(os.environ, TTS_FUSED_ATTN=fa, TTS_FUSED_OPROJ=fo)
        r = subprocess.run([sys.executable, "-c", _FUSED_CHILD, root], env=env, capture_output=True, text=True,
                           timeout=110)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[fa + fo] = json.loads(r.stdout.strip().splitlines()[-1])
    assert len(outs["11"]) == 1400 - 202
    assert outs["11"] == outs["10"] == outs["00"]


@pytest.mark.parametrize("rows", [1, 8])
def test_tts1_max_dims_logits_vs_oracle(rows):
    """BASELINE config 4's kernel shapes (TTS-1-Max: d 4096, hd 128, ffn 14336 in K-chunked
    layouts, untied lm_head) with 2 layers: teacher-forced logits of the engine's prefill
    (MFMA GEMM) and decode step (weight-streaming GEMVs, batch `rows`) against the CPU oracle
    on the same weights (generated on the GPU, bit-identical to synth.lm_weights_cpu)."""
    from tts_amd import configs, synth
    from tts_amd.speechlm import MI355XSpeechLM

    arch = configs.LM_ARCHS["tts1-max-2l"]
    m = MI355XSpeechLM.synthetic(arch, seed=77, max_batch=8, max_seq_len=256)
    w = {k: v.cpu() for k, v in synth.lm_weights_device(arch, 77, torch.device("cuda")).items()}
    torch.cuda.empty_cache()
    orc = lm_oracle.LlamaOracle(arch, w, max_seq_len=256)
    rng = np.random.default_rng(rows)
    seqs = [rng.integers(0, arch.vocab_size, 24 + 3 * r).tolist() for r in range(rows)]
    got = m.score(seqs, 3)  # the last 3 positions of each sequence
    for r, s in enumerate(seqs):
        ref = orc.score(s, 3)
        # two valid implementations differ by up to ~0.57 in a logit at TTS-1 dims
        # (transformers vs the oracle, tests/golden/manifest.json: bf16 activations that round
        # differently under other fp32 summation orders); the bar here is 0.5 absolute
        err = (got[r] - ref).abs()
        assert err.max().item() <= 0.5, (r, err.max().item(), ref.flatten()[err.argmax()].item())
        assert err.mean().item() <= 0.05, (r, err.mean().item())  # ~1 bf16 ulp of |logit| ~ 5
    # greedy decode through the batched step equals the oracle's greedy where margins allow
    new = m.generate_batch(seqs, max_length=max(len(s) for s in seqs) + 6, min_new_tokens=6, eos_token_id=-1,
                           repetition_penalty=1.1)
    for r, s in enumerate(seqs[:2]):  # (the CPU oracle's greedy is the slow part)
        ref_new, margins = orc.generate(s, len(s) + 6, 6, -1, 1.1)
        k = next((i for i, x in enumerate(margins) if x < 2 * 0.5 + 0.125), len(ref_new))
        assert new[r][:k] == ref_new[:k], (r, k)
    m.close()


def test_tts1_teacher_forced_logits_vs_transformers():
    """The engine's bf16 logits at TTS-1 dims (16 layers, V = 193,856) against transformers'
    own teacher-forced logits (tests/golden/lm_tts1.npz tf_idx / tf_val: HF's top-32 and 32
    fixed random ids at every generated position of both cases).  The deviation two valid
    implementations show here — transformers vs the CPU oracle, max 0.44 / mean 0.078
    (manifest tf_oracle_*) — comes from ulp-level bf16 differences (CPU flash-attention
    internals) that the random network amplifies to ~0.5 % of the hidden state per layer
    (DESIGN.md §4).  Bar: 1.25x the engine's own measured deviation, 0.375 / 0.0791
    (profiles/r4a_tts1_tf_logit_dev.json): max <= 0.47 (one bf16 ulp above the measured max
    at |logit| < 32), mean <= 0.099.  The argmax agrees wherever HF's top-2 margin exceeds 2."""
    arch, seed, cases = _cases("lm_tts1")
    m = _model(arch, seed)
    z = np.load(os.path.join(GOLDEN, "lm_tts1.npz"))
    idx, val = torch.from_numpy(z["tf_idx"]).long(), torch.from_numpy(z["tf_val"])
    off = 0
    devs = []
    for c in cases:
        seq = c["prompt"] + c["hf_new"]
        n = len(c["hf_new"])
        lg = m.score([seq[:-1]], n)[0]  # logits predicting each generated token
        got = torch.gather(lg, 1, idx[off:off + n])
        d = (got - val[off:off + n]).abs()
        devs.append(d)
        for i in range(n):
            top2 = torch.topk(val[off + i], 2).values  # (top-32 first: HF's own top-2)
            if float(top2[0] - top2[1]) > 2.0:
                assert int(idx[off + i][int(torch.argmax(got[i]))]) == int(idx[off + i][0]), i
        off += n
    d = torch.cat(devs)
    # the measured deviation is recorded (gpurun_out/ on the box; committed under profiles/)
    import json

    rec = {"max_abs": d.max().item(), "mean_abs": d.mean().item(), "n": int(d.numel()),
           "bar_max": TF_MAX, "bar_mean": TF_MEAN}
    print("engine vs transformers teacher-forced logits:", rec)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "tts1_tf_logit_dev.json"), "w") as f:
        json.dump(rec, f)
    assert d.max().item() <= TF_MAX, d.max().item()
    assert d.mean().item() <= TF_MEAN, d.mean().item()


# engine-vs-transformers bars of the long-context decode comparisons (tests/golden/
# lm_tts1_long.npz, lm_max2l_long.npz), from the first measurement
# (profiles/r4a_long_tf_dev_*.json; every run rewrites gpurun_out/long_tf_dev_<fixture>.json):
# * TTS-1 (positions to 1,791): max 0.4375 / 0.484 / 0.547 at 1 / 4 / 24 rows, mean 0.083 —
#   the class of the two valid implementations' own difference at the same positions (the
#   CPU oracle's prefill vs transformers' decode: 0.4375 / 0.083, manifest); bar 1.25x the
#   largest: 0.68 / 0.104;
# * TTS-1-Max dims (positions to 759): 0.25 / 0.0385 at 1 and 8 rows (oracle vs transformers
#   0.25 / 0.0384); bar max 0.375 (one bf16 ulp above at |logit| in [16, 32): logits reach
#   33), mean 1.25x = 0.048
LONG_BARS = {"lm_tts1_long": (0.68, 0.104), "lm_max2l_long": (0.375, 0.048)}


def _long_case(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    lens = z["lens"].tolist()
    offs = np.concatenate([[0], np.cumsum(lens)])
    seqs = [z["ids"][offs[i]:offs[i + 1]].tolist() for i in range(len(lens))]
    return str(z["arch"]), int(z["seed"]), int(z["n_last"]), seqs, z["tf_idx"], torch.from_numpy(z["tf_val"])


@pytest.mark.parametrize("name,row_sets", [
    ("lm_tts1_long", [[0], [0, 1, 2, 3], [0, 1, 2, 3] * 6]),   # fused one-row step; <=16 rows; 17..32 rows
    ("lm_max2l_long", [[0], list(range(8))]),                  # head dim 128, configs[3]'s 8 rows per GPU
])
def test_decode_attention_long_context_vs_transformers(name, row_sets):
    """The DECODE step's arithmetic (MI355XSpeechLM.score_decode: prefill of a prefix, then one
    decode step per position) against transformers' own cached decode (oracle/make_golden.py
    hf_decode_logits) at the contexts the reference's defaults reach: TTS-1 over positions
    208..1,791 (max_tokens = 1,792, inferencing.py:21), crossing the decode attention's
    1,024-position pass (16 waves x 64 positions at head dim 64, lm_attn_core.h); the TTS-1-Max
    dims over positions 60..759 (configs[3]: P 202 + N 500), crossing the 512-position pass at
    head dim 128.  Each row set runs as one batch: one row (TTS-1: the fused QKV + attention
    + o_proj launch), <= 16 rows, 17..32 rows (the two-m-tile GEMVs).  Bars: LONG_BARS (above);
    copies of a sequence must agree bit for bit, and the argmax must be HF's wherever HF's
    top-2 margin exceeds 2 x the max bar."""
    import json

    from tts_amd import configs
    from tts_amd.speechlm import MI355XSpeechLM

    arch_name, seed, n_last, seqs, idx, val = _long_case(name)
    bar_max, bar_mean = LONG_BARS[name]
    arch = configs.LM_ARCHS[arch_name]
    rows_max = max(len(r) for r in row_sets)
    m = MI355XSpeechLM.synthetic(arch, seed=seed, max_batch=rows_max, max_seq_len=max(len(s) for s in seqs) + 8)
    rec = {}
    try:
        for rs in row_sets:
            got = m.score_decode([seqs[i] for i in rs], n_last, idx[rs])
            ref = val[rs]
            d = (got - ref).abs()
            rec[len(rs)] = {"max_abs": d.max().item(), "mean_abs": d.mean().item(), "n": int(d.numel()),
                            "first_pos": [len(seqs[i]) - n_last for i in sorted(set(rs))],
                            "last_pos": [len(seqs[i]) - 1 for i in sorted(set(rs))]}
            print(name, len(rs), "rows:", rec[len(rs)])
            for j, i in enumerate(rs):  # copies of one sequence: identical bits
                first = rs.index(i)
                assert torch.equal(got[j], got[first]), (name, len(rs), j)
            top2 = torch.topk(ref[:, :, :16], 2, dim=-1).values  # (HF's top-16 first: its own top-2)
            decisive = (top2[..., 0] - top2[..., 1]) > 2 * bar_max
            hit = got[:, :, :16].argmax(-1) == 0
            assert bool(hit[decisive].all()), (name, len(rs), int((~hit & decisive).sum()))
            assert d.max().item() <= bar_max, (name, len(rs), rec[len(rs)])
            assert d.mean().item() <= bar_mean, (name, len(rs), rec[len(rs)])
    finally:
        m.close()
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", f"long_tf_dev_{name}.json"), "w") as f:
            json.dump({"bars": [bar_max, bar_mean], "by_rows": rec}, f, indent=1)


def test_prefill_rows_do_not_depend_on_the_batch():
    """The prefill GEMMs sum K in canonical 1024-chunks whatever their launch form (one chunk
    per workgroup for a short prompt, the running sum in registers for a batch of prompts) and
    the scored lm_head takes the decode GEMM's order at any row count, so a sequence scored or
    generated alone gives the bits it gives inside a 20-sequence batch (202 rows alone: the
    one-chunk form; 20 x ~200 rows: 128-row tiles)."""
    from tts_amd import configs, synth

    m = _model("tts1", 0x5EED, max_batch=20)
    vocab = configs.vocab_for(configs.TTS1)
    seqs = [synth.synthetic_prompt(vocab, u, 39, 150 + (u % 5)) for u in range(20)]
    alone = m.score(seqs[:1], 4).numpy()
    batch = m.score(seqs, 4).numpy()
    assert np.array_equal(alone[0], batch[0])
    one = m.generate_batch(seqs[:1], max_length=len(seqs[0]) + 6, min_new_tokens=6, eos_token_id=-1,
                           repetition_penalty=1.1)[0]
    many = m.generate_batch(seqs, max_length=max(len(s) for s in seqs) + 6, min_new_tokens=6, eos_token_id=-1,
                            repetition_penalty=1.1)[0]
    assert many[:len(one)] == one
