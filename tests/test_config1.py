"""BASELINE configs[0] on the CPU: the 100 samples.jsonl utterances (committed as
tests/golden/config1_samples.json) as synthesis requests with the reference's RLHF pairing
(tts/data/datasets/rlhf.py:56-67; tts_amd/config1.py), against tests/golden/config1.npz,
which the reference's own _synthesize_audio produced for every one of them (transformers
generate on the tiny LM, the reference AudioDecoder around the depth-2 codec; make_golden.py
config1).  Here: the request plumbing (every request's new-code count is what the reference
generated; prompt layout) and the CPU oracle's greedy ids on the shortest utterances.  The
engine runs all 100 in tests/test_gpu_config1.py."""

import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load():
    from tts_amd import config1, configs

    z = np.load(os.path.join(GOLDEN, "config1.npz"))
    arch = configs.LM_ARCHS[str(z["lm_arch"])]
    vocab = configs.vocab_for(arch)
    reqs = config1.requests(config1.load_samples(os.path.join(GOLDEN, "config1_samples.json")), vocab)
    return z, arch, vocab, reqs


def test_requests_match_reference_run():
    z, arch, vocab, reqs = _load()
    assert len(reqs) == 100 and len(z["new_lens"]) == 100
    assert [r["n_new"] for r in reqs] == z["new_lens"].tolist()  # min_new = max new = N_i
    assert sum(r["n_new"] for r in reqs) == 20185  # ceil(50 * duration) over the corpus (403.2 s)
    for r in reqs:
        p = r["prompt_ids"]
        assert p[0] == vocab.bos_id and vocab.speech_start_id in p
        k = p.index(vocab.speech_start_id)
        assert len(p) - k - 1 == len(r["speech_ids"]) and all(0 <= c < vocab.codebook_size for c in r["speech_ids"])


def test_oracle_greedy_matches_reference_on_shortest():
    from oracle import lm_oracle
    from tts_amd import synth

    z, arch, vocab, reqs = _load()
    w = {k: v.float() for k, v in synth.lm_weights_cpu(arch, int(z["lm_seed"])).items()}
    orc = lm_oracle.LlamaOracle(arch, w, max_seq_len=2048)
    offs = np.concatenate([[0], np.cumsum(z["new_lens"])])
    order = sorted(range(100), key=lambda i: len(reqs[i]["prompt_ids"]) + reqs[i]["n_new"])[:3]
    for i in order:
        r = reqs[i]
        P = len(r["prompt_ids"])
        new, _ = orc.generate(r["prompt_ids"], P + r["n_new"], r["n_new"], vocab.speech_end_id, 1.1)
        assert new == z["new_ids"][offs[i]:offs[i + 1]].tolist(), i
