"""Streaming (config 5): chunked generation returns the one-shot tokens; windowed codec
chunks equal the reference decoder applied to the same windows (CPU oracle)."""

import os

import numpy as np
import pytest
import torch

from oracle import codec_oracle

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_generate_stream_equals_one_shot():
    from tts_amd import configs
    from tts_amd.speechlm import MI355XSpeechLM

    z = np.load(os.path.join(GOLDEN, "lm_tiny.npz"))
    arch = configs.LM_ARCHS[str(z["arch"])]
    m = MI355XSpeechLM.synthetic(arch, seed=int(z["seed"]), max_batch=4, max_seq_len=512)
    P0, P1 = int(z["prompt_lens"][0]), int(z["prompt_lens"][1])
    prompts = [z["prompt_ids"][:P0].tolist(), z["prompt_ids"][P0:P0 + P1].tolist()]
    ref = z["hf_new"][:int(z["hf_new_lens"][0])].tolist()
    eos = ref[30] if len(ref) > 30 else -1
    kw = dict(max_length=max(P0, P1) + 70, min_new_tokens=3, eos_token_id=eos, repetition_penalty=1.1)
    one = m.generate_batch(prompts, **kw)
    chunks = list(m.generate_stream(prompts, chunk=7, **kw))
    assert chunks[-1][1] and not any(d for _, d in chunks[:-1])
    assert chunks[-1][0] == one
    for (a, _), (b, _) in zip(chunks, chunks[1:]):  # prefixes grow
        assert all(y[:len(x)] == x for x, y in zip(a, b))
    assert [len(r) for r in chunks[1][0]] == [min(8, len(r)) for r in one]
    m.close()


class _FakeLM:
    """Yields predetermined speech ids in chunks (ids == codes + 100)."""

    def __init__(self, rows, chunk):
        self.rows, self.chunk = rows, chunk

    def ids_to_codes(self, ids):
        return [i - 100 if i >= 100 else -1 for i in ids]

    def generate_stream(self, prompts, max_length, chunk, **kw):
        n = 1
        L = max(len(r) for r in self.rows)
        while True:
            done = n >= L
            yield [r[:n] for r in self.rows], done
            if done:
                return
            n += chunk


def test_streaming_windows_match_reference_decoder():
    from tts_amd import configs, synth
    from tts_amd.codec import MI355XAudioDecoder
    from tts_amd.streaming import StreamingSynthesizer

    zc = np.load(os.path.join(GOLDEN, "codec_24k_d2.npz"))
    carch = configs.CODEC_ARCHS[str(zc["arch"])]
    dec = MI355XAudioDecoder.synthetic(carch, seed=int(zc["seed"]), max_codes=256)
    rng = np.random.default_rng(5)
    rows = [(rng.integers(0, 65536, n) + 100).tolist() + [7] for n in (61, 40)]  # 7 = EOS (non-speech)
    pcodes = [rng.integers(0, 65536, 30).tolist(), rng.integers(0, 65536, 12).tolist()]
    st = StreamingSynthesizer(_FakeLM(rows, 25), dec, chunk=25, left_context=25)
    got = {0: [], 1: []}
    for out, _ in st.stream([[1], [1]], pcodes, max_length=200):
        for b, w in out:
            got[b].append(np.asarray(w))
    spc = carch.samples_per_code
    cw = synth.codec_weights_cpu(carch, int(zc["seed"]))
    for b in (0, 1):
        codes = [c - 100 for c in rows[b] if c >= 100]
        assert sum(len(w) for w in got[b]) == len(codes) * spc
        # the first chunk: its window = last 25 prompt codes (or all) + the first 25 codes
        win = pcodes[b][-25:] + codes[:25]
        ref = codec_oracle.decode(cw, torch.tensor(win), carch.hop_length, carch.upsample_factors,
                                  carch.kernel_sizes, carch.depth).reshape(-1).numpy()
        ref = ref[len(ref) - 25 * spc:]
        rel = np.linalg.norm(got[b][0] - ref) / np.linalg.norm(ref)
        assert rel < 1e-4, rel
    dec.close()
