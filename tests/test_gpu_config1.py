"""BASELINE configs[0] through the engine: all 100 samples.jsonl requests (tts_amd/config1.py)
with the tiny LM and the depth-2 codec, against the reference's own _synthesize_audio run
(tests/golden/config1.npz): every generated id (20,185) equal, and every waveform (9.6 M
samples) equal in length with its energy and 64 sampled values within the codec tolerance
(relative 1e-4)."""

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_config1_engine_matches_reference_run():
    from tts_amd import config1, configs, inference
    from tts_amd.codec import MI355XAudioDecoder
    from tts_amd.speechlm import MI355XSpeechLM

    z = np.load(os.path.join(GOLDEN, "config1.npz"))
    arch = configs.LM_ARCHS[str(z["lm_arch"])]
    vocab = configs.vocab_for(arch)
    reqs = config1.requests(config1.load_samples(os.path.join(GOLDEN, "config1_samples.json")), vocab)
    lm = MI355XSpeechLM.synthetic(arch, seed=int(z["lm_seed"]), max_batch=1, max_seq_len=2048)
    dec = MI355XAudioDecoder.synthetic(configs.CODEC_ARCHS[str(z["codec_arch"])], seed=int(z["codec_seed"]),
                                       max_codes=2048)
    offs = np.concatenate([[0], np.cumsum(z["new_lens"])])
    for i, r in enumerate(reqs):
        P, N = len(r["prompt_ids"]), r["n_new"]
        out = lm.generate(input_ids=torch.tensor([r["prompt_ids"]]), max_length=P + N, min_new_tokens=N,
                          eos_token_id=vocab.speech_end_id, do_sample=False, repetition_penalty=1.1, top_p=1.0,
                          temperature=0.0)
        assert out[0, P:].tolist() == z["new_ids"][offs[i]:offs[i + 1]].tolist(), i
        st = inference.InferenceSettings(temperature=0.0, max_tokens=P + N, min_tokens=N, repetition_penalty=1.1)
        wav, _ = inference.synthesize_audio(lm, dec, r["prompt_ids"], r["speech_ids"], vocab.speech_end_id, st)
        w = wav[0].double().numpy()
        L = int(z["wav_lens"][i])
        assert w.size == L, (i, w.size, L)
        if L:
            ss = float(z["wav_ss"][i])
            assert abs((w ** 2).sum() - ss) <= 2e-4 * ss, i
            pick = np.linspace(0, L - 1, 64).astype(np.int64)
            ref = z["wav_pick"][i].astype(np.float64)
            assert np.abs(w[pick] - ref).max() <= 1e-4 * max(np.sqrt(ss / L), 1e-6) * 10, i
    lm.close()
    dec.close()
