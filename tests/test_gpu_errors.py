"""Bad requests fail loudly through the C ABI (a tts_status + message, raised as TtsError or the
reference's own ValueError) before anything is launched, and leave the engine usable: the
next valid request returns exactly what it returns on a fresh engine."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_codec_rejects_bad_utterances_and_stays_usable():
    from tts_amd import configs
    from tts_amd._lib import TtsError
    from tts_amd.codec import MI355XAudioDecoder

    dec = MI355XAudioDecoder.synthetic(configs.CODEC_24K_D2, seed=3, max_codes=64)
    rng = np.random.default_rng(9)
    good = rng.integers(0, 65536, size=20)
    ref = dec.decode(torch.tensor(good))[0].numpy()
    with pytest.raises(TtsError, match="max_codes"):
        dec.decode_batch([good, rng.integers(0, 65536, size=65)])  # longer than max_codes
    with pytest.raises(TtsError, match="code out of range"):
        dec.decode_batch([good, np.array([3, 65536, 4])])  # FSQ index past 4^8
    with pytest.raises(TtsError, match="out of range"):
        dec.decode_batch([good, np.zeros(0, dtype=np.int32)])  # empty utterance
    again = dec.decode_batch([good, good[:7]])
    assert np.array_equal(again[0], ref)
    dec.close()


def test_lm_rejects_bad_requests_and_stays_usable():
    import os

    from tts_amd import configs
    from tts_amd._lib import TtsError
    from tts_amd.speechlm import MI355XSpeechLM

    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    z = np.load(os.path.join(golden, "lm_tiny.npz"))
    arch = configs.LM_ARCHS[str(z["arch"])]
    m = MI355XSpeechLM.synthetic(arch, seed=int(z["seed"]), max_batch=2, max_seq_len=64)
    p = z["prompt_ids"][:int(z["prompt_lens"][0])].tolist()[:20]
    kw = dict(max_length=len(p) + 12, min_new_tokens=12, eos_token_id=-1, repetition_penalty=1.1)
    ref = m.generate_batch([p], **kw)
    with pytest.raises(ValueError):
        m.generate_batch([p, p, p], **kw)  # more rows than max_batch
    with pytest.raises(ValueError):
        m.generate_batch([p], max_length=len(p), eos_token_id=-1)  # HF: input length >= max_length
    with pytest.raises(TtsError, match="max_seq_len"):
        m.generate_batch([p], max_length=len(p) + 60, min_new_tokens=60, eos_token_id=-1)
    with pytest.raises(TtsError, match="token id out of range"):
        m.generate_batch([p[:-1] + [arch.vocab_size]], **kw)
    assert m.generate_batch([p], **kw) == ref
    m.close()
