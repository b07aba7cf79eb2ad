"""The prompt-audio encoder against the reference's own Encoder.encode.

tests/golden/encoder_16k.npz holds, for three synthetic 16 kHz waveforms (0.5, 1.3 and 3.0 s:
26 / 66 / 151 frames), the reference's codes (tts/core/codec/encoder.py:115-128 run on CPU in
fp32 with synthetic weights, oracle/make_golden.py), the w2v-bert-2.0 layer-16 features it
computed (transformers' Wav2Vec2BertModel from a local config: the hub dimensions, parity of
those dimensions unpinned), its SeamlessM4T input features, the acoustic encoder output and
the values its FSQ rounded.
Every rounded value sits >= 0.03 from a rounding boundary (manifest: min_round_margin), far
above fp32 summation-order noise, so the codes must match exactly.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _cases():
    z = np.load(os.path.join(GOLDEN, "encoder_16k.npz"))
    out, wo, to = [], 0, 0
    for n, T in zip(z["wav_lens"], z["T"]):
        n, T = int(n), int(T)
        out.append(dict(wav=z["wav"][wo:wo + n], w2v=z["w2v"][to:to + T], codes=z["codes"][to:to + T],
                        pre=z["pre_round"][to:to + T], feats=z["feats"][to:to + T]))
        wo += n
        to += T
    return int(z["seed"]), out


_enc = {}


def _encoder():
    from tts_amd.encoder import MI355XAudioEncoder

    if "e" not in _enc:
        seed, _ = _cases()
        _enc["e"] = MI355XAudioEncoder.synthetic(seed=seed)
    return _enc["e"]


@pytest.mark.parametrize("idx", [0, 1, 2])
def test_encoder_codes_from_reference_features(idx):
    """HIP encoder on the reference's own w2v-bert features: identical codes, rounded values
    within fp32 noise."""
    _, cases = _cases()
    c = cases[idx]
    codes, pre = _encoder().encode_with_features(c["wav"], c["w2v"], return_pre=True)
    assert codes.shape == c["codes"].shape
    np.testing.assert_array_equal(codes, c["codes"])
    assert np.abs(pre - c["pre"]).max() < 5e-3


@pytest.mark.parametrize("idx", [0, 1, 2])
def test_encoder_w2v_bert_in_hip(idx):
    """w2v-bert-2.0 (16 conformer layers, relative-key attention) in HIP from the reference's
    SeamlessM4T features: the same codes, rounded values within fp32 noise."""
    _, cases = _cases()
    c = cases[idx]
    codes, pre = _encoder().encode_from_features(c["wav"], c["feats"], return_pre=True)
    np.testing.assert_array_equal(codes, c["codes"])
    assert np.abs(pre - c["pre"]).max() < 5e-3


def test_encoder_full_path_and_cache():
    """AudioEncoder.encode on the waveform alone (host features, everything after them in
    HIP) gives the reference's codes; CachingAudioEncoder returns them as a list, once."""
    from tts_amd.encoder import CachingAudioEncoder

    _, cases = _cases()
    enc = _encoder()
    for c in cases:
        codes = enc.encode(torch.from_numpy(c["wav"])[None])
        assert codes.dtype == torch.int64
        np.testing.assert_array_equal(codes.numpy(), c["codes"])
    cache = CachingAudioEncoder(enc)
    first = cache.encode("p0", torch.from_numpy(cases[0]["wav"])[None])
    assert first == cases[0]["codes"].tolist()
    assert cache.encode("p0", torch.zeros(1, 100)) is first
