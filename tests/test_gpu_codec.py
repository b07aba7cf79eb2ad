"""Codec decoder parity on the GPU (through the C ABI) against the waveforms the reference
``tts.core.codec.decoder.Decoder`` produced (tests/golden/codec_*.npz) and against the CPU
oracle (oracle/codec_oracle.py) on fresh inputs.

Tolerance: the engine computes in fp32 like the reference (different summation orders,
a GEMM-form irfft instead of pocketfft): relative L2 error of the waveform <= 1e-4 and
max abs error <= 1e-4 * max|wav| + 1e-6.
"""

import os

import numpy as np
import pytest
import torch

from oracle import codec_oracle

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REL_L2 = 1e-4


def _close(got, ref):
    rel = np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)
    assert rel <= REL_L2, rel
    assert np.abs(got - ref).max() <= 1e-4 * np.abs(ref).max() + 1e-6


_dec = {}


def _decoder(arch_name, seed):
    from tts_amd import configs
    from tts_amd.codec import MI355XAudioDecoder

    key = (arch_name, seed)
    if key not in _dec:
        for k in list(_dec):
            _dec.pop(k).close()
        _dec[key] = MI355XAudioDecoder.synthetic(configs.CODEC_ARCHS[arch_name], seed=seed, max_codes=256)
    return _dec[key]


@pytest.mark.parametrize("name", ["codec_24k", "codec_16k", "codec_48k", "codec_24k_d2"])
def test_decode_matches_reference(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    dec = _decoder(str(z["arch"]), int(z["seed"]))
    co = wo = 0
    for T, L in zip(z["lens"], z["wav_lens"]):
        codes = z["codes"][co:co + T]
        ref = z["wav"][wo:wo + L]
        wav = dec.decode(torch.tensor(codes))  # AudioDecoder.decode surface: [1, L] float32 CPU
        assert wav.shape == (1, L) and wav.dtype == torch.float32
        _close(wav[0].numpy(), ref)
        co += T
        wo += L


def test_batch_equals_single_and_oracle():
    from tts_amd import configs, synth

    arch = configs.CODEC_24K_D2
    seed = 77
    dec = _decoder(arch.name, seed)
    rng = np.random.default_rng(5)
    utts = [rng.integers(0, 65536, size=n) for n in (17, 1, 64, 5)]
    batch = dec.decode_batch(utts)
    w = synth.codec_weights_cpu(arch, seed)
    for u, b in zip(utts, batch):
        single = dec.decode(torch.tensor(u))[0].numpy()
        assert np.array_equal(single, b)  # same kernels, same order: bitwise
        ref = codec_oracle.decode(w, torch.tensor(u), arch.hop_length, arch.upsample_factors, arch.kernel_sizes,
                                  arch.depth)[0].numpy()
        _close(b, ref)
    # waveform kept in HBM
    total = sum(len(u) for u in utts) * arch.samples_per_code
    out = torch.empty(total, device="cuda")
    dev = dec.decode_batch(utts, out=out)
    for b, d in zip(batch, dev):
        assert np.array_equal(d.cpu().numpy(), b)


def test_decode_split_from_reference_codes_format(tmp_path):
    """Batched voicing of a stored split (codes_io.decode_split) == one decode per utterance."""
    from tts_amd import codes_io, configs
    from tts_amd.codec import MI355XAudioDecoder

    zc = np.load(os.path.join(GOLDEN, "codec_24k_d2.npz"))
    carch = configs.CODEC_ARCHS[str(zc["arch"])]
    dec = MI355XAudioDecoder.synthetic(carch, seed=int(zc["seed"]), max_codes=64)
    rng = np.random.default_rng(1)
    utts = [rng.integers(0, 65536, n).tolist() for n in (9, 30, 64, 70, 3, 12)]
    codes_io.write_codes(str(tmp_path / "ds"), "val", utts)
    st = codes_io.decode_split(dec, str(tmp_path / "ds"), "val", str(tmp_path / "out"), batch=4)
    assert st == {"utterances": 6, "voiced": 5, "skipped": 1,
                  "samples": sum(len(u) for u in utts if len(u) <= 64) * carch.samples_per_code}
    wav = np.fromfile(tmp_path / "out" / "val_wav.f32", dtype=np.float32)
    index = np.load(tmp_path / "out" / "val_wav_index.npy")
    assert index[3] == -1
    for i, u in enumerate(utts):
        if len(u) > 64:
            continue
        one = dec.decode(torch.tensor(u))[0].numpy()
        assert np.array_equal(wav[index[i]:index[i] + one.shape[0]], one)
    dec.close()
