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
        _dec[key] = MI355XAudioDecoder.synthetic(configs.CODEC_ARCHS[arch_name], seed=seed, max_codes=1024)
    return _dec[key]


@pytest.mark.parametrize("name", ["codec_24k", "codec_16k", "codec_48k", "codec_24k_d2", "codec_24k_long"])
def test_decode_matches_reference(name):
    """codec_24k_long is the bench's codec leg: T = 650 (11 key chunks of 64 in the codec
    attention's online softmax, the long-T GEMM plans), 300, 130 and 65 codes."""
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


def test_ragged_batch_up_to_650_codes():
    """32 ragged utterances up to the bench's 650 codes in one decode_batch call: each equals
    its own single decode bit for bit, and the 650-code one equals the reference waveform."""
    z = np.load(os.path.join(GOLDEN, "codec_24k_long.npz"))
    dec = _decoder(str(z["arch"]), int(z["seed"]))
    T0, L0 = int(z["lens"][0]), int(z["wav_lens"][0])
    ref650 = z["codes"][:T0]
    rng = np.random.default_rng(32)
    lens = [int(x) for x in rng.integers(1, 651, size=31)]
    utts = [ref650] + [rng.integers(0, 65536, size=n) for n in lens]
    batch = dec.decode_batch(utts)
    _close(batch[0], z["wav"][:L0])
    for i in (0, 1, 7, 19, 31):
        single = dec.decode(torch.tensor(utts[i]))[0].numpy()
        assert np.array_equal(single, batch[i]), i
    for i, u in enumerate(utts):
        assert batch[i].shape[0] == len(u) * 480


def _write_codec_dir(tmp_path, arch, weights, fmt):
    import json as _json

    d = tmp_path / f"{arch.name}_{fmt}"
    d.mkdir()
    cfg = arch.to_json_dict()
    if arch.depth != 12:
        cfg["depth"] = arch.depth  # reduced-depth test variant (tts_amd extension key)
    (d / "model_config.json").write_text(_json.dumps(cfg))
    if fmt == "model":  # Decoder.load_from_checkpoint's strict branch: {"model": {"generator.<Decoder key>"}}
        ck = {"model": {"generator." + k: v for k, v in weights.items()}}
    else:  # xcodec2 release layout: {"state_dict": {"generator.<Generator key>", "fc_post_a.*"}}
        sd = {}
        for k, v in weights.items():
            if k.startswith("decoder."):
                sd["generator." + k[len("decoder."):]] = v
            elif k.startswith("fc_post_a."):
                sd[k] = v
        ck = {"state_dict": sd}
    torch.save(ck, d / "codec.pt")
    return str(d / "codec.pt")


@pytest.mark.parametrize("name,fmt", [("codec_24k_d2", "model"), ("codec_16k", "state_dict")])
def test_create_from_both_checkpoint_layouts(tmp_path, name, fmt):
    """codec.create (decoding.create + Decoder.load_from_checkpoint, decoder.py:91-119) on
    both on-disk layouts — incl. the upsampler's weight_g / weight_v pair, folded at load —
    reproduces the reference waveforms; a missing key raises as load_state_dict(strict)."""
    from tts_amd import codec, configs, synth

    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    arch = configs.CODEC_ARCHS[str(z["arch"])]
    w = synth.codec_weights_cpu(arch, int(z["seed"]))
    path = _write_codec_dir(tmp_path, arch, w, fmt)
    dec = codec.create(path, device="cuda:0", max_codes=128)
    assert dec.sample_rate == arch.sample_rate and dec.token_rate == 50
    T, L = int(z["lens"][0]), int(z["wav_lens"][0])
    wav = dec.decode(torch.tensor(z["codes"][:T]))
    _close(wav[0].numpy(), z["wav"][:L])
    dec.close()
    # strict: a checkpoint without fc_post_a.bias is rejected before anything is uploaded
    import shutil

    d2 = tmp_path / "bad"
    d2.mkdir()
    shutil.copy(os.path.join(os.path.dirname(path), "model_config.json"), d2 / "model_config.json")
    src = torch.load(path, weights_only=True)
    top = "model" if fmt == "model" else "state_dict"
    src[top] = {k: v for k, v in src[top].items() if not k.endswith("fc_post_a.bias")}
    torch.save(src, d2 / "codec.pt")
    with pytest.raises(RuntimeError, match="missing keys"):
        codec.create(str(d2 / "codec.pt"), device=0, max_codes=16)


_PASS_CHILD = r'''
import json, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
from tts_amd import configs
from tts_amd.codec import MI355XAudioDecoder
out = {}
for name in ("codec-48k", "codec-24k-d2"):
    dec = MI355XAudioDecoder.synthetic(configs.CODEC_ARCHS[name], seed=11, max_codes=200)
    rng = np.random.default_rng(7)
    utts = [rng.integers(0, 65536, size=n) for n in (3, 150, 1, 77, 200, 64, 9)]
    batch = dec.decode_batch(utts)
    single = [dec.decode(torch.tensor(u))[0].numpy() for u in utts]
    out[name] = [bool(np.array_equal(a, b)) for a, b in zip(batch, single)]
    dec.close()
print(json.dumps(out))
'''


def test_ragged_batch_in_several_passes_and_two_upsample_stages():
    """A batch larger than one pass (TTS_CODEC_PASS_CODES=160: the 7 utterances run as 5
    passes, one of them longer than the pass size) and the 2-stage 48 kHz upsampler over a
    ragged batch (segment tables at three time resolutions): every utterance equals its
    single decode bit for bit."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _PASS_CHILD, root], capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, TTS_CODEC_PASS_CODES="160"))
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert all(res["codec-48k"]) and all(res["codec-24k-d2"]), res


_SCHED_CHILD = r'''
import hashlib, os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
from tts_amd import configs
from tts_amd.codec import MI355XAudioDecoder
dec = MI355XAudioDecoder.synthetic(configs.CODEC_ARCHS["codec-24k"], seed=0xC0DEC, max_codes=1024)
rng = np.random.default_rng(5)
utts = [rng.integers(0, 65536, size=int(n)).tolist() for n in [650, 13, 400, 1, 257, 650, 96, 511]]
wav = dec.decode_batch(utts)
print(hashlib.md5(np.concatenate(wav).tobytes()).hexdigest())
'''


def _sched_md5(env):
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _SCHED_CHILD, root], env=dict(os.environ, **env),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.strip().splitlines()[-1]


@pytest.fixture(scope="module")
def sched_default_md5():
    return _sched_md5({})


@pytest.mark.parametrize("env", [{"TTS_CODEC_X3P": "0"}, {"TTS_CODEC_X3P_ILV": "0"}, {"TTS_CODEC_X3P_ILV": "1"},
                                 {"TTS_CODEC_X3P_TILE": "5"}, {"TTS_CODEC_X3P_TILE": "4"},
                                 {"TTS_CODEC_X3P_PP": "1"}, {"TTS_CODEC_X3P_TILE": "4", "TTS_CODEC_X3P_SMALL4": "1"}],
                         ids=["bx3", "ilv0", "ilv1", "tile5_3stage", "tile4_1wave", "pp", "tile4_4stage"])
def test_codec_gemm_schedules_same_bits(env, sched_default_md5):
    """Every codec GEMM form — the fp32-staging kernel, the planes kernel on each tile shape and
    DMA schedule — sweeps an output's K in the same order, so a ragged batch decodes to the
    same bits under each (each form in its own process: the switches are read once)."""
    assert _sched_md5(env) == sched_default_md5, env
