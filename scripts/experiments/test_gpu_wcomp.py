"""Exponent-coded weight stream (lm_wcomp.hip): lossless by construction, checked bit for bit.

The one-row lm_head launch streams each 1 KiB weight tile as 768 B (sign + 7 mantissa bits
per value and a 4-bit exponent code against a per-matrix window [eb, eb + 15]); tiles with
any exponent outside the window (zeros, subnormals, tiny values, inf/NaN) stay raw in a side
buffer.  The decoded operands are the same bf16 bits, so (a) the round trip through the C ABI
returns its input exactly for every kind of tile, and (b) generation with the coded stream
produces the same ids as with the plain tiles (the decisive chain fixture at V = 193,856:
tests/test_gpu_chain.py runs with it on, the default).
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from tts_amd import _lib

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return _lib.load_library()


def _roundtrip(lib, bits: np.ndarray):
    import ctypes

    from tts_amd import _lib

    assert bits.dtype == np.uint16 and bits.size % 512 == 0
    src = torch.from_numpy(bits.view(np.int16).copy()).cuda()
    out = torch.full_like(src, 0x5555)
    eb, nesc = ctypes.c_int32(), ctypes.c_int64()
    _lib.check(lib.tts_op_wcomp_roundtrip(src.data_ptr(), bits.size // 512, out.data_ptr(), ctypes.byref(eb),
                                          ctypes.byref(nesc), None))
    back = out.cpu().numpy().view(np.uint16)
    return back, eb.value, nesc.value


def _bf16_bits(x: np.ndarray) -> np.ndarray:
    return (torch.from_numpy(x.astype(np.float32)).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16))


def test_roundtrip_uniform_weights(lib):
    """Weights as the synthetic models draw them (uniform, std 0.02): few escapes, exact."""
    rng = np.random.default_rng(1)
    bits = _bf16_bits(rng.uniform(-0.0346, 0.0346, 4096 * 512))
    back, eb, nesc = _roundtrip(lib, bits)
    assert np.array_equal(back, bits)
    assert nesc < 0.05 * 4096, nesc
    e = (bits >> 7) & 0xFF
    assert e.max() <= eb + 15


def test_roundtrip_normal_with_zeros_and_subnormals(lib):
    rng = np.random.default_rng(2)
    x = rng.normal(0, 0.02, 2048 * 512).astype(np.float32)
    x[rng.integers(0, x.size, 300)] = 0.0
    x[rng.integers(0, x.size, 300)] = -0.0
    x[rng.integers(0, x.size, 200)] = 1e-39  # subnormal in bf16 too
    x[rng.integers(0, x.size, 50)] = 3.0     # outliers above the window
    bits = _bf16_bits(x)
    back, _, nesc = _roundtrip(lib, bits)
    assert np.array_equal(back, bits)
    assert nesc >= 1


def test_roundtrip_every_bit_pattern(lib):
    """All 65,536 bf16 patterns (inf, NaN payloads, both zeros, subnormals) several times over,
    shuffled: mostly escaped tiles, all exact."""
    rng = np.random.default_rng(3)
    bits = np.tile(np.arange(65536, dtype=np.uint16), 4)
    rng.shuffle(bits)
    back, _, _ = _roundtrip(lib, bits)
    assert np.array_equal(back, bits)


def test_roundtrip_window_edges(lib):
    """A tile spanning exactly 16 exponents is coded, 17 is escaped; eb picked for most tiles."""
    tiles = []
    for span in (16, 17, 16, 1, 17, 16):
        e = 100 + (np.arange(512) % span)
        s = (np.arange(512) % 2).astype(np.uint16) << 15
        m = (np.arange(512) * 37 % 128).astype(np.uint16)
        tiles.append((s | (e.astype(np.uint16) << 7) | m).astype(np.uint16))
    bits = np.concatenate(tiles)
    back, eb, nesc = _roundtrip(lib, bits)
    assert np.array_equal(back, bits)
    assert eb == 100 and nesc == 2


def test_lm_head_coded_equals_plain_ids():
    """A TTS-1-dims model (V = 193,856, 2 layers): greedy ids, 1 and 8 rows, coded lm_head
    stream vs the plain tiles: identical (the same bf16 operands reach the MFMA)."""
    from tts_amd import configs
    from tts_amd.speechlm import MI355XSpeechLM

    arch = configs.LmArch("tts1-2l", 2048, 2, 32, 8, 64, 8192, 193856, True, rope_factor=32.0)
    m = MI355XSpeechLM.synthetic(arch, seed=5, max_batch=8, max_seq_len=512)
    assert m.coded_weights()["tiles"] == 0  # opt-in: nothing built by default
    info = m.coded_weights(True)
    assert info["tiles"] == 193856 * 2048 // 512
    assert info["escaped"] < 0.05 * info["tiles"], info
    rng = np.random.default_rng(7)
    prompts = [rng.integers(128_000, 193_000, 40 + 3 * i).tolist() for i in range(8)]
    res = {}
    for on in (True, False, True):
        m.coded_weights(on)
        one = m.generate_batch(prompts[:1], max_length=120, repetition_penalty=1.1)
        eight = m.generate_batch(prompts, max_length=120, repetition_penalty=1.1)
        res.setdefault(on, []).append((one, eight))
    assert res[True][0] == res[False][0] == res[True][1]
    # switching under an open generation is refused (the captured step holds the operands);
    # the generation then finishes with the stream it started with
    from tts_amd import _lib

    it = m.generate_stream(prompts[:1], max_length=120, chunk=20, repetition_penalty=1.1)
    next(it)
    with pytest.raises(_lib.TtsError):
        m.coded_weights(False)
    last = None
    for last in it:
        pass
    assert last[0] == res[True][0][0]
