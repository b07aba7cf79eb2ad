"""The decode step's fused QKV + attention + o_proj launches (lm_gemm_kernel.h) under
adverse conditions:

* its grid order (projection workgroups, then attention, then o_proj workgroups) lets every
  workgroup wait only on blocks of lower index, so it completes while other kernels hold CUs:
  a B = 1 generation running beside prompt-audio encodes on a second engine and stream gives
  the ids it gives alone;
* a granule wait that gives up (forced with TTS_FATTN_SPINS=1) is reported at the first read
  as an error, never returned as ids, and the engine stays usable."""

import os
import subprocess
import sys
import threading

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tts1_prompt():
    from tts_amd import configs, synth

    return synth.synthetic_prompt(configs.vocab_for(configs.TTS1), 5, 39, 150)


@pytest.mark.parametrize("arch_name,rows", [("tts1", 1), ("tts1", 8), ("tts1-max-2l", 8)])
def test_generation_beside_concurrent_encodes(arch_name, rows):
    """One row (QKV + attention + o_proj in one launch) and 8 rows (the 2..16-row form: the
    attention workgroups, then one o_proj workgroup per unit spinning on the attention's
    granules) complete beside a loop of prompt encodes on another stream, with the ids they
    give alone and no granule-wait timeout."""
    import torch

    from tts_amd import configs, synth
    from tts_amd.encoder import MI355XAudioEncoder
    from tts_amd.speechlm import MI355XSpeechLM

    arch = configs.LM_ARCHS[arch_name]
    p = synth.synthetic_prompt(configs.vocab_for(arch), 5, 39, 150)
    n = 300 if rows == 1 else 120
    m = MI355XSpeechLM.synthetic(arch, seed=0x5EED, max_batch=rows, max_seq_len=len(p) + n + 20)
    kw = dict(max_length=len(p) + n, min_new_tokens=n, eos_token_id=-1, repetition_penalty=1.1)
    alone = m.generate_batch([p] * rows, **kw)
    enc = MI355XAudioEncoder.synthetic(device=0)
    wav = torch.from_numpy(synth.synthetic_wav(3, 48000))[None]
    feats = enc.features(wav)
    ref_codes = enc.encode_from_features(wav[0].numpy(), feats)
    stop, n_enc, errs = threading.Event(), [0], []

    def encoder_loop():
        try:
            while not stop.is_set():
                c = enc.encode_from_features(wav[0].numpy(), feats)
                assert (c == ref_codes).all()
                n_enc[0] += 1
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    t = threading.Thread(target=encoder_loop)
    t.start()
    try:
        together = [m.generate_batch([p] * rows, **kw) for _ in range(3)]
    finally:
        stop.set()
        t.join()
    assert not errs, errs
    assert n_enc[0] >= 1
    assert all(x == alone for x in together)
    enc.close()
    m.close()


_SPIN_CHILD = r'''
import os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
from tts_amd import configs, synth
from tts_amd._lib import TtsError
from tts_amd.speechlm import MI355XSpeechLM
p = synth.synthetic_prompt(configs.vocab_for(configs.TTS1), 5, 39, 150)
m = MI355XSpeechLM.synthetic(configs.TTS1, seed=0x5EED, max_batch=2, max_seq_len=len(p) + 80)
kw = dict(max_length=len(p) + 64, min_new_tokens=64, eos_token_id=-1, repetition_penalty=1.1)
for trial in range(2):  # the error is raised at the first read, and again on the next request
    try:
        m.generate_batch([p], **kw)
        print("NO-ERROR")
        sys.exit(0)
    except TtsError as e:
        assert "granule wait timed out" in str(e), e
# the separate-launch step on the same engine still works
two = m.generate_batch([p, p], **kw)
assert two[0] == two[1] and len(two[0]) == 64
print("RAISED")
'''


def test_fused_wait_timeout_raises_at_first_read():
    # (TTS_FATTN_ROWS=0: the 2-row batch at the end takes the separate launches)
    r = subprocess.run([sys.executable, "-c", _SPIN_CHILD, ROOT],
                       env=dict(os.environ, TTS_FATTN_SPINS="1", TTS_FATTN_ROWS="0"),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == "RAISED", r.stdout


_ROWS_CHILD = r'''
import hashlib, os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
from tts_amd import configs
from tts_amd.speechlm import MI355XSpeechLM
arch = configs.LM_ARCHS[sys.argv[2]]
rows, L, n_last = int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
m = MI355XSpeechLM.synthetic(arch, seed=0x5EED, max_batch=rows, max_seq_len=L + 8)
rng = np.random.default_rng(rows)
seqs = [rng.integers(0, arch.vocab_size, L - 7 * r).tolist() for r in range(rows)]
idx = rng.integers(0, arch.vocab_size, (rows, n_last, 64)).astype(np.int32)
out = m.score_decode(seqs, n_last, idx).numpy()
print(hashlib.md5(out.tobytes()).hexdigest(), float(np.abs(out).max()))
'''


@pytest.mark.parametrize("arch,rows,L,n_last", [("tts1", 8, 1100, 24), ("tts1", 3, 700, 12), ("tts1", 2, 400, 12),
                                                 ("tts1", 16, 500, 8), ("tts1-max-2l", 8, 600, 24),
                                                 ("tts1-max-2l", 16, 560, 8)])
def test_batched_fused_qkv_attention_equals_separate_launches(arch, rows, L, n_last):
    """2..16-row decode steps with the attention carried by the QKV launch (the attention
    workgroups after the projection's, one per (row, kv head), waiting on each row's tagged
    granules) and o_proj behind it (its own workgroups, each wave waiting on its K range of
    every row's attention granules) give the same bits as the QKV launch without o_proj
    (TTS_FUSED_OPROJ_ROWS=0) and as the separate QKV, attention and o_proj launches
    (TTS_FATTN_ROWS=0), at contexts past the attention's first pass (1,024 positions at head
    dim 64, 512 at 128)."""
    outs = {}
    for name, env in (("fused", {}), ("no_oproj", {"TTS_FUSED_OPROJ_ROWS": "0"}), ("separate", {"TTS_FATTN_ROWS": "0"})):
        r = subprocess.run([sys.executable, "-c", _ROWS_CHILD, ROOT, arch, str(rows), str(L), str(n_last)],
                           env=dict(os.environ, **env), capture_output=True, text=True, timeout=200)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[name] = r.stdout.strip().splitlines()[-1]
    assert outs["fused"] == outs["no_oproj"] == outs["separate"], outs


@pytest.mark.parametrize("env", [{"TTS_FATTN_FIRST": "1"}, {"TTS_FATTN_FIRST": "1", "TTS_FUSED_OPROJ": "0"},
                                 {"TTS_FUSED_OPROJ": "0"}, {"TTS_FUSED_ATTN": "0"}])
def test_one_row_grid_orders_equal(env):
    """The one-row fused launch in round 3's grid order (TTS_FATTN_FIRST=1: attention
    workgroups first, o_proj on the projection workgroups after their QKV unit), with and
    without o_proj fused, gives the default launch's bits (and the separate launches')."""
    outs = []
    for e in ({}, env):
        r = subprocess.run([sys.executable, "-c", _ROWS_CHILD, ROOT, "tts1", "1", "1100", "24"],
                           env=dict(os.environ, **e), capture_output=True, text=True, timeout=200)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(r.stdout.strip().splitlines()[-1])
    assert outs[0] == outs[1], outs
