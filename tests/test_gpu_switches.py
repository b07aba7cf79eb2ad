"""Every runtime switch that README.md lists as "the same bits" gives the default's bits.

The switches are read once per process (static), so each setting runs in its own child
process (one at a time): a TTS-1 engine (and, for the switches that act on head dim 128 only,
the 2-layer TTS-1-Max model) scores the same sequences through the DECODE step
(`score_decode`: prefill of the prefixes, then one decode step per position — the step
`generate` replays) at the row counts the switch acts on, and runs one graph-captured
`generate_batch`.  The child prints an md5 of the bf16 logits (gathered at fixed ids) and of
the ids per row count; every setting must print the default's digests.

Switches that change the arithmetic on purpose (TTS_KSLICE32=0, TTS_AGR=0: another K sum
order; TTS_CODEC_EXPF=0, TTS_CODEC_BX3=0) are not "same bits" and are covered by the parity
bars of their own paths.  The codec GEMM schedule switches are checked bit for bit by
tests/test_gpu_codec.py::test_codec_gemm_schedules_same_bits."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import hashlib, json, os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
from tts_amd import configs, synth
from tts_amd.speechlm import MI355XSpeechLM
arch = configs.LM_ARCHS[sys.argv[2]]
rows_list = [int(r) for r in sys.argv[3].split(",")]
vocab = configs.vocab_for(arch)
m = MI355XSpeechLM.synthetic(arch, seed=0x5EED, max_batch=max(rows_list), max_seq_len=320)
out = {}
for rows in rows_list:
    rng = np.random.default_rng(11 + rows)  # (per row count: a child may run any subset)
    seqs = [synth.synthetic_prompt(vocab, 40 + u, 39, 150 + 3 * u) for u in range(rows)]
    n_last = 6
    gi = rng.integers(0, arch.vocab_size, size=(rows, n_last, 48)).astype(np.int32)
    lg = m.score_decode(seqs, n_last, gather_idx=gi).numpy()
    ps = [s[:-n_last] for s in seqs]
    ids = m.generate_batch(ps, max_length=max(len(p) for p in ps) + 24, min_new_tokens=24, eos_token_id=-1,
                           repetition_penalty=1.1)
    out[str(rows)] = hashlib.md5(lg.tobytes()).hexdigest()[:12] + "/" + hashlib.md5(str(ids).encode()).hexdigest()[:12]
print(json.dumps(out))
'''

# (switch setting, architecture, decode row counts it acts on)
CASES = [
    ("TTS_FUSED_ATTN=0", "tts1", "1"),
    ("TTS_FUSED_OPROJ=0", "tts1", "1,8"),
    ("TTS_FUSED_OPROJ_ROWS=0", "tts1", "8"),
    ("TTS_FATTN_ROWS=0", "tts1", "8"),
    ("TTS_FATTN_FIRST=1", "tts1", "1,8"),
    ("TTS_CSPLIT=0", "tts1", "1,8"),
    ("TTS_QKV_DEFER=0", "tts1", "24"),
    ("TTS_RING4=0", "tts1", "8,24"),
    ("TTS_RING4_32=0", "tts1", "24"),
    ("TTS_COMBINE_FIXED=0", "tts1", "24"),
    ("TTS_SLICED_GRID=0", "tts1", "24"),
    ("TTS_HEAD_GRID=512", "tts1", "1,24"),
    ("TTS_NORM_ONCE=0", "tts1", "8,16,24"),
    # the prefill of the prefixes (score_decode prefills ~190 rows a sequence): one prompt takes
    # the one-chunk-per-workgroup form, 8 prompts the running sum; both in the XCD tile order
    ("TTS_PGEMM_XCD=0", "tts1", "1,8"),
    ("TTS_PGEMM_SPLIT=0", "tts1", "1"),
    ("TTS_PGEMM_SPLIT=1", "tts1", "1"),
    ("TTS_NORM_ONCE=0", "tts1-max-2l", "8"),
    ("TTS_BALANCE=0", "tts1-max-2l", "8"),
    ("TTS_FUSED_OPROJ_ROWS=0", "tts1-max-2l", "8"),
    # the greedy lm_head's int8 screen + exact recheck: the full lm_head's ids
    ("TTS_HEAD_SCREEN=0", "tts1", "1,8,24"),
    ("TTS_HEAD_SCREEN=0", "tts1-max-2l", "8"),
    ("TTS_HEAD_SCREEN_WAIT=0", "tts1", "1,8"),
    ("TTS_HEAD_SCREEN_WAIT=1", "tts1", "1,8"),
]


def _run(env_setting, arch, rows):
    env = dict(os.environ)
    for k in [c[0].split("=")[0] for c in CASES]:
        env.pop(k, None)
    if env_setting:
        k, v = env_setting.split("=")
        env[k] = v
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, arch, rows], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, f"{env_setting or 'default'} ({arch}, rows {rows}): rc {r.returncode}\n{r.stderr[-1500:]}"
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def defaults():
    base = {}
    for arch in sorted({c[1] for c in CASES}):
        rows = sorted({int(r) for c in CASES if c[1] == arch for r in c[2].split(",")})
        base[arch] = _run(None, arch, ",".join(map(str, rows)))
    return base


@pytest.mark.parametrize("setting,arch,rows", CASES)
def test_switch_gives_default_bits(defaults, setting, arch, rows):
    got = _run(setting, arch, rows)
    for r, digest in got.items():
        assert digest == defaults[arch][r], f"{setting} at {r} rows ({arch}): logits/ids {digest} vs {defaults[arch][r]}"
