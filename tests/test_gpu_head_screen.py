"""The greedy lm_head as an exact two-pass argmax (lm_head_screen.hip): an int8 screen bounds
every column's processed score, then the tiles that can hold the argmax are recomputed exactly as
the bf16 lm_head computes them.  The pick must be the full lm_head's pick bit for bit — the
greedy step of GenerationMixin._sample (transformers generation/utils.py:2894-2925) that
/root/reference/tts/inference/inferencing.py:94-107 drives — whatever the weights.

The switch is read once per process, so each setting runs in its own child process: a
synthetic TTS-1 engine (K 2048, tied lm_head) and the 2-layer TTS-1-Max model (K 4096, untied)
generate at 1 / 8 / 24 / 32 rows with repetition penalties 1.0 / 1.1 / 1.4 and the min-new EOS
mask active; the screened run (default) must give the ids of TTS_HEAD_SCREEN=0, and
TTS_HEAD_SCREEN_CHECK=1 (every tile recomputed, every exact score checked against its int8
bound: a violation raises) must too.  The twins case duplicates every lm_head row pair (row
2i + 1 = row 2i): every score then has an exact tie, and torch.argmax's lowest-index rule must
pick the even id of each pair at penalty 1.0 — the recheck recomputes both and keeps the lower."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys
import torch
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
from tts_amd import configs, synth
from tts_amd.speechlm import MI355XSpeechLM
arch = configs.LM_ARCHS[sys.argv[2]]
mode = sys.argv[3]
vocab = configs.vocab_for(arch)
w = synth.lm_weights_device(arch, 0x5EED, torch.device("cuda", 0))
if mode == "twins":
    t = w["model.embed_tokens.weight" if arch.tie_word_embeddings else "lm_head.weight"]
    t[1::2] = t[0::2]
if mode == "outliers":  # heavy-tailed rows: every 7th row x8, one element in 64 of the matrix x40
    t = w["model.embed_tokens.weight" if arch.tie_word_embeddings else "lm_head.weight"]
    g = torch.Generator(device=t.device).manual_seed(5)
    t[::7] *= 8
    mask = torch.rand(t.shape, generator=g, device=t.device) < 1.0 / 64
    t[mask] *= 40
cases = [(1, 1.0), (1, 1.1), (8, 1.4), (24, 1.1), (32, 1.0)] if mode != "twins" else [(1, 1.0), (8, 1.0), (32, 1.0)]
m = MI355XSpeechLM(arch, w, max_batch=32, max_seq_len=400, id_to_code=vocab.id_to_code())
del w
torch.cuda.empty_cache()
out = {}
for rows, rep in cases:
    prompts = [synth.synthetic_prompt(vocab, 7 + u, 20 + u, 120 + 2 * u) for u in range(rows)]
    ids = m.generate_batch(prompts, max_length=max(map(len, prompts)) + 80, min_new_tokens=30,
                           eos_token_id=vocab.speech_end_id, repetition_penalty=rep)
    out[f"{rows}/{rep}"] = ids
print(json.dumps(out))
'''


def _run(setting, arch, mode="plain"):
    env = dict(os.environ)
    for k in ("TTS_HEAD_SCREEN", "TTS_HEAD_SCREEN_CHECK"):
        env.pop(k, None)
    if setting:
        k, v = setting.split("=")
        env[k] = v
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, arch, mode], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, f"{setting or 'default'} ({arch}, {mode}): rc {r.returncode}\n{r.stderr[-2000:]}"
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("arch", ["tts1", "tts1-max-2l"])
def test_screened_head_picks_the_full_heads_ids(arch):
    full = _run("TTS_HEAD_SCREEN=0", arch)
    screened = _run(None, arch)
    for case, ids in full.items():
        assert screened[case] == ids, f"{arch} {case}: screened ids differ from the full lm_head's"
    assert sum(len(r) for rows in full.values() for r in rows) > 3000


def test_check_mode_finds_every_score_inside_its_bound():
    """Every tile recomputed exactly; a score above its int8 upper bound raises."""
    checked = _run("TTS_HEAD_SCREEN_CHECK=1", "tts1")
    full = _run("TTS_HEAD_SCREEN=0", "tts1")
    assert checked == full


def test_heavy_tailed_weights_stay_inside_their_bounds():
    """Outlier rows and elements (far from the uniform synthetic weights): the per-column scale
    of the int8 copy gets coarse, the bounds wide — every exact score must still sit inside its
    bound (check mode) and the pick must still be the full head's."""
    checked = _run("TTS_HEAD_SCREEN_CHECK=1", "tts1", "outliers")
    full = _run("TTS_HEAD_SCREEN=0", "tts1", "outliers")
    screened = _run(None, "tts1", "outliers")
    assert checked == full and screened == full


def test_exact_ties_take_the_lowest_id():
    twins = _run(None, "tts1", "twins")
    full = _run("TTS_HEAD_SCREEN=0", "tts1", "twins")
    assert twins == full
    ids = [i for rows in twins.values() for r in rows for i in r]
    assert ids and all(i % 2 == 0 for i in ids), "a tied pair resolved to the higher id"
