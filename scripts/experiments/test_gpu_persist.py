"""The persistent one-row decode step (tts-max_amd/csrc/lm_persist.hip: every layer of the
batch-1 step in ONE launch, weights streamed through per-wave LDS-DMA rings across phase
boundaries, vectors handed between workgroups as tagged granules) against the per-layer
launches (TTS_PERSIST=0): the same arithmetic, so the same greedy ids, id for id.

Random TTS-1 weights (non-decisive: bf16 near-ties are frequent at V = 193,856, so any
difference in a single rounding would flip ids within a few hundred steps), prompts of the
reference's shape, contexts crossing every 128-position attention chunk of max_seq_len 1024
(8 chunks: the merge's chunk groups of two) and 512 (4 chunks: groups of one).  The
persistent step is opt-in (TTS_PERSIST=1; DESIGN.md §3.5: slower than the launches), so the
decisive transformers fixture (tests/test_gpu_chain.py) runs through the launches, and
this equality carries it over to the persistent step."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r'''
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
from tts_amd import configs, synth
from tts_amd.speechlm import MI355XSpeechLM
max_seq, new_n, utt, rep = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), float(sys.argv[5])
arch = configs.TTS1
m = MI355XSpeechLM.synthetic(arch, seed=0x5EED, max_batch=1, max_seq_len=max_seq)
vocab = configs.vocab_for(arch)
p = synth.synthetic_prompt(vocab, utt, 39, 150)
out = []
for trial in range(2):  # twice: the second run replays the captured step (tags advance)
    out.append(m.generate_batch([p], max_length=len(p) + new_n, min_new_tokens=new_n, eos_token_id=-1,
                                repetition_penalty=rep)[0])
print(json.dumps({"ids": out, "persistent": m.decode_persistent()}))
'''


def _run(persist: str, *args):
    env = dict(os.environ, TTS_PERSIST=persist)
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, *map(str, args)], env=env, capture_output=True, text=True,
                       timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("max_seq,new_n,utt,rep", [(1024, 1024 - 202 - 8, 3, 1.1), (512, 512 - 202 - 4, 5, 1.4)])
def test_persistent_step_equals_launches(max_seq, new_n, utt, rep):
    on = _run("1", max_seq, new_n, utt, rep)
    off = _run("0", max_seq, new_n, utt, rep)
    assert on["persistent"] and not off["persistent"]
    assert len(on["ids"][0]) == new_n
    assert on["ids"][0] == on["ids"][1]  # deterministic across graph replays / generations
    first = next((i for i, (a, b) in enumerate(zip(on["ids"][0], off["ids"][0])) if a != b), None)
    assert first is None, f"first differing id at step {first}"
