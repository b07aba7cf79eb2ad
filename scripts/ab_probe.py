"""Same-box A/B of library builds (ab/lib_*.so from scripts/ab_build.sh): per-kernel
decode times at rows=1 and the graph-replayed decode step, alternating A,B,A,B so box drift
shows.  Each measurement is its own child process (one engine at a time on the GPU).
usage: python scripts/ab_probe.py NAME1 NAME2 ... [--rounds 2]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, sys, time
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
import torch
from tts_amd import configs, synth
from tts_amd.speechlm import MI355XSpeechLM
arch = configs.TTS1
m = MI355XSpeechLM.synthetic(arch, max_batch=1, max_seq_len=720)
r = {k: round(m.bench_kernel(k, rows=1, ctx=450, iters=64)[0] * 1000, 2) for k in m.KERNELS}
vocab = configs.vocab_for(arch)
p = synth.synthetic_prompt(vocab, 0, 39, 150)
for _ in range(2):
    m.generate_batch([p], max_length=len(p) + 500, min_new_tokens=500, eos_token_id=vocab.speech_end_id,
                     repetition_penalty=1.1)
a, b, k = m.last_timing()
r["step_us"] = round(b / k * 1000, 1)
print(json.dumps(r))
'''
names = [a for a in sys.argv[1:] if not a.startswith("--")]
rounds = 2
if "--rounds" in sys.argv:
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1])
    names = [n for n in names if n != str(rounds)]
for rd in range(rounds):
    for n in names:
        env = dict(os.environ, TTS_LIB_PATH=os.path.join(ROOT, "ab", f"lib_{n}.so"))
        out = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True,
                             timeout=300)
        line = out.stdout.strip().splitlines()[-1] if out.returncode == 0 else f"FAILED rc={out.returncode} {out.stderr[-400:]}"
        print(f"round {rd} {n:10s} {line}", flush=True)
        if out.returncode != 0:
            sys.exit(1)
