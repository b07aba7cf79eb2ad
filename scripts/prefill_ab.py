"""Same-box A/B of the prefill (lm_pgemm.hip forms): prefill time of 1 and 32 bench prompts
(202 tokens each, the bs=1 / bs=32 workloads) and md5s of prompt 0's teacher-forced logits
scored alone and inside a 32-prompt batch (tts_lm_score runs the prefill kernels), each
setting in its own child process, alternating.
usage: python scripts/prefill_ab.py ROUNDS SETTING...   (SETTING: "VAR=V,VAR2=V2" or "-" for
none; TTS_LIB_PATH=... selects a frozen library)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import hashlib, json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
import numpy as np
from tts_amd import configs, synth
from tts_amd.speechlm import MI355XSpeechLM
arch = configs.LM_ARCHS[os.environ.get("AB_ARCH", "tts1")]
m = MI355XSpeechLM.synthetic(arch, max_batch=32, max_seq_len=720)
vocab = configs.vocab_for(arch)
ps = [synth.synthetic_prompt(vocab, u, 39, 150) for u in range(32)]
r = {}
for n in (1, 32):
    t = []
    for _ in range(6):
        m.generate_batch(ps[:n], max_length=len(ps[0]) + 2, min_new_tokens=2, eos_token_id=-1)
        t.append(m.last_timing()[0])
    r[f"prefill{n}_ms"] = round(sorted(t[1:])[len(t[1:]) // 2], 3)
alone = m.score(ps[:1], 4).numpy()
batch = m.score(ps[:32], 4).numpy()
r["p0_alone"] = hashlib.md5(alone[0].tobytes()).hexdigest()[:10]
r["p0_batch"] = hashlib.md5(batch[0].tobytes()).hexdigest()[:10]
r["batch"] = hashlib.md5(batch.tobytes()).hexdigest()[:10]
print(json.dumps(r))
'''
rounds = int(sys.argv[1])
for rd in range(rounds):
    for setting in sys.argv[2:]:
        env = dict(os.environ)
        if setting != "-":
            for kv in setting.split(","):
                k, v = kv.split("=", 1)
                env[k] = v
        out = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
        line = out.stdout.strip().splitlines()[-1] if out.returncode == 0 else f"FAILED rc={out.returncode} {out.stderr[-800:]}"
        print(f"round {rd} {setting}: {line}", flush=True)
        if out.returncode != 0:
            sys.exit(1)
