"""Same-box A/B of an engine environment switch (e.g. TTS_AREG, TTS_FUSED_ATTN): per-kernel
decode times at `rows`, the graph-replayed decode step of a `rows`-utterance batch (500
codes each) and an md5 of its ids, each setting in its own child process, alternating.
usage: python scripts/env_ab_probe.py VAR ROWS [ROUNDS]   (settings VAR=$AB_V0 (0) and VAR=$AB_V1 (1);
AB_ARCH: the LM architecture, default tts1)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, sys, hashlib
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
from tts_amd import configs, synth
from tts_amd.speechlm import MI355XSpeechLM
rows = int(sys.argv[2])
arch = configs.LM_ARCHS[os.environ.get("AB_ARCH", "tts1")]
m = MI355XSpeechLM.synthetic(arch, max_batch=max(rows, 1), max_seq_len=720)
r = {}
for k in list(m.KERNELS) + ["qkv_attn", "qkv_attn_oproj", "head_screened", "head_screen"]:  # (the fused forms where they apply)
    try:
        r[k] = round(m.bench_kernel(k, rows=rows, ctx=450, iters=64)[0] * 1000, 2)
    except Exception:
        pass
vocab = configs.vocab_for(arch)
ps = [synth.synthetic_prompt(vocab, u, 39, 150) for u in range(rows)]
for _ in range(2):
    out = m.generate_batch(ps, max_length=len(ps[0]) + 500, min_new_tokens=500, eos_token_id=vocab.speech_end_id,
                           repetition_penalty=1.1)
a, b, k = m.last_timing()
r["step_us"] = round(b / k * 1000, 1)
r["ids_md5"] = hashlib.md5(str(out).encode()).hexdigest()[:10]
print(json.dumps(r))
'''
var, rows = sys.argv[1], sys.argv[2]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
for rd in range(rounds):
    for v in (os.environ.get("AB_V0", "0"), os.environ.get("AB_V1", "1")):
        env = dict(os.environ, **{var: v})
        out = subprocess.run([sys.executable, "-c", CHILD, ROOT, rows], env=env, capture_output=True, text=True,
                             timeout=300)
        line = out.stdout.strip().splitlines()[-1] if out.returncode == 0 else f"FAILED rc={out.returncode} {out.stderr[-600:]}"
        print(f"round {rd} {var}={v} rows={rows}: {line}", flush=True)
        if out.returncode != 0:
            sys.exit(1)
