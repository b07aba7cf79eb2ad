"""Decode-step A/B of the fused QKV+attention launch (TTS_FUSED_ATTN=1 vs 0), each setting
in its own child process, alternating: per-kernel times at rows=1 and the replayed step,
plus the greedy ids of one 500-code utterance (must be identical across settings)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, sys, hashlib
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
from tts_amd import configs, synth
from tts_amd.speechlm import MI355XSpeechLM
arch = configs.TTS1
m = MI355XSpeechLM.synthetic(arch, max_batch=1, max_seq_len=720)
ks = list(m.KERNELS) + (["qkv_attn"] if os.environ.get("TTS_FUSED_ATTN", "1") != "0" else [])
r = {k: round(m.bench_kernel(k, rows=1, ctx=450, iters=64)[0] * 1000, 2) for k in ks}
vocab = configs.vocab_for(arch)
p = synth.synthetic_prompt(vocab, 0, 39, 150)
for _ in range(2):
    out = m.generate_batch([p], max_length=len(p) + 500, min_new_tokens=500, eos_token_id=vocab.speech_end_id,
                           repetition_penalty=1.1)
a, b, k = m.last_timing()
r["step_us"] = round(b / k * 1000, 1)
r["ids_md5"] = hashlib.md5(str(out[0]).encode()).hexdigest()[:10]
print(json.dumps(r))
'''
for rd in range(int(os.environ.get("ROUNDS", "2"))):
    for v in ("0", "1"):
        env = dict(os.environ, TTS_FUSED_ATTN=v)
        out = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
        line = out.stdout.strip().splitlines()[-1] if out.returncode == 0 else f"FAILED rc={out.returncode} {out.stderr[-600:]}"
        print(f"round {rd} fused={v}: {line}", flush=True)
        if out.returncode != 0:
            sys.exit(1)
