"""Prefill time of a batch of `rows` synthetic TTS-1 prompts (202 tokens each), median of 5,
and an md5 of the first 8 generated ids per row.   usage: python scripts/prefill_probe.py ROWS"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))
from tts_amd import configs, synth  # noqa: E402
from tts_amd.speechlm import MI355XSpeechLM  # noqa: E402

rows = int(sys.argv[1])
arch = configs.TTS1
m = MI355XSpeechLM.synthetic(arch, max_batch=rows, max_seq_len=240)
vocab = configs.vocab_for(arch)
ps = [synth.synthetic_prompt(vocab, u, 39, 150) for u in range(rows)]
ts = []
for _ in range(6):
    out = m.generate_batch(ps, max_length=len(ps[0]) + 8, min_new_tokens=8, eos_token_id=-1, repetition_penalty=1.1)
    ts.append(m.last_timing()[0])
ts = sorted(ts[1:])
print(json.dumps({"rows": rows, "prefill_ms": round(ts[len(ts) // 2], 3),
                  "ids_md5": hashlib.md5(str(out).encode()).hexdigest()[:10]}))
