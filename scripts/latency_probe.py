"""Where a one-row decode kernel's time goes (run on the MI355X box): per-kernel launch time
against context length (attention, fused QKV+attention) and against the wgemm timing
diagnostics (TTS_WGEMM_DIAG: 1 no prologue, 2 no epilogue, 3 neither), each setting in its
own child process.  usage: python scripts/latency_probe.py"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys, os
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
from tts_amd import configs
from tts_amd.speechlm import MI355XSpeechLM
m = MI355XSpeechLM.synthetic(configs.TTS1, max_batch=1, max_seq_len=1040)
mode = sys.argv[2]
r = {}
if mode == "ctx":
    for ctx in (1, 64, 256, 450, 700, 1024):
        r[ctx] = {k: round(m.bench_kernel(k, rows=1, ctx=ctx, iters=64)[0] * 1000, 2) for k in ("attention", "qkv_attn")}
else:
    ks = ("qkv", "o_proj", "gate_up", "down") + (("qkv_attn",) if os.environ.get("TTS_WGEMM_DIAG", "0") == "0" else ())
    r = {k: round(m.bench_kernel(k, rows=1, ctx=450, iters=64)[0] * 1000, 2) for k in ks}
print(json.dumps(r))
'''
runs = [("ctx", {})] + [("diag", {"TTS_WGEMM_DIAG": d}) for d in ("0", "1", "2", "3", "8")] + \
    [("diag", {"TTS_STREAM_PLAN": "1"}), ("diag", {"TTS_CSPLIT": "0"})]
for mode, extra in runs:
    env = dict(os.environ, **extra)
    out = subprocess.run([sys.executable, "-c", CHILD, ROOT, mode], env=env, capture_output=True, text=True, timeout=300)
    line = out.stdout.strip().splitlines()[-1] if out.returncode == 0 else f"FAILED rc={out.returncode} {out.stderr[-600:]}"
    print(mode, json.dumps(extra), line, flush=True)
    if out.returncode != 0:
        sys.exit(1)
