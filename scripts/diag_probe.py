"""Per-kernel decode times (rows=1, ctx=450) under TTS_WGEMM_DIAG settings, each in its own
child process: how much of each launch is prologue / epilogue / split-K exchange.
usage: python scripts/diag_probe.py 0 1 2 3"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
from tts_amd import configs
from tts_amd.speechlm import MI355XSpeechLM
rows = int(sys.argv[2])
m = MI355XSpeechLM.synthetic(configs.TTS1, max_batch=rows, max_seq_len=720)
print(json.dumps({k: round(m.bench_kernel(k, rows=rows, ctx=450, iters=64)[0] * 1000, 2) for k in m.KERNELS}))
'''
rows = os.environ.get("ROWS", "1")
for d in sys.argv[1:]:
    env = dict(os.environ, TTS_WGEMM_DIAG=d)
    out = subprocess.run([sys.executable, "-c", CHILD, ROOT, rows], env=env, capture_output=True, text=True, timeout=300)
    line = out.stdout.strip().splitlines()[-1] if out.returncode == 0 else f"FAILED rc={out.returncode} {out.stderr[-300:]}"
    print(f"diag {d:>3s} rows {rows}: {line}", flush=True)
