#!/usr/bin/env python
"""Per-kernel decode-step timings vs batch rows (TTS-1 dims), one line per (kernel, rows).
TTS_WGEMM_DIAG (1 no prologue, 2 no epilogue) is read once per process: run once per value."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))
from tts_amd import configs  # noqa: E402
from tts_amd.speechlm import MI355XSpeechLM  # noqa: E402

rows_list = [int(r) for r in (sys.argv[1] if len(sys.argv) > 1 else "1,16,24,32").split(",")]
m = MI355XSpeechLM.synthetic(configs.LM_ARCHS["tts1"], seed=7, device=0, max_batch=max(rows_list), max_seq_len=1024)
diag = os.environ.get("TTS_WGEMM_DIAG", "0")
for k in ("qkv", "o_proj", "gate_up", "down", "lm_head", "attention"):
    line = []
    for r in rows_list:
        ms, b = m.bench_kernel(k, rows=r, ctx=450, iters=40)
        line.append(f"r{r}:{ms * 1000:7.2f}us")
    print(f"diag{diag} {k:8s} " + " ".join(line), flush=True)
m.close()
