import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))
import torch
from tts_amd import configs
from tts_amd.speechlm import MI355XSpeechLM
m = MI355XSpeechLM.synthetic(configs.TTS1, max_batch=32, max_seq_len=2048)
for rows in (1, 8, 32):
    for ctx in (16, 128, 450, 1000, 2000):
        r = {k: m.bench_kernel(k, rows=rows, ctx=ctx, iters=64) for k in ("attention", "o_proj", "qkv")}
        print(rows, ctx, {k: round(v[0] * 1000, 2) for k, v in r.items()}, flush=True)
for rows in (1, 4, 8, 16, 32):
    r = {k: m.bench_kernel(k, rows=rows, ctx=450, iters=32) for k in m.KERNELS}
    print("rows", rows, {k: (round(v[0] * 1000, 2), round(v[1] / v[0] / 1e6)) for k, v in r.items()}, flush=True)
