"""Persistent one-row step vs the per-layer launches, one layer stack pass at a time
(tts_lm_step_probe): max |diff| of the residual stream after the last layer."""
import ctypes
import dataclasses
import os
import sys

import numpy as np
import torch

os.environ.setdefault("TTS_STEP", "1")
sys.path.insert(0, "tts-max_amd")
from tts_amd import _lib, configs  # noqa: E402
from tts_amd.speechlm import MI355XSpeechLM  # noqa: E402


def probe(m, token, pos, path):
    a = m.arch
    out = np.zeros(a.hidden_size + (a.num_heads + 2 * a.num_kv_heads) * a.head_dim + a.num_heads * a.head_dim,
                   dtype=np.float32)
    _lib.check(m._lib.tts_lm_step_probe(m._h, token, pos, path, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
    return out


for L in [int(x) for x in (sys.argv[1:] or ["1", "16"])]:
    arch = dataclasses.replace(configs.TTS1, num_layers=L, name=f"tts1-{L}l")
    m = MI355XSpeechLM.synthetic(arch, seed=0x5EED, max_batch=1, max_seq_len=1024)
    for pos in [0, 1, 2, 5, 40]:
        a = probe(m, 128300 + pos, pos, 0)
        b = probe(m, 128300 + pos, pos, 1)
        c = probe(m, 128300 + pos, pos, 0)
        H, Q = m.arch.hidden_size, (m.arch.num_heads + 2 * m.arch.num_kv_heads) * m.arch.head_dim
        dq = np.abs(a[H:H + Q] - b[H:H + Q])
        da = np.abs(a[H + Q:] - b[H + Q:])
        print(f"   qkv max diff {dq.max():.4g} (at {int(dq.argmax())}) mean {dq.mean():.4g}; attn max diff {da.max():.4g} "
              f"(at {int(da.argmax())}) mean {da.mean():.4g}", flush=True)
        if pos == 0:
            qa, qb = a[H:H + Q], b[H:H + Q]
            print("   launch qkv[:8]", np.round(qa[:8], 3), "\n   step   qkv[:8]", np.round(qb[:8], 3))
            best = [int(np.argmin(np.abs(qa - qb[i]))) for i in range(24)]
            print("   best launch column for step columns 0..23:", best, flush=True)
            print("   ratio stats", np.round(np.median(qb / np.where(np.abs(qa) > 1e-3, qa, 1)), 4), flush=True)
        a, b, c = a[:H], b[:H], c[:H]
        d = np.abs(a - b)
        i = int(d.argmax())
        print(f"L={L} pos={pos}: launches repeat {np.abs(a - c).max():.4g}  step vs launches max {d.max():.4g} "
              f"(col {i}: {a[i]:.4f} vs {b[i]:.4f}) mean {d.mean():.4g} |x| {np.abs(a).mean():.4f}  "
              f"nan {int(np.isnan(b).sum())}", flush=True)
    m.close()
    del m
    torch.cuda.empty_cache()

if len(sys.argv) > 1 and sys.argv[1] == "map":
    pass
