"""Phase timeline of the persistent one-row step (tts_lm_step_probe path 2): per layer, the
median / max over CUs of each phase stamp (us since the first stamp)."""
import ctypes
import os
import sys

import numpy as np

os.environ.setdefault("TTS_STEP", "1")
sys.path.insert(0, "tts-max_amd")
from tts_amd import _lib, configs  # noqa: E402
from tts_amd.speechlm import MI355XSpeechLM  # noqa: E402

NAMES = ["start", "x_ready", "qkv_done", "attn_pub", "attn_got", "o_done", "h_got", "gu_done", "d_start",
         "d_done", "col_sum", "x_pub", "ld_layer", "ld_stall", "at_gath", "at_core"]
m = MI355XSpeechLM.synthetic(configs.TTS1, seed=0x5EED, max_batch=1, max_seq_len=2048)
L, NCU, NEV = m.arch.num_layers, 256, 16
out = np.zeros(L * NCU * NEV, dtype=np.float32)
pos = int(sys.argv[1]) if len(sys.argv) > 1 else 390
path = int(sys.argv[2]) if len(sys.argv) > 2 else 2  # 3: hand-offs not awaited (the stream's pace)
for rep in range(3):
    _lib.check(m._lib.tts_lm_step_probe(m._h, 128300, pos, path, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
t = out.reshape(L, NCU, NEV)
print("event columns: median over CUs (max)")
print("layer " + " ".join(f"{n:>13s}" for n in NAMES))
for l in list(range(3)) + [L - 1]:
    row = []
    for e in range(16):
        v = t[l, :, e]
        v = v[v >= 0]
        row.append(f"{np.median(v):6.1f}({v.max():5.1f})" if len(v) else " " * 13)
    print(f"{l:5d} " + " ".join(row))
print("total us", float(t.max()))
# where the skew sits: per-XCD (c % 8) medians and the slowest CUs of layer 1
l = 1
for e in (7, 9, 10, 11):
    v = t[l, :, e]
    xcd = [float(np.median(v[x::8])) for x in range(8)]
    slow = np.argsort(-v)[:8]
    print(f"{NAMES[e]:8s} xcd medians {[round(x, 1) for x in xcd]} slowest CUs {slow.tolist()} {np.round(v[slow], 1).tolist()}")
np.save("gpurun_out/step_trace.npy", t)
