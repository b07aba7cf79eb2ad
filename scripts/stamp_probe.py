"""In-kernel timeline of the one-row decode kernels (run on the MI355X box): loads the
diagnostic library (make -C tts-max_amd/csrc stamps: -DTTS_STAMPS), runs one launch of each
kernel through bench_kernel and prints, per kernel, the workgroups' clock stamps (100 MHz,
us relative to the earliest entry): entry / after prologue / first unit streamed / first
unit's epilogue done (GEMM workgroups), entry / granules seen / before attention / after
attention (fused attention workgroups).  usage: python scripts/stamp_probe.py [CTX] [ROWS] [ARCH]
(ROWS > 1: the batched kernels, and qkv_attn where the QKV launch carries the attention)"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))
from tts_amd import _lib, configs  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "tts-max_amd", "tts_amd", "libtts_mi355x_stamps.so")
lib = _lib.load_library()
from tts_amd.speechlm import MI355XSpeechLM  # noqa: E402

ctx = int(sys.argv[1]) if len(sys.argv) > 1 else 450
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 1
arch = configs.LM_ARCHS[sys.argv[3]] if len(sys.argv) > 3 else configs.TTS1
m = MI355XSpeechLM.synthetic(arch, max_batch=rows, max_seq_len=1040)
N = 1 << 16
buf = np.zeros(N, dtype=np.uint64)
f = lib.tts_debug_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_int]


def q(v):
    return "/".join(f"{x:5.2f}" for x in (np.min(v), np.median(v), np.max(v)))


for k in ("qkv", "o_proj", "gate_up", "down", "attention", "qkv_attn", "qkv_attn_oproj"):
    for rep in range(3):
        m.bench_kernel(k, rows=rows, ctx=ctx, iters=1)
        assert f(buf.ctypes.data, N) == 0
    t = buf.astype(np.int64)
    diag64 = (int(os.environ.get("TTS_WGEMM_DIAG", "0")) & 64) != 0
    simd = None
    if diag64:  # (the per-wave norm-end stamps carry the wave's SIMD in bits 60..61)
        simd = (t >> 60) & 3
        t = t & ((1 << 56) - 1)
    if k == "attention":
        st = t[16384:16384 + rows * arch.num_kv_heads * 8].reshape(-1, 8)
    else:
        st = t[:16384].reshape(-1, 32)
    st = st[st[:, 0] > 0]
    t0 = st[:, 0].min()
    us = (st - t0) / 100.0
    us[st == 0] = np.nan
    print(f"{k} ctx={ctx} rows={rows}: {len(st)} workgroups (min/median/max us from first entry)")
    if k in ("qkv_attn", "qkv_attn_oproj"):
        # grid order (WgemmArgs::fattn_first): default projection | attention | o_proj workgroups;
        # TTS_FATTN_FIRST=1: attention first
        first = os.environ.get("TTS_FATTN_FIRST", "0") == "1"
        na = rows * arch.num_kv_heads
        # (the one-row o_proj workgroups write no stamps; the 2..16-row ones do, last in the grid)
        no = arch.hidden_size // 16 if (k == "qkv_attn_oproj" and rows > 1) else 0
        nq = len(us) - na - no  # projection workgroups
        proj, cons = (us[na:], us[:na]) if first else (us[:nq], us[nq:nq + na])
        if no:
            op = us[nq + na:]
            print(f"  o_proj      entry {q(op[:, 0])}  row 0 granules {q(op[:, 1])}  all rows {q(op[:, 2])}  done {q(op[:, 3])}")

        print(f"  projection  entry {q(proj[:, 0])}  prologue {q(proj[:, 1])}  streamed {q(proj[:, 2])}  epilogue {q(proj[:, 3])}")
        print(f"  attention   entry {q(cons[:, 0])}  granules {q(cons[:, 1])}  rope {q(cons[:, 2])}  max {q(cons[:, 5])}  pv {q(cons[:, 6])}  attended {q(cons[:, 3])}")
    elif k == "attention":
        print(f"  entry {q(us[:, 0])}  rope {q(us[:, 2])}  attended {q(us[:, 3])}")
    else:
        print(f"  entry {q(us[:, 0])}  prologue {q(us[:, 1])}  streamed {q(us[:, 2])}  epilogue {q(us[:, 3])}")
        if not np.all(np.isnan(us[:, 6])):
            print(f"  A rows landed (LDS-DMA) {q(us[:, 6])}")
        if not np.all(np.isnan(us[:, 7])):
            print(f"  RMSNorm (wave 0): row statistic {q(us[:, 7])}  rows scaled {q(us[:, 24])}")

        w = us[:, 8:24]
        print(f"  waves streamed: first {q(np.nanmin(w, 1))} last {q(np.nanmax(w, 1))}  split-K barrier {q(us[:, 4])}  summed {q(us[:, 5])}")
        if diag64 and not np.all(np.isnan(w)):  # norm end per wave: delay behind the WG's first, by wave and SIMD
            ss = (simd[:16384].reshape(-1, 32))[t[:16384].reshape(-1, 32)[:, 0] > 0][:, 8:24]
            d = w - np.nanmin(w, 1, keepdims=True)
            print("  norm end behind the WG's first wave, mean us by wave: " +
                  " ".join(f"{np.nanmean(d[:, i]):.2f}" for i in range(16)))
            print("  ... by SIMD: " + " ".join(f"s{s}={np.nanmean(d[ss == s]):.2f}(n={int(np.sum(ss == s) / len(d))})"
                                            for s in range(4)))
            print("  SIMD of waves 0..15 in the first WG: " + " ".join(str(int(x)) for x in ss[0]))
    sys.stdout.flush()
