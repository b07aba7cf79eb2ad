#!/usr/bin/env python
"""Phase timeline of the persistent one-row decode step (lm_persist.hip).

Runs one traced persistent step (TTS_PERSIST_TRACE: thread 0 of every workgroup stamps
the 100 MHz clock at each phase point of each layer) on TTS-1 random weights at the bench's
context, and prints, per layer, when each hand-off's LAST producer finished and when its
consumers were ready (microseconds from the step's first stamp), plus the phase spans.

Events: 0 layer start, 1 qkv input gathered + normed, 2 qkv published, 3 attention chunks
published, 10 merge published, 4 o input gathered, 5 o published (h), 6 gate/up input
gathered + normed, 7 act published, 8 down input gathered, 9 down published (next x).
usage: python scripts/persist_trace.py [ctx]
"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))


def main():
    ctx = int(sys.argv[1]) if len(sys.argv) > 1 else 452
    path = os.path.join(tempfile.gettempdir(), "persist_trace.bin")
    os.environ["TTS_PERSIST_TRACE"] = path
    os.environ["TTS_PERSIST"] = "1"
    from tts_amd import configs
    from tts_amd.speechlm import MI355XSpeechLM

    arch = configs.TTS1
    m = MI355XSpeechLM.synthetic(arch, seed=0x5EED, max_batch=1, max_seq_len=718)
    ms, by = m.bench_kernel("persist", rows=1, ctx=ctx, iters=10)
    print(f"persistent step: {ms * 1000:.1f} us/launch, {by / ms / 1e6:.0f} GB/s")
    L = arch.num_layers
    t = np.fromfile(path, dtype=np.uint64).reshape(256, L, 32).astype(np.int64)
    t0 = t[:, 0, 0].min()
    us = (t - t0) / 100.0  # 100 MHz ticks -> us
    A, B, C = slice(0, 128), slice(128, 192), slice(192, 256)
    BC = slice(128, 256)
    AB = slice(0, 192)  # qkv producers
    M = slice(192, 200)
    rows = []
    for l in range(L):
        r = dict(
            x_ready=us[A, l - 1, 9].max() if l else us[:, 0, 0].min(),
            qkv_in_max=us[AB, l, 1].max(), qkv_out=us[AB, l, 2].max(),
            attn_out=us[C, l, 3].max(), merge_out=us[M, l, 10].max(),
            o_in_max=us[BC, l, 4].max(), h_out=us[BC, l, 5].max(),
            gu_in_max=us[:, l, 6].max(), act_out=us[:, l, 7].max(),
            down_in_max=us[A, l, 8].max(), x_out=us[A, l, 9].max(),
        )
        rows.append(r)
    keys = list(rows[0])
    print("layer " + " ".join(f"{k:>10s}" for k in keys))
    for l, r in enumerate(rows):
        print(f"{l:5d} " + " ".join(f"{r[k]:10.2f}" for k in keys))
    d = np.array([[r[k] for k in keys] for r in rows])
    steps = np.diff(d, axis=1)
    print("\nmedian hop (us), layers 1..L-1:")
    for i in range(len(keys) - 1):
        print(f"  {keys[i]:>10s} -> {keys[i + 1]:<10s} {np.median(steps[1:, i]):7.2f}")
    # inside the phases (medians over layers 1.. of the per-layer max over the role's workgroups)
    def med(sl, ev):
        return np.median([us[sl, l, ev].max() for l in range(1, L)] - np.array([rows[l]["x_ready"] for l in range(1, L)]))
    print("\nphase points, us after x_ready (median over layers; max over workgroups):")
    for ev, name, sl in [(0, "layer start (B,C)", BC), (11, "qkv: x flags seen", AB), (1, "qkv: x normed", AB),
                         (14, "qkv: tiles done", AB), (2, "qkv: published", AB),
                         (12, "attn: qkv flags seen", C), (13, "attn: q/k/v in LDS", C), (16, "attn: rope + tiles", C),
                         (17, "attn: softmax", C), (18, "attn: P.V", C), (3, "attn: chunks out", C),
                         (10, "merge out", M), (4, "o: input gathered", BC), (5, "o: h published", BC),
                         (15, "gu: h flags seen", slice(0, 256)), (6, "gu: h normed", slice(0, 256)),
                         (7, "gu: act published", slice(0, 256)), (8, "down: act gathered", A), (9, "down: x out", A)]:
        print(f"  {name:>24s} {med(sl, ev):8.2f}")
    per_layer = np.diff([r["x_out"] for r in rows])
    print(f"\nlayer period (x_out to x_out): median {np.median(per_layer):.2f} us, total {rows[-1]['x_out']:.1f} us")
    # spreads: how long the slowest producer trails the median one
    for ev, name, sl in [(2, "qkv_out", AB), (5, "h_out", BC), (7, "act_out", slice(0, 256)), (9, "x_out", A)]:
        sp = [np.max(us[sl, l, ev]) - np.median(us[sl, l, ev]) for l in range(1, L)]
        print(f"  {name}: slowest - median producer {np.median(sp):.2f} us")


if __name__ == "__main__":
    main()
