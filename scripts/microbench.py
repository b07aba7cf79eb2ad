#!/usr/bin/env python
"""GPU micro-benchmarks for the decode-step GEMVs (run on the MI355X box).

Each shape rotates over enough weight copies (> 600 MB) that every launch streams from
HBM, not from the 256 MiB Infinity Cache, as in the real decode step.
Prints: name, MB per launch, us per launch, GB/s.   --wgemm-only skips the torch lines.
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))

import torch  # noqa: E402

from tts_amd import _lib  # noqa: E402


def timeit(fns, iters=64):
    for f in fns:
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(iters):
        fns[i % len(fns)]()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1000.0  # us


def main():
    only = "--wgemm-only" in sys.argv
    lib = _lib.load_library()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    shapes = [("qkv", 3072, 2048), ("o_proj", 2048, 2048), ("gate_up", 16384, 2048), ("down", 2048, 8192),
              ("lm_head", 193856, 2048)]
    for name, N, K in shapes:
        mb = N * K * 2 / 1e6
        R = max(2, int(600 / mb) + 1)
        x = torch.randn(1, K, device=dev).to(torch.bfloat16)
        wts = []
        for _ in range(R):
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            wt = torch.empty_like(w)
            _lib.check(lib.tts_op_retile(w.data_ptr(), wt.data_ptr(), N, K, 2 if name == "gate_up" else 0, stream))
            wts.append(wt)
            del w
        out = torch.empty(1, N if name != "gate_up" else N // 2, device=dev, dtype=torch.bfloat16)
        nw = torch.ones(K, device=dev, dtype=torch.bfloat16)
        epi = 2 if name == "gate_up" else 0
        norm = nw.data_ptr() if name in ("qkv", "gate_up") else None
        ldo = out.shape[1]
        fns = [(lambda wt=wt: lib.tts_op_wgemm(x.data_ptr(), 1, K, K, wt.data_ptr(), N, norm, 1e-5, out.data_ptr(),
                                                ldo, None, epi, stream)) for wt in wts]
        us = timeit(fns)
        print(f"wgemm_{name:8s} {mb:8.1f} MB {us:9.2f} us {mb * 1e6 / us / 1e3:8.1f} GB/s", flush=True)
        if not only:
            ws = [torch.randn(N, K, device=dev).to(torch.bfloat16) for _ in range(min(R, 4))]
            us2 = timeit([(lambda w=w: torch.mv(w, x[0])) for w in ws])
            print(f"torch_mv_{name:6s} {mb:8.1f} MB {us2:9.2f} us {mb * 1e6 / us2 / 1e3:8.1f} GB/s", flush=True)
            del ws
        del wts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
