#!/usr/bin/env python
"""Throughput of the codec's fp32 GEMM (tts_op_gemm_f32: bf16x3 MFMA, no split-K) on the
transformer / conv shapes at one utterance (M = 650) and at a batch of 32 (M = 20800),
next to torch.matmul fp32 (hipBLASLt) on the same operands.

usage: python scripts/codec_gemm_probe.py
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))

from tts_amd import _lib  # noqa: E402


def main():
    lib = _lib.load_library()
    dev = torch.device("cuda:0")
    shapes = [(3072, 1024, "c_attn"), (1024, 1024, "c_proj"), (4096, 1024, "fc1"), (1024, 4096, "fc2"),
              (1024, 3072, "conv k=3"), (1024, 7168, "embed k=7")]
    s = torch.cuda.current_stream()
    for M in (650, 20800):
        for N, K, name in shapes:
            A = torch.randn(M, K, device=dev)
            B = torch.randn(N, K, device=dev)
            C = torch.empty(M, N, device=dev)

            def run():
                _lib.check(lib.tts_op_gemm_f32(A.data_ptr(), M, K, K, B.data_ptr(), N, None, C.data_ptr(), N, None, 0,
                                               ctypes.c_void_p(s.cuda_stream)))

            def ref():
                torch.matmul(A, B.t(), out=C)

            res = []
            for fn in (run, ref):
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                n = 20
                e0.record()
                for _ in range(n):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / n
                res.append((ms, 2.0 * M * N * K / ms / 1e9))
            print(f"M={M:6d} {name:10s} N={N:5d} K={K:5d}  bx3 {res[0][0] * 1000:8.1f} us {res[0][1]:7.1f} TF/s "
                  f"(bf16-equiv {6 * res[0][1]:7.1f})   torch fp32 {res[1][0] * 1000:8.1f} us {res[1][1]:7.1f} TF/s",
                  flush=True)


if __name__ == "__main__":
    main()
