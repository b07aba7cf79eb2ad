"""Debug probe: tts_op_wgemm at K = 768 (not a multiple of 512) with and without the fused
norm, against the standalone norm + plain GEMM and the oracle.  usage: python scripts/k768_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from oracle import lm_oracle  # noqa: E402
from tts_amd import _lib  # noqa: E402

lib = _lib.load_library()
for M in (1, 8, 24):
    for K in (768, 1024):
        N = 1024
        g = torch.Generator().manual_seed(768 + M)
        x = torch.randn(M, K, generator=g).to(torch.bfloat16)
        nw = (1 + 0.2 * torch.randn(K, generator=g)).to(torch.bfloat16)
        w = (torch.randn(N, K, generator=g) * 0.03).to(torch.bfloat16)
        xn_ref = lm_oracle.rmsnorm(x, nw, 1e-5)
        ref = lm_oracle.linear(xn_ref, w)
        wd = w.cuda()
        wt = torch.empty_like(wd)
        _lib.check(lib.tts_op_retile(wd.data_ptr(), wt.data_ptr(), N, K, 0, None))
        xd = x.cuda()
        xn = torch.empty_like(xd)
        _lib.check(lib.tts_op_rmsnorm(xd.data_ptr(), nw.cuda().data_ptr(), 1e-5, xn.data_ptr(), M, K, None))
        o1 = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        _lib.check(lib.tts_op_wgemm(xn.data_ptr(), M, K, K, wt.data_ptr(), N, None, 0.0, o1.data_ptr(), N, None, 0, None))
        o2 = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        _lib.check(lib.tts_op_wgemm(xd.data_ptr(), M, K, K, wt.data_ptr(), N, nw.cuda().data_ptr(), 1e-5, o2.data_ptr(), N,
                                    None, 0, None))
        o3 = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        _lib.check(lib.tts_op_wgemm(xn_ref.cuda().data_ptr(), M, K, K, wt.data_ptr(), N, None, 0.0, o3.data_ptr(), N,
                                    None, 0, None))
        torch.cuda.synchronize()
        d = lambda a, b: float((a.float().cpu() - b.float()).abs().max())  # noqa: E731
        print(f"M={M} K={K}: norm vs oracle {d(xn, xn_ref):.4g}; plain(xn) vs ref {d(o1, ref):.4g}; "
              f"fused-norm vs ref {d(o2, ref):.4g}; plain(oracle xn) vs ref {d(o3, ref):.4g}; ref max {float(ref.abs().max()):.3g}",
              flush=True)
