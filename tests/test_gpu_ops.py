"""Op-level parity of the HIP kernels (through the C ABI) against the CPU oracle ops.

Tolerances: bf16 outputs may differ from the fp32-accumulated oracle by a different
summation order only, i.e. by at most a couple of bf16 ulps on a small fraction of
elements; fp32 codec GEMMs to ~1e-5 relative.
"""

import ctypes

import numpy as np
import pytest
import torch

from oracle import lm_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from tts_amd import _lib

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return _lib.load_library()


def _check(st):
    from tts_amd import _lib

    _lib.check(st)


def _bf16_close(got, ref, max_ulps=2, frac=0.01):
    """Elementwise within max_ulps bf16 ulps, and at most `frac` of elements differ at all."""
    g, r = got.float(), ref.float()
    ulp = torch.clamp(r.abs(), min=1e-30) * 2.0 ** -7
    bad = (g - r).abs() > max_ulps * ulp + 1e-6
    assert bad.sum().item() == 0, f"{bad.sum().item()} elements beyond {max_ulps} ulps"
    ndiff = (g != r).float().mean().item()
    assert ndiff <= frac, f"{ndiff:.4f} of elements differ"


def test_synth_fill_bit_identical(lib):
    from tts_amd import synth, _lib

    for n, seed, scale in [(1000, 1, 0.5), (4097, 0xDEADBEEF12345, 0.0346)]:
        ref = synth.synth_values(seed, n, scale)
        d = torch.empty(n, dtype=torch.float32, device="cuda")
        _check(lib.tts_synth_fill(d.data_ptr(), _lib.DT_F32, n, seed, scale, None))
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy().view(np.uint32), ref.view(np.uint32))
        b = torch.empty(n, dtype=torch.bfloat16, device="cuda")
        _check(lib.tts_synth_fill(b.data_ptr(), _lib.DT_BF16, n, seed, scale, None))
        torch.cuda.synchronize()
        assert torch.equal(b.cpu(), torch.from_numpy(ref).to(torch.bfloat16))


def _tiled(lib, w, epi=0):
    N, K = w.shape
    t = torch.empty_like(w)
    _check(lib.tts_op_retile(w.data_ptr(), t.data_ptr(), N, K, epi, None))
    return t


@pytest.mark.parametrize("M", [1, 2, 5, 16, 17, 40, 64])
@pytest.mark.parametrize("N,K", [(256, 256), (3072, 2048), (2048, 8192), (6144, 4096), (4096, 14336)])
def test_wgemm_store(lib, M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N)
    x = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.02).to(torch.bfloat16)
    ref = lm_oracle.linear(x, w)
    xd, wd = x.cuda(), w.cuda()
    wt = _tiled(lib, wd)
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    _check(lib.tts_op_wgemm(xd.data_ptr(), M, K, K, wt.data_ptr(), N, None, 0.0, out.data_ptr(), N, None, 0, None))
    torch.cuda.synchronize()
    _bf16_close(out.cpu(), ref)


@pytest.mark.parametrize("M", [1, 4, 16])
def test_wgemm_norm_resid_swiglu(lib, M):
    K, FF = 2048, 1024
    g = torch.Generator().manual_seed(M)
    x = (torch.randn(M, K, generator=g)).to(torch.bfloat16)
    nw = (1 + 0.2 * torch.randn(K, generator=g)).to(torch.bfloat16)
    wg = (torch.randn(FF, K, generator=g) * 0.02).to(torch.bfloat16)
    wu = (torch.randn(FF, K, generator=g) * 0.02).to(torch.bfloat16)
    h = lm_oracle.rmsnorm(x, nw, 1e-5)
    ref_act = torch.nn.functional.silu(lm_oracle.linear(h, wg)) * lm_oracle.linear(h, wu)
    # interleaved gate/up tiles, as the engine lays out mlp.gate_proj / mlp.up_proj
    wgu = _tiled(lib, torch.cat([wg, wu]).cuda(), epi=2)
    out = torch.empty(M, FF, dtype=torch.bfloat16, device="cuda")
    xd, nd = x.cuda(), nw.cuda()
    _check(lib.tts_op_wgemm(xd.data_ptr(), M, K, K, wgu.data_ptr(), 2 * FF, nd.data_ptr(), 1e-5, out.data_ptr(), FF,
                            None, 2, None))
    torch.cuda.synchronize()
    _bf16_close(out.cpu(), ref_act, max_ulps=3, frac=0.03)
    # residual epilogue: resid += act . Wd^T
    wd = (torch.randn(K, FF, generator=g) * 0.02).to(torch.bfloat16)
    ref_res = x + lm_oracle.linear(ref_act, wd)
    wdt = _tiled(lib, wd.cuda())
    res = xd.clone()
    act = ref_act.cuda()
    _check(lib.tts_op_wgemm(act.data_ptr(), M, FF, FF, wdt.data_ptr(), K, None, 0.0, None, K, res.data_ptr(), 1, None))
    torch.cuda.synchronize()
    _bf16_close(res.cpu(), ref_res, max_ulps=2, frac=0.02)


@pytest.mark.parametrize("M", [1, 8, 24])
def test_wgemm_norm_k_not_multiple_of_512(lib, M):
    """K = 768 (a multiple of 256, not of 512): the LDS-DMA prologue cannot stage the rows, so
    the op API normalises in a standalone pass first — the fused form's canonical sum order,
    so the result equals the fused launch's arithmetic; checked against the oracle's
    RMSNorm + nn.Linear, and row copies must agree bit for bit."""
    K, N = 768, 1024
    g = torch.Generator().manual_seed(768 + M)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    x[-1] = x[0]
    nw = (1 + 0.2 * torch.randn(K, generator=g)).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.03).to(torch.bfloat16)
    ref = lm_oracle.linear(lm_oracle.rmsnorm(x, nw, 1e-5), w)
    wt = _tiled(lib, w.cuda())
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    xd, nd = x.cuda(), nw.cuda()  # (held: a temporary's block could be reused by the next one)
    _check(lib.tts_op_wgemm(xd.data_ptr(), M, K, K, wt.data_ptr(), N, nd.data_ptr(), 1e-5, out.data_ptr(), N, None, 0,
                            None))
    torch.cuda.synchronize()
    _bf16_close(out.cpu(), ref, max_ulps=3, frac=0.03)
    assert torch.equal(out[0].cpu(), out[-1].cpu())


def test_wgemm_rejects_matrix_beyond_buffer_range(lib):
    """The weight stream addresses a matrix through one 32-bit buffer resource: a shape of
    4 GiB or more is refused with an error (no launch), never silently truncated."""
    st = lib.tts_op_wgemm(None, 1, 65536, 65536, None, 32768, None, 0.0, None, 32768, None, 0, None)
    assert st != 0
    assert b"unsupported" in lib.tts_last_error()


def test_rmsnorm(lib):
    M, K = 7, 2048
    x = torch.randn(M, K).to(torch.bfloat16)
    w = (1 + 0.2 * torch.randn(K)).to(torch.bfloat16)
    ref = lm_oracle.rmsnorm(x, w, 1e-5)
    xd, wd = x.cuda(), w.cuda()
    y = torch.empty_like(xd)
    _check(lib.tts_op_rmsnorm(xd.data_ptr(), wd.data_ptr(), 1e-5, y.data_ptr(), M, K, None))
    torch.cuda.synchronize()
    _bf16_close(y.cpu(), ref, max_ulps=1, frac=0.01)


@pytest.mark.parametrize("M,N,K", [(1, 1, 16), (65, 130, 48), (300, 1024, 2048), (129, 642, 656)])
def test_gemm_f32(lib, M, N, K):
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g)
    bias = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g)
    for act in (0, 1):
        ref = A.double() @ B.double().t() + bias.double()
        if act:
            ref = ref * torch.sigmoid(ref)
        ref = ref + R.double()
        Ad, Bd, bd, Rd = A.cuda(), B.cuda(), bias.cuda(), R.cuda()
        C = torch.empty(M, N, device="cuda")
        _check(lib.tts_op_gemm_f32(Ad.data_ptr(), M, K, K, Bd.data_ptr(), N, bd.data_ptr(), C.data_ptr(), N,
                                   Rd.data_ptr(), act, None))
        torch.cuda.synchronize()
        err = (C.cpu().double() - ref).abs().max().item()
        assert err <= 2e-6 * (A.abs() @ B.abs().t()).max().item() + 1e-5, err


def test_gemm_f32_sliding_window_conv(lib):
    """Conv1d(k=3, pad=1) as a GEMM over a zero-padded time-major buffer (lda = C < K)."""
    T, C, Co, k = 37, 64, 48, 3
    x = torch.randn(1, C, T)
    w = torch.randn(Co, C, k) * 0.1
    b = torch.randn(Co)
    ref = torch.nn.functional.conv1d(x, w, b, padding=1)[0].t()  # [T, Co]
    xp = torch.zeros(T + 2, C)
    xp[1:T + 1] = x[0].t()
    wr = w.permute(0, 2, 1).reshape(Co, k * C).contiguous()  # [co][j*C + ci]
    xd, wd, bd = xp.cuda(), wr.cuda(), b.cuda()
    out = torch.empty(T, Co, device="cuda")
    _check(lib.tts_op_gemm_f32(xd.data_ptr(), T, k * C, C, wd.data_ptr(), Co, bd.data_ptr(), out.data_ptr(), Co,
                               None, 0, None))
    torch.cuda.synchronize()
    assert torch.allclose(out.cpu(), ref, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("M", [16, 24, 32, 40, 64])
@pytest.mark.parametrize("N,K,epi", [(3072, 2048, 0), (2048, 8192, 1), (2048, 2048, 1), (16384, 2048, 2)])
def test_wgemm_rows_independent(lib, M, N, K, epi):
    """Rows never mix: M copies of one activation row give M identical output rows, whatever
    launch form the row count selects (A in LDS or global, K-sliced, 1/2/4 m-tiles)."""
    g = torch.Generator().manual_seed(N + K + epi)
    x1 = (torch.randn(1, K, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.02).to(torch.bfloat16)
    nw = (1 + 0.2 * torch.randn(K, generator=g)).to(torch.bfloat16) if epi != 1 and M <= 32 else None
    xd = x1.repeat(M, 1).cuda()
    wt = _tiled(lib, w.cuda(), epi=epi)
    nout = N // 2 if epi == 2 else N
    out = torch.zeros(M, nout, dtype=torch.bfloat16, device="cuda")
    res = (torch.randn(1, N, generator=g) * 0.5).to(torch.bfloat16).repeat(M, 1).cuda() if epi == 1 else None
    _check(lib.tts_op_wgemm(xd.data_ptr(), M, K, K, wt.data_ptr(), N, nw.cuda().data_ptr() if nw is not None else None,
                            1e-5, out.data_ptr() if epi != 1 else None, nout,
                            res.data_ptr() if res is not None else None, epi, None))
    torch.cuda.synchronize()
    y = (res if epi == 1 else out).cpu()
    assert torch.equal(y, y[:1].expand_as(y)), [int((y[i] != y[0]).sum()) for i in range(M)]


@pytest.mark.parametrize("M", [65, 202, 700])
@pytest.mark.parametrize("N,K", [(384, 256), (3072, 2048), (2048, 8192), (4096, 14336)])
def test_pgemm_store_and_rows_independent(lib, M, N, K):
    """Prefill GEMM (tiles of the decode stream-plan layout, LDS-staged MFMA blocks) against
    the oracle's bf16 nn.Linear; the first and last rows are copies, so they must agree bit
    for bit whatever row block they fall in."""
    g = torch.Generator().manual_seed(M + N + K)
    x = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16)
    x[-1] = x[0]
    w = (torch.randn(N, K, generator=g) * 0.02).to(torch.bfloat16)
    ref = lm_oracle.linear(x, w)
    wt = _tiled(lib, w.cuda())
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    _check(lib.tts_op_pgemm(x.cuda().data_ptr(), M, K, wt.data_ptr(), N, out.data_ptr(), N, None, 0, None))
    torch.cuda.synchronize()
    o = out.cpu()
    if K > 8192:  # long sums: cancelled outputs carry more than 2 ulps of their own size
        err = (o.float() - ref.float()).abs()
        assert bool((err <= 2 * 2.0 ** -7 * ref.float().abs() + 2e-3).all())
    else:
        _bf16_close(o, ref)
    assert torch.equal(o[0], o[-1])


@pytest.mark.parametrize("M", [130, 600])
def test_pgemm_resid_swiglu(lib, M):
    K, FF = 2048, 1024
    g = torch.Generator().manual_seed(M)
    h = (torch.randn(M, K, generator=g)).to(torch.bfloat16)
    wg = (torch.randn(FF, K, generator=g) * 0.02).to(torch.bfloat16)
    wu = (torch.randn(FF, K, generator=g) * 0.02).to(torch.bfloat16)
    ref_act = torch.nn.functional.silu(lm_oracle.linear(h, wg)) * lm_oracle.linear(h, wu)
    wgu = _tiled(lib, torch.cat([wg, wu]).cuda(), epi=2)
    act = torch.empty(M, FF, dtype=torch.bfloat16, device="cuda")
    _check(lib.tts_op_pgemm(h.cuda().data_ptr(), M, K, wgu.data_ptr(), 2 * FF, act.data_ptr(), FF, None, 2, None))
    torch.cuda.synchronize()
    _bf16_close(act.cpu(), ref_act, max_ulps=3, frac=0.03)
    wd = (torch.randn(K, FF, generator=g) * 0.02).to(torch.bfloat16)
    ref_res = h + lm_oracle.linear(ref_act, wd)
    res = h.cuda()
    a = ref_act.cuda()
    _check(lib.tts_op_pgemm(a.data_ptr(), M, FF, _tiled(lib, wd.cuda()).data_ptr(), K, None, K, res.data_ptr(), 1, None))
    torch.cuda.synchronize()
    # residual add: an ulp of the projection is an ulp of max(|h|, |y|), not of the
    # (possibly cancelled) sum
    y = lm_oracle.linear(ref_act, wd).float()
    scale = torch.maximum(h.float().abs(), y.abs())
    err = (res.cpu().float() - ref_res.float()).abs()
    assert (err > 4 * scale * 2.0 ** -8 + 1e-6).sum().item() == 0


@pytest.mark.parametrize("epi,N,K", [(0, 3072, 2048), (1, 2048, 8192), (2, 2048, 2048), (0, 384, 256), (1, 4096, 14336)])
def test_pgemm_rows_bit_identical_across_batch_sizes(lib, epi, N, K):
    """Canonical K chunks: the first 65 rows of a prefill GEMM give the same bits whether the
    launch holds 65, 202 (one canonical chunk per workgroup + the in-order combine), 300
    (small tiles, the running sum in registers) or 700 rows (128-row tiles): a prompt's
    prefill does not depend on the batch it is prefilled in."""
    g = torch.Generator().manual_seed(epi * 7 + N + K)
    x = (torch.randn(700, K, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.02).to(torch.bfloat16)
    wt = _tiled(lib, w.cuda(), epi=epi)
    nout = N // 2 if epi == 2 else N
    base = (torch.randn(700, nout, generator=g) * 0.5).to(torch.bfloat16) if epi == 1 else None
    got = {}
    for M in (65, 202, 300, 700):
        xd = x[:M].cuda()
        if epi == 1:
            res = base[:M].cuda()
            _check(lib.tts_op_pgemm(xd.data_ptr(), M, K, wt.data_ptr(), N, None, nout, res.data_ptr(), 1, None))
            torch.cuda.synchronize()
            got[M] = res[:65].cpu()
        else:
            out = torch.empty(M, nout, dtype=torch.bfloat16, device="cuda")
            _check(lib.tts_op_pgemm(xd.data_ptr(), M, K, wt.data_ptr(), N, out.data_ptr(), nout, None, epi, None))
            torch.cuda.synchronize()
            got[M] = out[:65].cpu()
    for M in (202, 300, 700):
        assert torch.equal(got[M], got[65]), (M, int((got[M] != got[65]).sum()))
