"""CPU restatement of the screened greedy head's bound (lm_head_screen.hip).

The GPU screen picks the greedy id of a step from an int8 copy of the lm_head: for every column
c it computes a_c = sx*scale_c*(X . q_c) (X: the normalised row as 16-bit integers, q_c: the
column as int8 with scale_c = max|W_c| / 127) and the half-width
    e_c = |x| (r_c + gam |W_c|) + |x - sx X| |scale_c q_c|,   gam = 2 K 2^-24,
and recomputes exactly only the columns whose upper bound reaches the best lower bound.  The
pick equals the full bf16 lm_head's (the argmax of fp32(bf16(x . W_c)) after the repetition
penalty, lowest index on ties — generation/utils.py:2894-2925) exactly when every fp32 logit
lies inside [a_c - e_c, a_c + e_c].  This test checks that property in numpy on random and
heavy-tailed matrices at TTS-1's K, against fp32 sums in three different orders (so it does not
depend on one accumulation order), and that the candidate set always holds the argmax.  The GPU
tests (tests/test_gpu_head_screen.py) check the same on the device through the C ABI."""

import numpy as np

K, V = 2048, 4096


def bf16(a):
    """Round fp32 to the nearest bf16 (ties to even), returned as fp32."""
    u = np.asarray(a, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def quantise_columns(W):
    """head_quant_kernel: per column scale = max|W_c| / 127 (fp32), q = rint(W / scale)."""
    mx = np.abs(W).max(axis=1).astype(np.float32)
    scale = np.where(mx > 0, mx / np.float32(127), np.float32(1)).astype(np.float32)
    q = np.clip(np.rint(W / scale[:, None]), -127, 127).astype(np.int64)
    Wh = scale[:, None].astype(np.float64) * q
    r = np.sqrt(((W.astype(np.float64) - Wh) ** 2).sum(axis=1))
    nW = np.sqrt((W.astype(np.float64) ** 2).sum(axis=1))
    nWh = np.sqrt((Wh ** 2).sum(axis=1))
    up = 1 + 1e-9
    return scale, q, r * up, nW * up, nWh * up


def quantise_row(x):
    """The screen prologue: sx = max|x| / 32639, X = rint(x / sx); |x|, |x - sx X| rounded up."""
    mx = np.float32(np.abs(x).max())
    sx = mx / np.float32(32639) if mx > 0 else np.float32(1)
    X = np.clip(np.rint(x / sx), -32639, 32639).astype(np.int64)
    nx = np.sqrt((x.astype(np.float64) ** 2).sum()) * (1 + 2 ** -10)
    ndx = np.sqrt(((x.astype(np.float64) - np.float64(sx) * X) ** 2).sum()) * (1 + 2 ** -10) + 1e-30
    return sx, X, nx, ndx


def fp32_dots(x, W, order):
    """fp32 logits accumulated in a given order of k (the GPU's MFMA order is one of many)."""
    xs, Ws = x[order].astype(np.float32), W[:, order].astype(np.float32)
    acc = np.zeros(W.shape[0], np.float32)
    for k in range(0, K, 32):  # chunks of 32 products, each summed, then added in sequence
        acc = (acc + (xs[k:k + 32] * Ws[:, k:k + 32]).sum(axis=1, dtype=np.float32)).astype(np.float32)
    return acc


def check(W, x, seen, penalty, rng):
    W = bf16(W)
    x = bf16(x)
    scale, q, r, nW, nWh = quantise_columns(W)
    sx, X, nx, ndx = quantise_row(x)
    a = np.float64(sx) * scale.astype(np.float64) * (q @ X).astype(np.float64)
    e = nx * (r + 2.0 * K * 2.0 ** -24 * nW) + ndx * nWh + 1e-12 * np.abs(a) + 1e-30
    orders = [np.arange(K), np.arange(K)[::-1], rng.permutation(K)]
    for order in orders:
        L = fp32_dots(x, W, order).astype(np.float64)
        assert np.all(np.abs(L - a) <= e), float(np.max(np.abs(L - a) / e))

    def proc(v):  # repetition penalty on the seen ids, in fp32 after the bf16 rounding
        v = bf16(v).astype(np.float32)
        pv = np.where(v < 0, v * np.float32(penalty), v / np.float32(penalty)).astype(np.float32)
        return np.where(seen, pv, v)

    ub, lb = proc(a + e), proc(a - e)
    cand = ub >= lb.max()
    for order in orders:
        s = proc(fp32_dots(x, W, order))
        best = int(np.argmax(s))  # lowest index on ties
        assert cand[best] and np.all(s[~cand] < s[best])
    return int(cand.sum())


def test_bounds_hold_for_uniform_weights():
    rng = np.random.default_rng(1)
    W = rng.uniform(-0.05, 0.05, size=(V, K)).astype(np.float32)
    for t in range(3):
        x = rng.standard_normal(K).astype(np.float32) * np.float32(1.5)
        seen = rng.random(V) < 0.02
        n = check(W, x, seen, 1.1, rng)
        assert n < V // 20  # the screen keeps a small candidate set


def test_bounds_hold_for_heavy_tailed_weights():
    rng = np.random.default_rng(2)
    W = rng.standard_normal((V, K)).astype(np.float32) * np.float32(0.02)
    W[::7] *= 8
    mask = rng.random(W.shape) < 1.0 / 64
    W[mask] *= 40
    x = (rng.standard_t(3, K) * 0.7).astype(np.float32)  # heavy-tailed activations too
    seen = rng.random(V) < 0.05
    check(W, x, seen, 1.4, rng)


def test_exact_ties_stay_in_the_candidate_set():
    rng = np.random.default_rng(3)
    W = rng.uniform(-0.05, 0.05, size=(V, K)).astype(np.float32)
    W[1::2] = W[0::2]  # every score has an exact twin; the argmax must be the even one
    x = rng.standard_normal(K).astype(np.float32)
    check(W, x, np.zeros(V, bool), 1.0, rng)
