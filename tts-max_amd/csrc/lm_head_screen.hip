// lm_head_screen.hip — the greedy lm_head as an exact two-pass argmax over an int8 screen.
//
// The greedy pick (GenerationMixin._sample, generation/utils.py:2894-2925, driven by
// /root/reference/tts/inference/inferencing.py:94-107) needs only the argmax of the processed
// scores s_c = proc(bf16(x . W_c)) (proc = repetition penalty, frequency penalty, min-new EOS
// mask: monotone non-decreasing in the logit), not the 193,856 logits themselves.  The full
// bf16 lm_head streams V*K*2 bytes (794 MB for TTS-1) every step; here:
//
//  1. head_screen_kernel streams an int8 copy of the matrix (per-column scale, made once at
//     load: V*K bytes, half the bytes) and computes for every column an interval that provably
//     holds the exact fp32 logit L_c the bf16 kernel would compute:
//        a_c = sx*scale_c * (X . q_c)     (X = x / sx rounded to 16-bit integers, split into two
//                                          int8 rows hi*256 + lo: v_mfma_i32_16x16x64_i8 sums
//                                          them exactly)
//        |L_c - a_c| <= |L_c - x.W_c| + |x.(W_c - Wh_c)| + |(x - xh).Wh_c| + rounding of a_c
//                    <= gam*|x|*|W_c| + |x|*r_c + |x - xh|*|Wh_c| + tiny   =: e_c
//     (Cauchy-Schwarz; gam = 2*K*2^-24 bounds the fp32 accumulation of K bf16 products; r_c,
//     |W_c|, |Wh_c| are computed in double at load and rounded up; the fp32 roundings of a_c, e_c
//     and the sums are covered by relative margins).  It writes ub_c =
//     proc(bf16(a_c + e_c)) per (row, column) and the workgroup maximum of lb_c = proc(bf16(a_c
//     - e_c)).  Every argmax c* of the exact scores has ub_{c*} >= s_{c*} >= max_c lb_c =: LB.
//  2. head_recheck_kernel reduces LB, finds the 16-column tiles holding a column with ub >= LB
//     (a few dozen of 12,116 on TTS-1 weights) and recomputes those tiles exactly as the bf16
//     lm_head does — the same tiled weights, v_mfma_f32_16x16x32_bf16 over the k-tiles in
//     ascending order into one accumulator, the same epilogue — and writes argmax partials
//     (lowest index on ties) for finalize_greedy_kernel.
//
// So the chosen id is bit-for-bit the full lm_head's (tests/test_gpu_head_screen.py, and every
// greedy parity test runs through this path), whatever the weights: a loose bound only costs
// more recomputed tiles (all of them at worst).  Sampling (do_sample) needs every processed logit
// and keeps the full lm_head.  TTS_HEAD_SCREEN=0: the full lm_head for greedy steps too;
// TTS_HEAD_SCREEN_CHECK=1: every tile recomputed and checked against its bound (tests).
#include <math.h>

#include "hip_common.h"
#include "lm_kernels.h"

namespace tts {

typedef __attribute__((ext_vector_type(4))) int i32x4_t;

namespace {

constexpr int kScrWaves = 4;  // screen workgroup: 4 waves, one per SIMD
constexpr int kScrKU = 8;     // 1-KiB int8 blocks (64 k each) per stage
#ifndef TTS_SCR_R
#define TTS_SCR_R 2
#endif
constexpr int kScrR = TTS_SCR_R;  // stages in flight per wave (experiment builds: -DTTS_SCR_R=4)

// the float nearest a double, rounded up (bounds stay bounds)
TTS_DEV float f_up(double d) {
  float f = (float)d;
  if ((double)f < d) f = nextafterf(f, INFINITY);
  return f;
}
TTS_DEV double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// the maximum over the 16 lanes of each DPP row, in every lane (row_ror 1, 2, 4, 8: VALU speed)
TTS_DEV float row16_max(float v) {
  v = fmaxf(v, dpp_mov<0x121>(v, v));
  v = fmaxf(v, dpp_mov<0x122>(v, v));
  v = fmaxf(v, dpp_mov<0x124>(v, v));
  return fmaxf(v, dpp_mov<0x128>(v, v));
}

// head_proc for the screen's bounds, without the division: the penalty as a product with the
// reciprocal, then the result widened by 2^-21 of the magnitudes it came from (up for an upper
// bound, down for a lower one) — it stays on its side of head_proc's exact value (every rounding
// here is below 2^-22 of those magnitudes)
template <bool UP>
TTS_DEV float head_proc_bound(float v, uint32_t seen_word, int n, float penalty, float inv_penalty,
                              const uint16_t* counts_row, float freq, int eos) {
  const bool seen = (seen_word >> (n & 31)) & 1u;
  float mag = fabsf(v);
  if (seen) v = v * (v < 0.f ? penalty : inv_penalty);
  mag = fmaxf(mag, fabsf(v));
  if (counts_row) {
    const float sub = freq * (float)counts_row[n];
    v -= sub;
    mag += fabsf(sub) + fabsf(v);
  }
  v = UP ? v + mag * 0x1p-21f : v - mag * 0x1p-21f;
  return n == eos ? -INFINITY : v;
}

// The lm_head epilogue's processing of one bf16-rounded logit (lm_gemm_kernel.h EPI_LOGITS):
// repetition penalty on seen ids, frequency penalty, min-new EOS mask.  Monotone in v.
TTS_DEV float head_proc(float v, uint32_t seen_word, int n, float penalty, const uint16_t* counts_row,
                        float freq, int eos) {
  if ((seen_word >> (n & 31)) & 1u) v = (v < 0.f) ? v * penalty : v / penalty;
  if (counts_row) v -= freq * (float)counts_row[n];
  if (n == eos) v = -INFINITY;
  return v;
}

// ------------------------------------------------------------------ load-time quantiser --
// One wave per column c of the row-major [V][K] bf16 matrix: scale = max|W_c| / 127, q =
// rint(W / scale) in [-127, 127], written as the 1-KiB blocks the screen streams (block kb of
// unit c / 16 at plan_tile(1, 1, KU, ur, units, K / 64, 1, c / 16, kb); lane l of a block holds
// column l & 15, k = kb*64 + 16*(l >> 4) + j, j < 16), and cst[c] = {scale, |W - Wh|, |W|, |Wh|}
// (double sums, rounded up).
__global__ __launch_bounds__(256) void head_quant_kernel(const bf16_t* __restrict__ w, int V, int K, int ur,
                                                         int8_t* __restrict__ q, float4* __restrict__ cst) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= V) return;  // (wave-uniform)
  const bf16_t* wr = w + (size_t)c * K;
  const int units = V >> 4, KT8 = K >> 6, npc = K >> 4;  // 16-value pieces per column
  float mx = 0.f;
  for (int p = lane; p < npc; p += 64) {
    const u32x4_t* src = (const u32x4_t*)(wr + p * 16);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const u32x4_t v = src[h];
#pragma unroll
      for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fmaxf(fabsf(bf_lo(v[e])), fabsf(bf_hi(v[e]))));
    }
  }
  mx = wave_max_dpp(mx);
  const float scale = mx > 0.f ? mx / 127.f : 1.f;
  double r2 = 0.0, w2 = 0.0, h2 = 0.0;
  for (int p = lane; p < npc; p += 64) {
    const u32x4_t* src = (const u32x4_t*)(wr + p * 16);
    uint32_t packed[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const u32x4_t v = src[h];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x0 = bf_lo(v[e]), x1 = bf_hi(v[e]);
        const int q0 = max(-127, min(127, (int)rintf(x0 / scale)));
        const int q1 = max(-127, min(127, (int)rintf(x1 / scale)));
        const double d0 = (double)x0 - (double)scale * q0, d1 = (double)x1 - (double)scale * q1;
        const double h0 = (double)scale * q0, h1 = (double)scale * q1;
        r2 += d0 * d0 + d1 * d1;
        w2 += (double)x0 * x0 + (double)x1 * x1;
        h2 += h0 * h0 + h1 * h1;
        const int j = h * 8 + e * 2;  // value index within the 16-value piece
        const uint32_t b = ((uint32_t)(q0 & 0xff)) | ((uint32_t)(q1 & 0xff) << 8);
        if (j % 4 == 0) packed[j / 4] = b;
        else packed[j / 4] |= b << 16;
      }
    }
    const int kb = p >> 2, g = p & 3;
    const long long tile = plan_tile(1, 1, kScrKU, ur, units, KT8, 1, c >> 4, kb);
    *(u32x4_t*)(q + tile * 1024 + (16 * g + (c & 15)) * 16) = u32x4_t{packed[0], packed[1], packed[2], packed[3]};
  }
  r2 = wave_sum_f64(r2);
  w2 = wave_sum_f64(w2);
  h2 = wave_sum_f64(h2);
  if (lane == 0) {
    const double up = 1.0 + 1e-9;
    cst[c] = make_float4(scale, f_up(sqrt(r2) * up), f_up(sqrt(w2) * up), f_up(sqrt(h2) * up));
  }
}

// One normalised bf16 row (a wave, CPL 16-B chunks per lane, chunk j of lane l at k = 512 j + 8 l)
// as the screen's integer row: X = rint(x / sx), sx = max|x| / 32639, stored as the int8 rows
// hi (X = 256 hi + lo) and lo; nx >= |x|, ndx >= |x - sx X|.  (fp32 sums: their relative error,
// < K 2^-24, and the sqrt's are covered by the 2^-10 margin; d = x - sx X is one fma, exact to
// 2^-24 of itself; any X is valid: the bound uses the X taken)
template <int CPL>
TTS_DEV void quant_row(const u32x4_t (&v)[CPL], int lane, int8_t* hi_row, int8_t* lo_row, float& sx, float& nx,
                       float& ndx) {
  float mx = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) mx = fmaxf(mx, fmaxf(fabsf(bf_lo(v[j][q])), fabsf(bf_hi(v[j][q]))));
  mx = wave_max_dpp(mx);
  sx = mx > 0.f ? mx / 32639.f : 1.f;
  const float isx = 1.f / sx;
  float s2 = 0.f, d2 = 0.f;
#pragma unroll
  for (int j = 0; j < CPL; ++j) {
    uint32_t hw[2] = {0u, 0u}, lw[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = (e & 1) ? bf_hi(v[j][e >> 1]) : bf_lo(v[j][e >> 1]);
      const int X = max(-32639, min(32639, (int)rintf(x * isx)));
      const float d = fmaf(-sx, (float)X, x);
      s2 = fmaf(x, x, s2);
      d2 = fmaf(d, d, d2);
      const int hi = (X + 128) >> 8, lo = X - hi * 256;
      hw[e >> 2] |= (uint32_t)(hi & 0xff) << (8 * (e & 3));
      lw[e >> 2] |= (uint32_t)(lo & 0xff) << (8 * (e & 3));
    }
    const int k = j * 512 + lane * 8;
    *(uint2*)(hi_row + k) = make_uint2(hw[0], hw[1]);
    *(uint2*)(lo_row + k) = make_uint2(lw[0], lw[1]);
  }
  s2 = wave_sum_dpp(s2);
  d2 = wave_sum_dpp(d2);
  nx = sqrtf(s2) * (1.f + 0x1p-10f);
  ndx = sqrtf(d2) * (1.f + 0x1p-10f) + 1e-30f;
}

// ------------------------------------------------------------------------- the screen ----
// Workgroup = 4 waves; wave gw = blockIdx.x*4 + wave streams units gw, gw + ur, ... (ur = the
// layout's units per round = grid * 4): KT8 / 8 stages of 8 KiB per unit, two stages in flight
// (buffer loads, non-temporal; a refill past the wave's last unit reads out of range = zeros).
// Prologue: wave w takes rows w, w + 4, ... (RPW of them, loaded ahead of the weight stream so
// the stream is in flight while they are processed): RMSNorm (when a.normw) in the canonical
// order (chunk_sumsq, the wave DPP tree per 512 values, segments in order: the bits of every
// other RMSNorm path) into the bf16 rows Xl, then X = rint(x / sx), sx = max|x| / 32639, as two
// int8 A rows (2m: hi, 2m + 1: lo, X = 256 hi + lo) and |x|, |x - sx X| in double.
// Tail (the recheck): the workgroup's maxima of the lower bounds go into a per-row global
// maximum (64-bit atomic max of (decode step << 32 | order key): a value from an earlier step
// always loses, so the slots need no reset); after a bounded wait for every workgroup's bounds
// the maximum read back is the final LB (or, if the wait gave up, a lower bound of it), so the
// units flagged against it (their 16-column maximum of ub >= it) include every unit that can
// hold the argmax.  Each
// flagged unit is recomputed exactly as the bf16 lm_head does — its tiles, v_mfma_f32_16x16x32_bf16
// over the k-tiles in ascending order into one accumulator (wave w takes k-tiles w KT/4 .. and
// continues wave w - 1's accumulator through LDS), the same epilogue — and the workgroup writes
// its argmax partial (lowest index on ties) for finalize_greedy_kernel.
constexpr int kScrMaxUPW = 16;  // units a wave streams (host-checked: units <= 16 * ur)
#ifndef TTS_SCR_DB32
#define TTS_SCR_DB32 0
#endif
constexpr bool kScrDB32 = TTS_SCR_DB32;  // two flagged units in flight at K 4096 too (AGPRs hold the second): measured slower (165 -> 167 us at TTS-1-Max 8 rows), off
#ifdef TTS_SCR_PROBE
constexpr int kScrProbe = TTS_SCR_PROBE;  // timing probes only (scripts: wrong ids): 1 no MFMA, 2 no epilogue
#else
constexpr int kScrProbe = 0;
#endif

TTS_DEV uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
TTS_DEV float key2f(uint32_t k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k); }

// PRE (17..32 rows): the rows come normalised (a.x) and quantised by head_rowquant_kernel (a.xq,
// a.xstat: one pass instead of every workgroup quantising every row); the recompute then reads
// its A fragments from a.x (L2) instead of an LDS copy, and the int8 image takes the LDS
template <int MT, int KT8, int RPW, bool PRE>
__global__ __launch_bounds__(kScrWaves * 64) void head_screen_kernel(HeadScreenArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int K = KT8 * 64, ldA = K + 16, ldX = K + 8, KU = kScrKU, R = kScrR, S = KT8 / KU, CPL = K / 512;
  constexpr int MMAX = 8 * MT;  // rows of the int8 image (two A rows each)
  constexpr int MTB = PRE ? 2 : 1;  // 16-row m-tiles of the exact recompute
  static_assert(S % R == 0, "stages per unit must be a multiple of the ring depth");
  int8_t* Al = (int8_t*)smem;                                       // [16 MT][ldA] int8
  bf16_t* Xl = (bf16_t*)(smem + (size_t)16 * MT * ldA);             // [MMAX][ldX] normalised rows (!PRE)
  float* rsx = (float*)(Xl + (PRE ? 0 : (size_t)MMAX * ldX));       // [MMAX] sx
  float* rnx = rsx + MMAX;                                          // [MMAX] |x| (rounded up)
  float* rndx = rnx + MMAX;                                         // [MMAX] |x - sx X|
  float* rlb = rndx + MMAX;                                         // [waves][MMAX] lower-bound maxima
  float* LBc = rlb + kScrWaves * MMAX;                              // [MMAX] the global maximum read back
  float* umx = LBc + MMAX;                                          // [waves][kScrMaxUPW][MMAX] unit max of ub
  int* tl = (int*)(umx + kScrWaves * kScrMaxUPW * MMAX);            // [waves * kScrMaxUPW] flagged units
  int* ntl = tl + kScrWaves * kScrMaxUPW;
  f32x4_t* xacc = (f32x4_t*)(ntl + 4);                              // [MTB][64] chain hand-off (16-B aligned)
  const int M = a.M, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g4 = lane >> 4, col = lane & 15;

  // ---- the rows (and the norm weight) first, then the weight stream
  constexpr int XQJ = PRE ? 2 * MMAX * K / 16 / (kScrWaves * 64) : 1;  // PRE: 16-B pieces of the image per thread
  u32x4_t xv[PRE ? 1 : RPW][CPL], gv[CPL], xq[XQJ];
  float st3[3] = {1.f, 0.f, 0.f};
  if constexpr (PRE) {
#pragma unroll
    for (int j = 0; j < XQJ; ++j) {  // (rows past 2M: the last row again, never used)
      const int c = tid + j * kScrWaves * 64, row = min(c / (K / 16), 2 * M - 1);
      xq[j] = *(const u32x4_t*)(a.xq + (size_t)row * K + (c % (K / 16)) * 16);
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) st3[q] = a.xstat[min(tid, M - 1) * 4 + q];
  } else {
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const bf16_t* xr = a.x + (size_t)min(wave + 4 * r, M - 1) * a.ldx;
#pragma unroll
      for (int j = 0; j < CPL; ++j) xv[r][j] = *(const u32x4_t*)(xr + j * 512 + lane * 8);
    }
    const bf16_t* nw = a.normw ? a.normw : a.x;  // (unconditional loads: exact vmcnt waits)
#pragma unroll
    for (int j = 0; j < CPL; ++j) gv[j] = *(const u32x4_t*)(nw + j * 512 + lane * 8);
  }

  int eosr[MT][2];  // the rows' EOS masks (every unit's epilogue)
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int p = 0; p < 2; ++p) eosr[mt][p] = a.eos_mask[min(8 * mt + 2 * g4 + p, M - 1)];

  const int units = a.V >> 4, ur = a.ur;
  const int gw = blockIdx.x * kScrWaves + wave;
  const uint32_t qbytes = (uint32_t)((long long)units * KT8 * 1024);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)a.q, (short)0, (int)qbytes, 0x00020000);
  constexpr uint32_t kPast = kWgemmSentinel - (uint32_t)(KU - 1) * 1024u;
  u32x4_t wr[R][KU];
  int pu = gw, ps = 0;
  auto issue = [&](u32x4_t (&dst)[KU]) {
    const uint32_t o = pu < units ? (uint32_t)plan_tile(1, 1, KU, ur, units, KT8, 1, pu, ps * KU) * 1024u + lane * 16u
                                  : kPast;
#pragma unroll
    for (int kk = 0; kk < KU; ++kk) dst[kk] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(o + kk * 1024u), 0, 2);
    if (++ps == S) { ps = 0; pu += ur; }
  };
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < R; ++j) issue(wr[j]);
  __builtin_amdgcn_sched_barrier(0);

  if constexpr (PRE) {
#pragma unroll
    for (int j = 0; j < XQJ; ++j) {
      const int c = tid + j * kScrWaves * 64, row = c / (K / 16);
      if (row < 2 * M) *(u32x4_t*)(Al + (size_t)row * ldA + (c % (K / 16)) * 16) = xq[j];
    }
    if (tid < M) { rsx[tid] = st3[0]; rnx[tid] = st3[1]; rndx[tid] = st3[2]; }
  }
#pragma unroll
  for (int r = 0; r < (PRE ? 0 : RPW); ++r) {
    const int m = wave + 4 * r;
    if (m < M) {  // (wave-uniform)
      u32x4_t (&v)[CPL] = xv[r];
      if (a.normw) {
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < CPL; ++j) ss += wave_sum_dpp(chunk_sumsq(v[j]));
        const float rr = 1.0f / sqrtf(ss / (float)K + a.eps);
#pragma unroll
        for (int j = 0; j < CPL; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            v[j][q] = pack_bf2(bf_lo(gv[j][q]) * rbf(bf_lo(v[j][q]) * rr), bf_hi(gv[j][q]) * rbf(bf_hi(v[j][q]) * rr));
      }
#pragma unroll
      for (int j = 0; j < CPL; ++j) *(u32x4_t*)(Xl + (size_t)m * ldX + j * 512 + lane * 8) = v[j];
      float sx, nx, ndx;
      quant_row<CPL>(v, lane, Al + (size_t)(2 * m) * ldA, Al + (size_t)(2 * m + 1) * ldA, sx, nx, ndx);
      if (lane == 0) { rsx[m] = sx; rnx[m] = nx; rndx[m] = ndx; }
    }
  }
  lds_barrier();  // (LDS only: the weight stream stays in flight)

  const float gam = 2.f * K / 16777216.f, inv_pen = 1.f / a.penalty;
  float lbm[MT][2];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) lbm[mt][0] = lbm[mt][1] = -INFINITY;
  int nu = 0;  // units this wave streamed
  for (int u = gw; u < units; u += ur, ++nu) {
    // (the A fragments are the same for every unit: one m-tile at K 2048 keeps them in registers
    // across units, 128 VGPRs; larger images are re-read from LDS per unit, not hoisted)
    int aoff = 0;
    if constexpr (MT * KT8 > 32 || kScrR > 2) asm volatile("" : "+v"(aoff));
    // this unit's epilogue operands, issued behind its first stages and ahead of their refills
    const int c = u * 16 + col;
    const float4 cs = a.cst[c];
    uint32_t sw[MT][2];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int p = 0; p < 2; ++p) sw[mt][p] = a.seen[(size_t)min(8 * mt + 2 * g4 + p, M - 1) * a.seen_stride + (c >> 5)];
    i32x4_t acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = i32x4_t{0, 0, 0, 0};
#pragma unroll
    for (int st = 0; st < S; st += R) {
#pragma unroll
      for (int j = 0; j < R; ++j) {
#pragma unroll
        for (int kk = 0; kk < KU; ++kk) {
          const int kb = (st + j) * KU + kk;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            if constexpr (kScrProbe & 1) {  // (probe build: no A reads, no MFMA)
              acc[mt][0] ^= (int)wr[j][kk][0];
            } else {
              const i32x4_t af = *(const i32x4_t*)(Al + aoff + (16 * mt + col) * ldA + kb * 64 + 16 * g4);
              acc[mt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, __builtin_bit_cast(i32x4_t, wr[j][kk]), acc[mt], 0, 0, 0);
            }
          }
        }
        issue(wr[j]);
      }
    }
    // rows 8 mt + 2 g4 + p: acc[2p] = hi . q, acc[2p + 1] = lo . q
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int m = 8 * mt + 2 * g4 + p;
        float ub = -INFINITY;
        if (kScrProbe & 2) {  // (probe build: no per-unit epilogue)
          if (acc[mt][0] == 12345) a.part_val[0] = 0.f;
          continue;
        }
        if (m < M) {
          // fp32, every rounding covered: av is within 3 roundings (< 2^-22 |av|) of sx scale (X.q),
          // e within 2^-22 of its value; the margins (2^-21 |av|, e (1 + 2^-20)) also cover the
          // final sums' roundings, so ub / lb stay outside [L - true e, L + true e]
          // (X.q = 256 hi.q + lo.q; the two int -> fp32 conversions and the fma round to within
          // 2^-23 (256 |hi.q| + |lo.q|), a term of its own: they may cancel)
          const float hq = (float)acc[mt][2 * p], lq = (float)acc[mt][2 * p + 1];
          const float Sf = fmaf(hq, 256.f, lq);
          const float av = Sf * rsx[m] * cs.x;
          const float e = fmaf(rnx[m], fmaf(gam, cs.z, cs.y), rndx[m] * cs.w) * (1.f + 0x1p-20f) +
                          (fabsf(av) + fmaf(fabsf(hq), 256.f, fabsf(lq)) * rsx[m] * cs.x) * 0x1p-21f + 1e-30f;
          const uint16_t* crow = a.counts ? a.counts + (size_t)m * a.seen_stride * 32 : nullptr;
          ub = head_proc_bound<true>(rbf(av + e), sw[mt][p], c, a.penalty, inv_pen, crow, a.freq_penalty, eosr[mt][p]);
          const float lb =
              head_proc_bound<false>(rbf(av - e), sw[mt][p], c, a.penalty, inv_pen, crow, a.freq_penalty, eosr[mt][p]);
          if (a.ub) a.ub[(size_t)m * a.ldu + c] = ub;  // (check mode)
          lbm[mt][p] = fmaxf(lbm[mt][p], lb);
        }
        // the unit's maximum of ub per row (its 16 columns = the 16 lanes of the group)
        ub = row16_max(ub);
        if (col == 0 && nu < kScrMaxUPW) umx[(wave * kScrMaxUPW + nu) * MMAX + m] = ub;
      }
  }

  // ---- tail: this workgroup's lower bounds into the global maximum, read back
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) lbm[mt][p] = fmaxf(lbm[mt][p], __shfl_xor(lbm[mt][p], o, 64));
      if (col == 0) rlb[wave * MMAX + 8 * mt + 2 * g4 + p] = lbm[mt][p];
    }
  if (tid == 0) *ntl = 0;
  if (a.check) __threadfence();  // (check mode reads the ub values other waves stored)
  __syncthreads();  // (the stream has ended: nothing in flight to keep)
  // Bounds and arrivals go to one of 8 shards (workgroup b to shard b % 8: 32 workgroups per
  // address at 256 — atomics that all workgroups aim at ONE address serialise, ~25 ns each)
  const unsigned long long ep = (unsigned long long)*a.epoch;
  const int shard = blockIdx.x & 7;
  if (tid < M) {
    float v = rlb[tid];
#pragma unroll
    for (int w = 1; w < kScrWaves; ++w) v = fmaxf(v, rlb[w * MMAX + tid]);
    const unsigned long long mine = (ep << 32) | f2key(v);
    const unsigned long long old =
        __hip_atomic_fetch_max(a.lbg + tid * 8 + shard, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long cur = old > mine ? old : mine;
    LBc[tid] = key2f((uint32_t)cur);  // (cur's step is this one: mine is, and nothing later exists)
  }
  __syncthreads();
  // Wait (bounded; a.spins = 0: not at all) until every workgroup of the launch has added its
  // bounds, so the units are flagged against the final LB (the exact candidate set).  The
  // arrival counters only grow: a launch adds exactly gridDim.x / 8 to each, so this launch's
  // arrivals end at the next multiple of that.  A wait that gives up (a workgroup not yet
  // resident: nothing guarantees co-residency) keeps the maximum it has, a lower bound of the
  // final LB — more units recomputed, the same pick.  (Relaxed: the only data read behind the
  // wait are the bounds, themselves agent-scope atomics; an acquire per poll would invalidate
  // the XCD's L2 at every poll.)
  if (a.spins > 0 && tid < 64) {
    const uint32_t per = gridDim.x >> 3;
    uint32_t target = 0;
    if (tid == 0) {
      const uint32_t old = __hip_atomic_fetch_add(a.arrive + shard * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      target = (old / per + 1) * per;
    }
    target = __shfl(target, 0, 64);
    const uint32_t* ctr = a.arrive + (lane & 7) * 16;
    for (int n = 0; n < a.spins; ++n) {
      const bool ok = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target < 0x80000000u;
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (tid < M * 8) {  // (also without the wait: the other shards' maxima so far cut the recompute,
    const int m = tid >> 3;  //  one row 75 -> 68 us, profiles/r6am_ab_shardread_1.txt)
    const unsigned long long cur = __hip_atomic_load(a.lbg + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float v = (cur >> 32) == ep ? key2f((uint32_t)cur) : -INFINITY;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    if ((tid & 7) == 0) LBc[m] = fmaxf(LBc[m], v);
  }
  __syncthreads();
  // flag this workgroup's units: (wave w, its i-th unit) where some row's ub reaches LBc
  if (tid < kScrWaves * kScrMaxUPW) {
    const int w = tid / kScrMaxUPW, i = tid % kScrMaxUPW;
    const int u = (blockIdx.x * kScrWaves + w) + i * ur;
    bool f = false;
    if (u < units) {
      if (a.check) f = true;
      for (int m = 0; m < M; ++m) f = f || umx[(w * kScrMaxUPW + i) * MMAX + m] >= LBc[m];
    }
    if (f) tl[atomicAdd(ntl, 1)] = u;
  }
  __syncthreads();

  // ---- exact recompute of the flagged units (MTB 16-row m-tiles)
  constexpr int KT = K / 32, KTW = KT / kScrWaves;
  const int nflag = (a.diag & 1) ? 0 : *ntl;  // (diag 1: timing probe without the recompute)
  if ((a.diag & 2) && tid == 0) atomicAdd(a.err + 2, *ntl);  // (diag 2: count the flagged units)
  float bv[MTB][4];
  int bi[MTB][4];
#pragma unroll
  for (int mb = 0; mb < MTB; ++mb)
#pragma unroll
    for (int r = 0; r < 4; ++r) { bv[mb][r] = -INFINITY; bi[mb][r] = 0x7fffffff; }
  // this wave's k-tiles of unit t (the lm_head layout: plan_tile(1, 1, hku, hur, units, KT, hkc))
  auto load = [&](u32x4_t (&wf)[KTW], int t) {
#pragma unroll
    for (int j = 0; j < KTW; ++j) {
      const int kt = wave * KTW + j;
      const int KTc = KT / a.hkc, ch = kt / KTc, ki = kt - ch * KTc;
      const int st = ch * (KTc / a.hku) + ki / a.hku, kk = ki % a.hku;
      const int rr = t / a.hur, ui = t - rr * a.hur, nr = min(units - rr * a.hur, a.hur);
      const int tile = rr * a.hur * KT + (st * nr + ui) * a.hku + kk;
      wf[j] = __builtin_nontemporal_load((const u32x4_t*)a.w + (size_t)tile * 64 + lane);
    }
  };
  // A fragments of this wave's k-tiles: the LDS rows, or (PRE) the normalised rows in global memory
  // (the same for every unit: loaded once)
  u32x4_t axg[PRE ? MTB : 1][PRE ? KTW : 1];
  if constexpr (PRE) {
#pragma unroll
    for (int mb = 0; mb < MTB; ++mb)
#pragma unroll
      for (int j = 0; j < KTW; ++j)
        axg[mb][j] = *(const u32x4_t*)(a.x + (size_t)min(16 * mb + col, M - 1) * a.ldx + (wave * KTW + j) * 32 + 8 * g4);
  }
  const bf16_t* xrow = Xl + (size_t)min(col, M - 1) * ldX + 8 * g4;
  auto chain = [&](const u32x4_t (&wf)[KTW], int t) {
    f32x4_t acc4[MTB];
#pragma unroll
    for (int mb = 0; mb < MTB; ++mb) acc4[mb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < kScrWaves; ++s) {
      if (wave == s) {
#pragma unroll
        for (int mb = 0; mb < MTB; ++mb)
          if (s > 0) acc4[mb] = xacc[mb * 64 + lane];
#pragma unroll
        for (int j = 0; j < KTW; ++j)
#pragma unroll
          for (int mb = 0; mb < MTB; ++mb) {
            u32x4_t av;
            if constexpr (PRE) av = axg[mb][j];
            else av = *(const u32x4_t*)(xrow + (s * KTW + j) * 32);
            acc4[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, av),
                                                               __builtin_bit_cast(bf16x8_t, wf[j]), acc4[mb], 0, 0, 0);
          }
        if (s < kScrWaves - 1) {
#pragma unroll
          for (int mb = 0; mb < MTB; ++mb) xacc[mb * 64 + lane] = acc4[mb];
        }
      }
      lds_barrier();
    }
    if (wave == kScrWaves - 1) {
      const int n = t * 16 + col;
#pragma unroll
      for (int mb = 0; mb < MTB; ++mb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * mb + 4 * g4 + r;
          if (m < M) {
            const uint16_t* crow = a.counts ? a.counts + (size_t)m * a.seen_stride * 32 : nullptr;
            const float v = head_proc(rbf(acc4[mb][r]), a.seen[(size_t)m * a.seen_stride + (n >> 5)], n, a.penalty,
                                      crow, a.freq_penalty, a.eos_mask[m]);
            if (a.check && !(v <= a.ub[(size_t)m * a.ldu + n]) && v == v)
              __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v > bv[mb][r] || (v == bv[mb][r] && n < bi[mb][r])) { bv[mb][r] = v; bi[mb][r] = n; }
          }
        }
    }
  };
  if constexpr (!PRE && (KTW <= 16 || kScrDB32)) {
    // two units in flight: the next flagged unit's tiles load while this one's chain runs (the
    // loads are unconditional — an index past the list repeats the last unit, never used — so
    // the chain's waits count only its own loads)
    u32x4_t wa[KTW], wb[KTW];
    if (nflag > 0) load(wa, tl[0]);
    for (int f = 0; f < nflag; f += 2) {
      load(wb, tl[min(f + 1, nflag - 1)]);
      chain(wa, tl[f]);
      if (f + 1 < nflag) {
        load(wa, tl[min(f + 2, nflag - 1)]);
        chain(wb, tl[f + 1]);
      }
    }
  } else {
    u32x4_t wa[KTW];
    for (int f = 0; f < nflag; ++f) {
      load(wa, tl[f]);
      chain(wa, tl[f]);
    }
  }
  if (wave == kScrWaves - 1) {
#pragma unroll
    for (int mb = 0; mb < MTB; ++mb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          const float v2 = __shfl_xor(bv[mb][r], o, 64);
          const int i2 = __shfl_xor(bi[mb][r], o, 64);
          if (v2 > bv[mb][r] || (v2 == bv[mb][r] && i2 < bi[mb][r])) { bv[mb][r] = v2; bi[mb][r] = i2; }
        }
        const int m = 16 * mb + 4 * g4 + r;
        if (col == 0 && m < M) {
          a.part_val[(size_t)m * a.part_stride + blockIdx.x] = bv[mb][r];
          a.part_idx[(size_t)m * a.part_stride + blockIdx.x] = bi[mb][r];
        }
      }
  }
}

// One wave per row of normalised bf16 rows (17..32-row screen, PRE): X = rint(x / sx), sx =
// max|x| / 32639, as the int8 rows 2m (hi) and 2m + 1 (lo) of xq [2M][K], and xstat[m] = {sx,
// |x| (up), |x - sx X| (up), 0} — the screen prologue's arithmetic, once per row
template <int CPL>
__global__ __launch_bounds__(256) void head_rowquant_kernel(const bf16_t* __restrict__ x, int ldx, int M,
                                                            int8_t* __restrict__ xq, float* __restrict__ xstat) {
  constexpr int K = CPL * 512;
  const int lane = threadIdx.x & 63, m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;  // (wave-uniform)
  u32x4_t v[CPL];
#pragma unroll
  for (int j = 0; j < CPL; ++j) v[j] = *(const u32x4_t*)(x + (size_t)m * ldx + j * 512 + lane * 8);
  float sx, nx, ndx;
  quant_row<CPL>(v, lane, xq + (size_t)(2 * m) * K, xq + (size_t)(2 * m + 1) * K, sx, nx, ndx);
  if (lane == 0) *(float4*)(xstat + m * 4) = make_float4(sx, nx, ndx, 0.f);
}

}  // namespace

// rows the screen takes: K 2048 up to 16 rows with the rows normalised and quantised in the
// prologue (the int8 image + the bf16 rows share the LDS), 17..32 pre-quantised (PRE: the int8
// image alone); K 4096 up to 8
static int scr_mt(int M) { return M <= 8 ? 1 : (M <= 16 ? 2 : 4); }
static size_t scr_lds(int M, int K) {
  const int mt = scr_mt(M), mm = 8 * mt;
  const bool pre = M > 16;
  return (size_t)16 * mt * (K + 16) + (pre ? 0 : (size_t)mm * (K + 8) * 2) +
         4 * ((size_t)mm * (4 + kScrWaves) + (size_t)kScrWaves * kScrMaxUPW * mm + kScrWaves * kScrMaxUPW + 4) +
         2 * 64 * 16 + 16;
}

bool head_screen_supported(int M, int K, int V) {
  return M >= 1 && M <= (K == 2048 ? 32 : 16) && (K == 2048 || K == 4096) && V % 16 == 0 && V >= 4096 &&
         (long long)V * K <= (long long)kWgemmMaxBytes && scr_lds(M, K) <= 160 * 1024;
}
bool head_screen_prequant(int M) { return M > 16; }
int head_screen_waves() { return kScrWaves; }

void launch_head_quant(const bf16_t* w, int V, int K, int ur, int8_t* q, float* cst, hipStream_t s) {
  if (dry_record("head_quant_kernel")) return;
  hipLaunchKernelGGL(head_quant_kernel, dim3((V + 3) / 4), dim3(256), 0, s, w, V, K, ur, q, (float4*)cst);
}

void launch_head_rowquant(const bf16_t* x, int ldx, int M, int K, int8_t* xq, float* xstat, hipStream_t s) {
  if (K != 2048) throw std::runtime_error("head row quantiser: K 2048 only");
  if (dry_record("head_rowquant_kernel")) return;
  hipLaunchKernelGGL((head_rowquant_kernel<4>), dim3((M + 3) / 4), dim3(256), 0, s, x, ldx, M, xq, xstat);
}

void launch_head_screen(const HeadScreenArgs& a, int grid, hipStream_t s) {
  const bool pre = head_screen_prequant(a.M);
  if (!head_screen_supported(a.M, a.K, a.V) || a.ur != grid * kScrWaves || (a.V / 16) > kScrMaxUPW * a.ur ||
      a.hKT != a.K / 32 || grid > LOGITS_MAX_PARTS || (pre && (a.K != 2048 || a.normw)))
    throw std::runtime_error("head screen: unsupported shape");
  const int mt = scr_mt(a.M), rpw = (a.M + kScrWaves - 1) / kScrWaves;
  const int rp = pre ? 1 : (rpw <= 1 ? 1 : (rpw <= 2 ? 2 : 4));
  if (dry_record("head_screen_kernel<" + std::to_string(mt) + ", " + std::to_string(a.K / 64) + ", " +
                 std::to_string(rp) + ", " + (pre ? "true" : "false") + ">"))
    return;
  if (!a.epoch || !a.lbg || !a.arrive || (a.check && !(a.ub && a.err)) || (pre && !(a.xq && a.xstat)))
    throw std::runtime_error("head screen: missing workspace");
  const size_t lds = scr_lds(a.M, a.K);
  HeadScreenArgs b = a;
  if (grid % 8) b.spins = 0;  // (the wait's 8 arrival shards need equal shares of the grid)
#define TTS_SCR(MT_, KT8_, RP_, PRE_) \
  hipLaunchKernelGGL((head_screen_kernel<MT_, KT8_, RP_, PRE_>), dim3(grid), dim3(kScrWaves * 64), lds, s, b)
  if (a.K == 2048) {
    if (pre) TTS_SCR(4, 32, 1, true);
    else if (rp == 1) TTS_SCR(1, 32, 1, false);
    else if (rp == 2) TTS_SCR(1, 32, 2, false);
    else TTS_SCR(2, 32, 4, false);
  } else {
    if (rp == 1) TTS_SCR(1, 64, 1, false); else if (rp == 2) TTS_SCR(1, 64, 2, false); else TTS_SCR(2, 64, 4, false);
  }
#undef TTS_SCR
}

}  // namespace tts
