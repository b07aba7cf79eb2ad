// lm_attn_core.h — decode attention of one (sequence, kv head) on the matrix cores, shared by
// the standalone decode kernel (lm_attn.hip) and the attention workgroups fused into the
// one-row QKV launch (lm_gemm_kernel.h), so both produce bit-identical outputs.
//
// Reference numerics (transformers LlamaAttention + SDPA at decode, restated by
// oracle/lm_oracle.py:95-107): scores in fp32 from the roped bf16 q / k, scale D^-0.5,
// p = exp(s - max) with max over the WHOLE context, p rounded to bf16 for P.V, normaliser =
// fp32 sum of the unrounded p, o = (P.V) / l rounded to bf16.  The max and the sums are the
// reference's; only the fp32 summation order differs (products of bf16 operands are exact).
//
// KV cache of a layer: K [slot][kv head][S][D] (rows), V^T [slot][kv head] as tiles of 16
// dimensions x 32 positions (vt_off below), S = the position stride (a multiple of 64).  Both
// are the MFMA operand layouts below, so every fragment is ONE 16-byte load straight from HBM /
// L2 into registers (no LDS staging), and a wave's V^T fragment of one dimension tile is one
// contiguous KiB — eight whole 128-B lines (round 6: with V^T as plain [D][S] columns a head-dim
// 128 wave, 32 positions per pass, read half of each 128-B line and its neighbour wave the
// other half).
//
// Work split: NW waves; wave w owns positions base = (pass * NW + w) * PW .. + PW - 1 of each
// pass.  Per wave and pass:
//   S^T[pos][head] = K . Q^T  (v_mfma_f32_16x16x32_bf16; A = K rows, B = the group's four roped
//                              q heads, columns 4..15 duplicating heads 0..3).  The A rows of
//                              m-tile mt are positions pi(mt, row) = base + 32 (mt >> 1)
//                              + 8 (row >> 2) + 4 (mt & 1) + (row & 3), so that lane group g
//                              (lane >> 4) ends up holding positions base + 32 ps + 8 g + e,
//                              e = 0..7, of k-step ps in the accumulators of m-tiles 2ps, 2ps+1;
//   O^T[dim][head] += V^T . P^T (A = V^T: 8 consecutive positions of one dimension = one load;
//                              B = P^T straight from the S^T accumulators rounded to bf16).
// The maximum is taken over all waves first (LDS), then p, l and P.V; the waves' partial O
// and l are summed in wave order through LDS.
#pragma once
#include "hip_common.h"

namespace tts {

template <int D, int PW>
struct DecShape {
  static constexpr int MT = PW / 16;  // m-tiles of S^T per wave and pass
  static constexpr int KS = D / 32;   // k-steps of S^T
  static constexpr int PS = PW / 32;  // k-steps of P.V
  static constexpr int DT = D / 16;   // dimension tiles of O^T
};

constexpr int DEC_G = 4;  // q heads per kv head (GQA 4:1, TTS-1 and TTS-1-Max)
// Decode workgroup geometry: DEC_NW = 16 waves of dec_pw positions each per pass (head dim 64:
// 64 positions, 1,024 per pass; 128: 32 positions, 512 per pass — the fragments of a position
// are twice as wide, so half the positions keep the registers of the D = 64 wave).  Standalone
// and fused (QKV launch) attention share the geometry, hence the bits.
constexpr int DEC_NW = 16;
template <int D> constexpr int dec_nw() { return 16; }
template <int D> constexpr int dec_pw() { return D == 64 ? 64 : 32; }

// element (d, p) of a (slot, kv head) V^T block: tile (d / 16, p / 32) of 16 x 32 bf16, the 32
// positions of each dimension contiguous
TTS_DEV int vt_off(int S, int d, int p) {
  return (((d >> 4) * (S >> 5) + (p >> 5)) * 16 + (d & 15)) * 32 + (p & 31);
}

// position of A row `row` of m-tile mt (see pi above)
TTS_DEV int dec_pos(int base, int mt, int row) {
  return base + 32 * (mt >> 1) + 8 * (row >> 2) + 4 * (mt & 1) + (row & 3);
}

// One pass's fragments of this wave: kf = K rows (clamped to the last valid position; the
// rows past ctx are masked), vf = V^T columns (clamped inside the stride).  Unconditional
// loads: a fixed load count keeps the compiler's vmcnt waits exact.  O32: 32-bit element
// offsets inside the (slot, kv head) block (S * D < 2^31) — in the standalone kernel the 64-bit
// ones stayed live across the passes in register pairs and spilled; the fused consumer
// allocates best with the 64-bit form.  (Addresses only: the same bits either way.)
template <int D, int PW, bool O32 = false>
TTS_DEV void dec_load_k(const bf16_t* kc, int base, int ctx, int lane,
                        u32x4_t (&kf)[DecShape<D, PW>::MT][DecShape<D, PW>::KS]) {
  using C = DecShape<D, PW>;
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt) {
    const int p = min(dec_pos(base, mt, c), ctx - 1);
#pragma unroll
    for (int ks = 0; ks < C::KS; ++ks)
      kf[mt][ks] = O32 ? *(const u32x4_t*)(kc + (p * D + 32 * ks + 8 * g))
                       : *(const u32x4_t*)(kc + (size_t)p * D + 32 * ks + 8 * g);
  }
}
template <int D, int PW, bool O32 = false>
TTS_DEV void dec_load_v(const bf16_t* vtc, int S, int base, int lane,
                        u32x4_t (&vf)[DecShape<D, PW>::PS][DecShape<D, PW>::DT]) {
  using C = DecShape<D, PW>;
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int ps = 0; ps < C::PS; ++ps) {
    // (position blocks past the stride: clamped to the last one; those positions are masked)
    const int pb = min((base >> 5) + ps, (S >> 5) - 1);
    const int o0 = (pb * 16 + c) * 32 + 8 * g;  // (vt_off of (16 dt + c, 32 pb + 8 g) = o0 + 16 S dt)
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
      vf[ps][dt] = O32 ? *(const u32x4_t*)(vtc + (o0 + dt * 16 * S)) : *(const u32x4_t*)(vtc + o0 + (size_t)dt * 16 * S);
  }
}

// The new position (ctx - 1) is not in the cache yet: its roped k / its v (LDS, bf16) replace
// the stale row / column elements in the fragments; V elements past ctx are zeroed (their p is
// 0, and 0 * NaN from never-written memory would poison the sum).  Branch-free: the LDS values
// are read unconditionally and merged with bit masks (a select whose operand is a load is
// otherwise turned into a branch around the load, and every such branch also drains vmcnt).
TTS_DEV uint32_t bits_sel(uint32_t mask, uint32_t a, uint32_t b) { return (a & mask) | (b & ~mask); }
template <int D, int PW>
TTS_DEV void dec_patch_k(int base, int ctx, int lane, const bf16_t* knew,
                         u32x4_t (&kf)[DecShape<D, PW>::MT][DecShape<D, PW>::KS]) {
  using C = DecShape<D, PW>;
  const int c = lane & 15, g = lane >> 4, pn = ctx - 1;
  u32x4_t kn[C::KS];
#pragma unroll
  for (int ks = 0; ks < C::KS; ++ks) kn[ks] = *(const u32x4_t*)(knew + 32 * ks + 8 * g);
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt) {
    const uint32_t m = dec_pos(base, mt, c) == pn ? 0xffffffffu : 0u;
#pragma unroll
    for (int ks = 0; ks < C::KS; ++ks)
#pragma unroll
      for (int q = 0; q < 4; ++q) kf[mt][ks][q] = bits_sel(m, kn[ks][q], kf[mt][ks][q]);
  }
}
template <int D, int PW>
TTS_DEV void dec_patch_v(int base, int ctx, int lane, const bf16_t* vnew,
                         u32x4_t (&vf)[DecShape<D, PW>::PS][DecShape<D, PW>::DT]) {
  using C = DecShape<D, PW>;
  const int c = lane & 15, g = lane >> 4, pn = ctx - 1;
  uint32_t vn[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt) vn[dt] = vnew[16 * dt + c];
#pragma unroll
  for (int ps = 0; ps < C::PS; ++ps) {
    const int p0 = base + 32 * ps + 8 * g;
    // per 32-bit word e2 (elements 2 e2, 2 e2 + 1): keep mask and new-value mask
    uint32_t keep[4], put[4];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
      const int pl = p0 + 2 * e2, ph = pl + 1;
      keep[e2] = (pl < pn ? 0x0000ffffu : 0u) | (ph < pn ? 0xffff0000u : 0u);
      put[e2] = (pl == pn ? 0x0000ffffu : 0u) | (ph == pn ? 0xffff0000u : 0u);
    }
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
      const uint32_t nv = vn[dt] | (vn[dt] << 16);
#pragma unroll
      for (int e2 = 0; e2 < 4; ++e2) vf[ps][dt][e2] = (vf[ps][dt][e2] & keep[e2]) | (nv & put[e2]);
    }
  }
}

// q B fragment of k-step ks (roped q of the group's four heads, fp32 LDS holding bf16
// values; read at each use: registers are the scarce resource here, LDS reads are cheap)
template <int D>
TTS_DEV bf16x8_t dec_qfrag(const float* qs, int lane, int ks) {
  const int h = (lane & 15) & 3, g = lane >> 4;
  const float4 a = *(const float4*)(qs + h * D + 32 * ks + 8 * g);
  const float4 b = *(const float4*)(qs + h * D + 32 * ks + 8 * g + 4);
  const u32x4_t w = {pack_bf2(a.x, a.y), pack_bf2(a.z, a.w), pack_bf2(b.x, b.y), pack_bf2(b.z, b.w)};
  return __builtin_bit_cast(bf16x8_t, w);
}

// S^T of one pass (scaled, positions >= ctx at -inf)
template <int D, int PW>
TTS_DEV void dec_scores(const u32x4_t (&kf)[DecShape<D, PW>::MT][DecShape<D, PW>::KS], const float* qs,
                        int base, int ctx, float scale, int lane, f32x4_t (&s)[DecShape<D, PW>::MT]) {
  using C = DecShape<D, PW>;
  const int g = lane >> 4;
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt) s[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < C::KS; ++ks) {
    const bf16x8_t qb = dec_qfrag<D>(qs, lane, ks);
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt)
      s[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, kf[mt][ks]), qb, s[mt], 0, 0, 0);
  }
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) s[mt][r] = (dec_pos(base, mt, 4 * g + r) < ctx) ? s[mt][r] * scale : -INFINITY;
}

// p = exp(s - M), l += p, O^T += V^T . P^T (bf16 P)
template <int D, int PW>
TTS_DEV void dec_pv(float M, float& lsum, f32x4_t (&s)[DecShape<D, PW>::MT],
                    const u32x4_t (&vf)[DecShape<D, PW>::PS][DecShape<D, PW>::DT], f32x4_t (&o)[DecShape<D, PW>::DT]) {
  using C = DecShape<D, PW>;
#pragma unroll
  for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // exp as the hardware 2^x of (s - M) log2 e, as FlashAttention's kernels evaluate it (one
      // v_exp_f32; the libm expf is a ~20-instruction range reduction).  M is the finite
      // context maximum: a masked score gives 2^-inf = 0, no branch.
      const float p = __builtin_amdgcn_exp2f((s[mt][r] - M) * 1.44269504088896341f);
      lsum += p;
      s[mt][r] = p;
    }
#pragma unroll
  for (int ps = 0; ps < C::PS; ++ps) {
    const u32x4_t pw = {pack_bf2(s[2 * ps][0], s[2 * ps][1]), pack_bf2(s[2 * ps][2], s[2 * ps][3]),
                        pack_bf2(s[2 * ps + 1][0], s[2 * ps + 1][1]), pack_bf2(s[2 * ps + 1][2], s[2 * ps + 1][3])};
    const bf16x8_t pb = __builtin_bit_cast(bf16x8_t, pw);
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, vf[ps][dt]), pb, o[dt], 0, 0, 0);
  }
}

// LDS scratch of dec_attend (floats): wave maxima, wave sums, wave partial O
template <int D, int NW>
constexpr int dec_red_floats() { return NW * DEC_G * 2 + NW * DEC_G * D; }

// The whole attention of one (row, kv head) by the NW waves of the workgroup (called by every
// thread; contains barriers).  kf0 / vf0: this wave's pass-0 fragments, already issued (the
// callers load them before anything else).  qs: roped q [4][D] fp32 (LDS, visible); knew /
// vnew: the new position's roped k and v (LDS bf16, visible).  out: the group's four heads'
// output, bf16 [4][D] (row of attn_out at the group's first head).
// (general form: `wave` / `tid` = this wave's / thread's index among the NW attending waves,
// `bar` = a barrier over exactly those waves; dec_attend below: the whole workgroup)
template <int D, int PW, int NW, class Bar, bool O32 = false>
TTS_DEV void dec_attend_w(const bf16_t* kc, const bf16_t* vtc, int S, int ctx, float scale, const float* qs,
                          const bf16_t* knew, const bf16_t* vnew, float* red,
                          u32x4_t (&kf0)[DecShape<D, PW>::MT][DecShape<D, PW>::KS],
                          u32x4_t (&vf0)[DecShape<D, PW>::PS][DecShape<D, PW>::DT], bf16_t* out, int wave,
                          int tid, Bar bar, unsigned long long* stp = nullptr, uint64_t* gout = nullptr,
                          uint32_t gtag = 0) {
  using C = DecShape<D, PW>;
  const int lane = tid & 63;
  const int c = lane & 15, g = lane >> 4;
  const int npass = (ctx + NW * PW - 1) / (NW * PW);
  float* mred = red;                 // [NW][4]
  float* lred = red + NW * DEC_G;    // [NW][4]
  float* ored = lred + NW * DEC_G;   // [NW][4][D]
  const int base0 = wave * PW;

  // phase 1: the context maximum per head (pass 0 from the prefetched fragments, its scores
  // kept; later passes (contexts beyond NW * PW positions) reload K only)
  f32x4_t s0[C::MT];
  float mx = -INFINITY;
  if (base0 < ctx) {
    dec_patch_k<D, PW>(base0, ctx, lane, knew, kf0);
    dec_patch_v<D, PW>(base0, ctx, lane, vnew, vf0);
    dec_scores<D, PW>(kf0, qs, base0, ctx, scale, lane, s0);
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s0[mt][r]);
  }
  for (int ps = 1; ps < npass; ++ps) {
    const int base = (ps * NW + wave) * PW;
    if (base >= ctx) break;
    u32x4_t kf[C::MT][C::KS];
    dec_load_k<D, PW, O32>(kc, base, ctx, lane, kf);
    dec_patch_k<D, PW>(base, ctx, lane, knew, kf);
    f32x4_t s[C::MT];
    dec_scores<D, PW>(kf, qs, base, ctx, scale, lane, s);
#pragma unroll
    for (int mt = 0; mt < C::MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[mt][r]);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  if (lane < DEC_G) mred[wave * DEC_G + lane] = mx;
  bar();
  TTS_STAMP(stp, 5);
  float M = -INFINITY;
#pragma unroll
  for (int w = 0; w < NW; ++w) M = fmaxf(M, mred[w * DEC_G + (c & 3)]);

  // phase 2: p, l and P.V
  float lsum = 0.f;
  f32x4_t o[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt) o[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  if (base0 < ctx) dec_pv<D, PW>(M, lsum, s0, vf0, o);
  for (int ps = 1; ps < npass; ++ps) {
    const int base = (ps * NW + wave) * PW;
    if (base >= ctx) break;
    u32x4_t kf[C::MT][C::KS], vf[C::PS][C::DT];
    dec_load_v<D, PW, O32>(vtc, S, base, lane, vf);
    dec_load_k<D, PW, O32>(kc, base, ctx, lane, kf);
    dec_patch_k<D, PW>(base, ctx, lane, knew, kf);
    f32x4_t s[C::MT];
    dec_scores<D, PW>(kf, qs, base, ctx, scale, lane, s);
    dec_patch_v<D, PW>(base, ctx, lane, vnew, vf);
    dec_pv<D, PW>(M, lsum, s, vf, o);
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  // lane (c < 4, g) holds O^T[dim 16 dt + 4 g + r][head c]
  if (c < DEC_G) {
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
      *(float4*)(ored + (wave * DEC_G + c) * D + 16 * dt + 4 * g) = make_float4(o[dt][0], o[dt][1], o[dt][2], o[dt][3]);
    if (g == 0) lred[wave * DEC_G + c] = lsum;
  }
  bar();
  TTS_STAMP(stp, 6);
  bf16_t gob = 0;  // (granule output: this thread's element, i == tid: one iteration)
  for (int i = tid; i < DEC_G * D; i += NW * 64) {
    const int h = i / D, d = i - h * D;
    float v[NW];  // each group of reads in flight before its sums (wave order: deterministic)
#pragma unroll
    for (int w = 0; w < NW; ++w) v[w] = lred[w * DEC_G + h];
    float O = 0.f, L = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) L += v[w];
#pragma unroll
    for (int w = 0; w < NW; ++w) v[w] = ored[(w * DEC_G + h) * D + d];
#pragma unroll
    for (int w = 0; w < NW; ++w) O += v[w];
    const bf16_t ob = f2bf(O / L);
    out[h * D + d] = ob;
    if (gout) gob = ob;
  }
  if (gout) {  // the row as granules: pairs (d, d + 1) through LDS (the partials are read)
    bar();
    if (tid < DEC_G * D) ((bf16_t*)ored)[tid] = gob;
    bar();
    if (tid < DEC_G * D / 2)
      __hip_atomic_store(gout + tid, ((uint64_t)gtag << 32) | ((const uint32_t*)ored)[tid], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int D, int PW, int NW, bool O32 = false>
TTS_DEV void dec_attend(const bf16_t* kc, const bf16_t* vtc, int S, int ctx, float scale, const float* qs,
                        const bf16_t* knew, const bf16_t* vnew, float* red,
                        u32x4_t (&kf0)[DecShape<D, PW>::MT][DecShape<D, PW>::KS],
                        u32x4_t (&vf0)[DecShape<D, PW>::PS][DecShape<D, PW>::DT], bf16_t* out,
                        unsigned long long* stp = nullptr, uint64_t* gout = nullptr, uint32_t gtag = 0) {
  auto bar = [] { lds_barrier(); };
  dec_attend_w<D, PW, NW, decltype(bar), O32>(kc, vtc, S, ctx, scale, qs, knew, vnew, red, kf0, vf0, out,
                          __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), threadIdx.x, bar, stp, gout, gtag);
}

// RoPE of one element (HF apply_rotary_pos_emb in bf16: x*cos + rotate_half(x)*sin, each
// op rounded to bf16): x = element d, xr = element d +- D/2 (its rotate_half partner)
TTS_DEV float rope_elem(bf16_t x, bf16_t xr, bool lower_half, float c, float sn) {
  const float rot = lower_half ? -bf2f(xr) : bf2f(xr);
  return rbf(rbf(bf2f(x) * c) + rbf(rot * sn));
}

}  // namespace tts
