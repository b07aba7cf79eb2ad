// lm_gemm_kernel.h — the weight-streaming GEMM kernel template and its launch shapes,
// instantiated per epilogue in lm_gemm_{store,resid,swiglu,logits}.hip (parallel builds).
// See lm_gemm.hip for the design notes, the weight layout and the stream plans.
#pragma once
#include <algorithm>
#include <cstdio>
#include <stdexcept>
#include <type_traits>

#include "hip_common.h"
#include "lm_kernels.h"
#include "lm_attn_core.h"

namespace tts {

// register budget of the early prologue: A chunks per thread
constexpr int wgemm_ea(int waves) { return waves >= 16 ? 1 : (waves >= 8 ? 2 : 4); }
// floats of the kernel's scratch region `red`: split-K partials of the waves with kpart > 0,
// the lm_head argmax exchange, the early RMSNorm segment sums (+64 slack)
__host__ __device__ inline int wgemm_red_floats(int waves, int ksplit, int ng, int mt, int M, int Kl) {
  const int upw = waves / ksplit;
  int r = upw * (ksplit - 1) * ng * mt * 4 * 64;
  r = r > upw * mt * 16 * 2 ? r : upw * mt * 16 * 2;
  const int segs = (M * (Kl / 8) + 63) / 64;
  r = r > segs ? r : segs;
  r = r > Kl / 2 ? r : Kl / 2;  // RMSNorm weight (bf16) parked here during the LDS-DMA prologue
  return r + 64;
}

// ------------------------------------------------- attention fused into the QKV launch -----
// One appended workgroup per (row, kv head) of the one-row decode step: its 16 waves issue
// their first-pass K / V^T fragment loads at entry, while the projection workgroups still
// stream the QKV weights; then threads poll the granules of the group's q and of the new k,
// v until their tag is this launch's, and the attention runs exactly as attn_decode_kernel's
// (lm_attn_core.h dec_attend: same waves, same order, same bits), writing the group's four
// heads of the bf16 attention row (fa.out) that o_proj then reads as a plain A row.
// the head dim a fused QKV shape carries (one consumer per instantiation keeps the registers
// of the other out of it): KU 2 = TTS-1's QKV (K 2048, head dim 64), KU 4 = TTS-1-Max's (K 4096, 128)
constexpr int wgemm_fattn_d(int ku) { return ku == 2 ? 64 : 128; }
template <int D>
constexpr size_t fattn_lds_bytes() {
  return (size_t)DEC_G * D * 4 + (DEC_G * D / 2 + D) * 4 + 2 * D * 2 + (size_t)dec_red_floats<D, DEC_NW>() * 4;
}
// A bounded granule wait: polls until `ready()` or `spins` polls; on timeout it sets the error
// flag, and every later wait (this launch or the following ones) that finds the flag set
// (checked every 512 polls, so never on a wait that succeeds quickly) gives up at once — a
// failure costs one timeout, then the results are garbage and the host raises at the next read
template <typename Poll>
TTS_DEV bool fattn_wait(Poll ready, int* err, int spins, bool report) {
  for (int n = 1; !ready(); ++n) {
    if (n > spins) {
      if (report) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    if ((n & 511) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// The residual epilogue's half of the hand-off: lane holds the updated bf16 value of column n
// of row m (rows differ by lane group only, so a lane and its neighbour lane ^ 1 hold the same
// row's columns n and n ^ 1); even lanes publish the pair {tag, (n + 1, n)} with one agent-scope
// 8-byte store.  Called by every lane of the wave (the shuffle); `pub` = this lane's value is a
// real output (row < M, the lane's column half)
TTS_DEV void publish_pair(uint64_t* gran_row, int n, bf16_t val, uint32_t tag, bool pub) {
  const uint32_t mine = (uint32_t)val;
  const uint32_t other = (uint32_t)__shfl_xor((int)mine, 1, 64);
  if (pub && !(n & 1))
    __hip_atomic_store(gran_row + (n >> 1), ((uint64_t)tag << 32) | (other << 16) | mine, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

template <int NT, int D>
TTS_DEV void fattn_consumer(const WgemmArgs& wa, char* smem, int b) {
  static_assert(NT == DEC_NW * 64, "the fused attention runs on 16-wave workgroups");
  constexpr int PW = dec_pw<D>(), G = DEC_G, H2 = D / 2;
  using C = DecShape<D, PW>;
  const AttnArgs& a = wa.fa;
  float* qs = (float*)smem;                   // [G][D] roped q
  uint32_t* raw = (uint32_t*)(qs + G * D);    // q pairs [G*D/2] | k pairs [D/2] | v pairs [D/2]
  const bf16_t* rawb = (const bf16_t*)raw;
  bf16_t* knew = (bf16_t*)(raw + G * D / 2 + D);
  bf16_t* vnew = knew + D;
  float* red = (float*)(vnew + D);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row = b / a.KVH, kvh = b % a.KVH;
  const int slot = a.row_slot[row], pos = a.row_pos[row], ctx = pos + 1;
  const size_t kvbase = ((size_t)slot * a.KVH + kvh) * a.max_seq * D;
  const bf16_t* kc = a.kcache + kvbase;
  const bf16_t* vtc = a.vtcache + kvbase;
  unsigned long long* stp = wa.stamps ? wa.stamps + (size_t)blockIdx.x * 32 : nullptr;
  TTS_STAMP(stp, 0);
  u32x4_t kf[C::MT][C::KS], vf[C::PS][C::DT];
  if (wave * PW < ctx) {
    dec_load_k<D, PW>(kc, wave * PW, ctx, lane, kf);
    dec_load_v<D, PW>(vtc, a.max_seq, wave * PW, lane, vf);
  }
  const int qd = tid % D;
  const float qc = bf2f(a.rope_cos[(size_t)pos * D + qd]), qsn = bf2f(a.rope_sin[(size_t)pos * D + qd]);

  // wait for the projection's granules of this kv group: q of its G heads, the new k and v
  const uint32_t tag = ((uint32_t)pos << 6) | (uint32_t)wa.fattn_layer;
  const int nq = G * D / 2, ngr = nq + D;
  if (tid < ngr) {
    int col;
    if (tid < nq) col = kvh * G * D + 2 * tid;
    else if (tid < nq + D / 2) col = a.H * D + kvh * D + 2 * (tid - nq);
    else col = a.H * D + a.KVH * D + kvh * D + 2 * (tid - nq - D / 2);
    const uint64_t* gp = wa.gran + (size_t)row * (a.ld_qkv / 2) + col / 2;
    uint64_t v;
    fattn_wait([&] {
      v = __hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return (uint32_t)(v >> 32) == tag;
    }, wa.fattn_err, wa.fattn_spins, true);
    raw[tid] = (uint32_t)v;
  }
  lds_barrier();
  TTS_STAMP(stp, 1);
  // RoPE of the group's q heads and of the new k (HF apply_rotary_pos_emb in bf16)
  if (tid < G * D) {
    const int g = tid / D;
    qs[tid] = rope_elem(rawb[tid], rawb[g * D + (qd < H2 ? qd + H2 : qd - H2)], qd < H2, qc, qsn);
  } else if (tid < G * D + D) {
    const int d = tid - G * D;
    knew[d] = f2bf(rope_elem(rawb[G * D + d], rawb[G * D + (d < H2 ? d + H2 : d - H2)], d < H2, qc, qsn));
    vnew[d] = rawb[G * D + D + d];
  }
  lds_barrier();
  TTS_STAMP(stp, 2);
  dec_attend<D, PW, DEC_NW>(kc, vtc, a.max_seq, ctx, a.scale, qs, knew, vnew, red, kf, vf,
                            a.out + (size_t)row * a.H * D + kvh * G * D, stp,
                            wa.fo_units ? wa.gran + (size_t)wa.M * (wa.N / 2) + (size_t)row * (a.H * D / 2) + kvh * G * D / 2
                                        : nullptr,
                            tag);
  TTS_STAMP(stp, 3);
  // the new position's roped k and v to the cache, after this workgroup's reads
  if (tid < D) {
    a.kcache[kvbase + (size_t)pos * D + tid] = knew[tid];
    a.vtcache[kvbase + vt_off(a.max_seq, tid, pos)] = vnew[tid];
  }
}

TTS_DEV bf16x8_t as_bf16x8(u32x4_t v) { return __builtin_bit_cast(bf16x8_t, v); }

// ------------------------------------------- o_proj fused behind the attention -----
// Projection workgroup u (< fo_units) of the one-row QKV + attention launch, after its QKV
// unit: o_proj unit u (16 output columns, K = H*D split over the 16 waves as in the o_proj
// launch, whose stream plan has the same shape, so the tiles, the split-K order and the
// residual epilogue are the o_proj launch's: same bits).  Its weight stages are issued first
// and land while the attention runs; then each wave waits for the 64 granules of its K range
// (one per lane: the attention row of kv group kpart / 2), stages them in LDS and multiplies.
template <int KU, int KSPLIT, int R>
TTS_DEV void fused_oproj(const WgemmArgs& a, bf16_t* xs, float* red, int wave, int lane, uint32_t tag, int u) {
  const int kpart = wave % KSPLIT;
  const int nr = min(a.fo_ur, a.fo_units);
  u32x4_t wr[R][KU];
#pragma unroll
  for (int st = 0; st < R; ++st)
#pragma unroll
    for (int kk = 0; kk < KU; ++kk)
      wr[st][kk] = __builtin_nontemporal_load((const u32x4_t*)a.fo_w +
                                              ((((long long)st * nr + u) * KSPLIT + kpart) * KU + kk) * 64 + lane);
  const bf16_t rr = a.fo_resid[u * 16 + (lane & 15)];
  const uint64_t* g = a.gran + a.N / 2 + kpart * 64 + lane;
  uint64_t v;
  fattn_wait([&] {
    v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (bool)__all((uint32_t)(v >> 32) == tag);
  }, a.fattn_err, a.fattn_spins, lane == 0);
  // this wave's 128 attention values into its own K range of the LDS row (read back by this
  // wave only: LDS operations of one wave complete in order)
  *(uint32_t*)(xs + kpart * 128 + 2 * lane) = (uint32_t)v;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  const int akoff = 8 * (lane >> 4);
#pragma unroll
  for (int st = 0; st < R; ++st)
#pragma unroll
    for (int kk = 0; kk < KU; ++kk) {
      const int k = ((kpart * R + st) * KU + kk) * 32 + akoff;
      const u32x4_t av = *(const u32x4_t*)(xs + k);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(av), as_bf16x8(wr[st][kk]), acc, 0, 0, 0);
    }
  // split-K combine (as the GEMM kernel's: 16-B partials, p ascending), residual epilogue
  if (kpart > 0) *(f32x4_t*)(red + ((size_t)(kpart - 1) * 64 + lane) * 4) = acc;
  lds_barrier();
  if (kpart == 0) {
    constexpr int HB = 8;  // reads in flight per batch (register budget of the 16-wave launch)
#pragma unroll
    for (int p0 = 1; p0 < KSPLIT; p0 += HB) {
      f32x4_t pv[HB];
#pragma unroll
      for (int j = 0; j < HB; ++j)
        if (p0 + j < KSPLIT) pv[j] = *(const f32x4_t*)(red + ((size_t)(p0 + j - 1) * 64 + lane) * 4);
#pragma unroll
      for (int j = 0; j < HB; ++j)
        if (p0 + j < KSPLIT) acc += pv[j];
    }
    if (lane < 16) a.fo_resid[u * 16 + lane] = f2bf(bf2f(rr) + rbf(acc[0]));
  }
}

// The same for the 2..32-row QKV launch (FROWS, order 0): o_proj unit u on its own workgroup.
// Each wave's K range of the o_proj plan (the launch's shape: KSPLIT == WAVES, R stages = the
// item, fo_kc K chunks) comes from the attention rows' granules (gran + M*N/2: row m's
// H*D/2 granules, tag = that row's (pos, layer)), R*KU/4 per lane and row, staged into the
// wave's own columns of the LDS rows (read back by this wave only), then the o_proj launch's
// MFMAs over MT 16-row m-tiles (rows clamped to M - 1 as its m-tiles do), split-K order and
// residual epilogue.
template <int KU, int KSPLIT, int R, int MT>
TTS_DEV void fused_oproj_rows(const WgemmArgs& a, bf16_t* xs, float* red, int wave, int lane, int u) {
  const int M = a.M, HD = a.fa.H * a.fa.D, ldxs = HD + 8, hid = a.fo_units * 16;
  unsigned long long* stp = a.stamps ? a.stamps + (size_t)blockIdx.x * 32 : nullptr;
  TTS_STAMP(stp, 0);
  const int kpart = wave % KSPLIT;
  const int nr = min(a.fo_ur, a.fo_units);
  const int KTc = (HD >> 5) / a.fo_kc, kt_pc = KTc / KSPLIT, Sc = kt_pc / KU;
  auto ktile = [&](int st, int kk) {  // absolute k-tile of stage st, tile kk of this wave
    const int ch = st / Sc;
    return ch * KTc + kpart * kt_pc + (st - ch * Sc) * KU + kk;
  };
  u32x4_t wr[R][KU];
#pragma unroll
  for (int st = 0; st < R; ++st)
#pragma unroll
    for (int kk = 0; kk < KU; ++kk)
      wr[st][kk] = __builtin_nontemporal_load((const u32x4_t*)a.fo_w +
                                              ((((long long)st * nr + u) * KSPLIT + kpart) * KU + kk) * 64 + lane);
  bf16_t rr[MT][4];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) rr[mt][r] = a.fo_resid[(size_t)min(mt * 16 + 4 * (lane >> 4) + r, M - 1) * hid + u * 16 + (lane & 15)];
  constexpr int NGL = R * KU >= 4 ? R * KU / 4 : 1;  // granules per lane and row (R*KU k-tiles of 16; host: R*KU % 4 == 0)
  int col[NGL];
#pragma unroll
  for (int j = 0; j < NGL; ++j) {
    const int gi = j * 64 + lane, ktl = gi >> 4;
    col[j] = ktile(ktl / KU, ktl % KU) * 32 + (gi & 15) * 2;
  }
  const uint64_t* g0 = a.gran + (size_t)M * (a.N / 2);
  // RB rows per poll: their granule loads in flight together (a row at a time was one
  // L2 round trip per row after the attention: +3.3 us at 8 rows)
  constexpr int RB = NGL >= 4 ? 1 : 4;
  for (int m0 = 0; m0 < M; m0 += RB) {
    uint32_t tag[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
      tag[rb] = ((uint32_t)a.fa.row_pos[min(m0 + rb, M - 1)] << 6) | (uint32_t)a.fattn_layer;
    uint64_t v[RB][NGL];
    fattn_wait([&] {
      bool ok = true;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int j = 0; j < NGL; ++j) {  // (rows past M: row M - 1 again, never stored)
          v[rb][j] = __hip_atomic_load(g0 + (size_t)min(m0 + rb, M - 1) * (HD / 2) + col[j] / 2, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
          ok = ok && (uint32_t)(v[rb][j] >> 32) == tag[rb];
        }
      return (bool)__all(ok);
    }, a.fattn_err, a.fattn_spins, lane == 0);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
      if (m0 + rb < M) {
#pragma unroll
        for (int j = 0; j < NGL; ++j) *(uint32_t*)(xs + (size_t)(m0 + rb) * ldxs + col[j]) = (uint32_t)v[rb][j];
      }
    if (m0 == 0) TTS_STAMP(stp, 1);
  }
  TTS_STAMP(stp, 2);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  f32x4_t acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < R; ++st)
#pragma unroll
    for (int kk = 0; kk < KU; ++kk)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16_t* xr = xs + (size_t)min(mt * 16 + (lane & 15), M - 1) * ldxs + 8 * (lane >> 4);
        const u32x4_t av = *(const u32x4_t*)(xr + ktile(st, kk) * 32);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(av), as_bf16x8(wr[st][kk]), acc[mt], 0, 0, 0);
      }
  // split-K combine (as the GEMM kernel's: 16-B partials, p ascending; slot (p - 1, mt))
  if (kpart > 0) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) *(f32x4_t*)(red + (((size_t)(kpart - 1) * MT + mt) * 64 + lane) * 4) = acc[mt];
  }
  lds_barrier();
  if (kpart == 0) {
    constexpr int HB = 8 / MT;
#pragma unroll
    for (int p0 = 1; p0 < KSPLIT; p0 += HB) {
      f32x4_t pv[HB][MT];
#pragma unroll
      for (int j = 0; j < HB; ++j)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          if (p0 + j < KSPLIT) pv[j][mt] = *(const f32x4_t*)(red + (((size_t)(p0 + j - 1) * MT + mt) * 64 + lane) * 4);
#pragma unroll
      for (int j = 0; j < HB; ++j)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          if (p0 + j < KSPLIT) acc[mt] += pv[j][mt];
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mt * 16 + 4 * (lane >> 4) + r;
        const bf16_t ob = f2bf(bf2f(rr[mt][r]) + rbf(acc[mt][r]));
        if (m < M) a.fo_resid[(size_t)m * hid + u * 16 + (lane & 15)] = ob;
        if (a.nrm_wgs)  // (wave-uniform)
          publish_pair(a.nw_gran + (size_t)min(m, M - 1) * (hid / 2), u * 16 + (lane & 15), ob,
                       (*a.nw_epoch << 6) | (uint32_t)a.nw_layer, m < M);
      }
  }
  TTS_STAMP(stp, 3);
}

// ------------------------------------------------------------ RMSNorm once per row -----
// Appended workgroup `row` of a launch whose residual epilogue publishes the updated hidden
// rows as granules (WgemmArgs::nrm_wgs): gathers the row into LDS once every pair carries this
// launch's tag, then the standalone rmsnorm_kernel's arithmetic — a wave per 512-value segment
// (chunk_sumsq + the wave DPP tree), the segments summed in order, every product rounded as in
// every other RMSNorm path — and writes the normalised row to nw_out.
template <int NT>
TTS_DEV void norm_role(const WgemmArgs& a, char* smem, int row) {
  const int hid = a.nw_hid, ng = hid / 2, nseg = hid / 512;  // (host: hid % 512 == 0, hid <= 8192)
  bf16_t* xr = (bf16_t*)smem;
  float* segs = (float*)(smem + (((size_t)hid * 2 + 15) & ~(size_t)15));
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned long long* stp = a.stamps ? a.stamps + (size_t)blockIdx.x * 32 : nullptr;
  TTS_STAMP(stp, 0);
  const uint32_t tag = (*a.nw_epoch << 6) | (uint32_t)a.nw_layer;
  const uint64_t* gp = a.nw_gran + (size_t)row * ng;
  constexpr int GPT = 8192 / 2 / NT > 0 ? 8192 / 2 / NT : 1;  // granules per thread (hid <= 8192)
  uint64_t v[GPT];
  fattn_wait([&] {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < GPT; ++j) {
      const int i = min(j * NT + tid, ng - 1);
      v[j] = __hip_atomic_load(gp + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ok = ok && (uint32_t)(v[j] >> 32) == tag;
    }
    return ok;
  }, a.fattn_err, a.fattn_spins, true);
#pragma unroll
  for (int j = 0; j < GPT; ++j)
    if (j * NT + tid < ng) ((uint32_t*)xr)[j * NT + tid] = (uint32_t)v[j];
  lds_barrier();
  TTS_STAMP(stp, 1);
  for (int sg = wave; sg < nseg; sg += NT / 64) {  // canonical order (chunk_sumsq)
    const float s = wave_sum_dpp(chunk_sumsq(*(const u32x4_t*)(xr + sg * 512 + lane * 8)));
    if (lane == 0) segs[sg] = s;
  }
  lds_barrier();
  float ss = 0.f;
  for (int sg = 0; sg < nseg; ++sg) ss += segs[sg];
  const float r = 1.0f / sqrtf(ss / (float)hid + a.eps);
  for (int k = tid * 8; k < hid; k += NT * 8) {
    u32x4_t x = *(const u32x4_t*)(xr + k);
    const u32x4_t g = *(const u32x4_t*)(a.nw_w + k);
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = pack_bf2(bf_lo(g[q]) * rbf(bf_lo(x[q]) * r), bf_hi(g[q]) * rbf(bf_hi(x[q]) * r));
    *(u32x4_t*)(a.nw_out + (size_t)row * hid + k) = x;
  }
  TTS_STAMP(stp, 2);
}

// ---------------------------------------------------------------- the GEMM kernel -----
// One workgroup = WAVES waves; KSPLIT consecutive waves split the K range of one unit
// (a unit = NG n-tiles of 16 output columns), WAVES/KSPLIT units run side by side, and
// the workgroup walks units grid-stride.  Each wave streams its weight tiles in stages
// of KU tiles (KU KiB), double-buffered, and the stream never stops: the first stage is
// issued before the A-operand prologue (RMSNorm / attention combine), and the last stage
// of a unit prefetches the first stage of the wave's next unit.

// Better (value, index): larger value wins, lower index on ties (torch.argmax semantics).
TTS_DEV void argmax_merge(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}

constexpr int A_GLOBAL = 0, A_LDS = 1;

// MT_MAX: compile-time bound on 16-row m-tiles (1 for decode, 4 for up to 64 rows)
// KSW < KSPLIT (K-sliced over workgroups, kc = 1 layouts): a unit's KSPLIT layout k-parts are
// spread over SL = KSPLIT / KSW workgroups (grid.y), KSW waves each; a.K = the K / SL columns
// a workgroup stages, fp32 partials of each slice to part_out (summed by a combine kernel).
// FROWS: the 2..32-row QKV launch carrying the decode attention (its own instantiation, so the
// consumer's registers stay out of the plain launches of the same shape; MT_MAX 1 or 2)
template <int WAVES, int KU, int MT_MAX, int NG, int KSPLIT, int ASRC, bool NORM, int EPI, int R,
          bool EARLY, int KSW = KSPLIT, bool FROWS = false>
__global__ __launch_bounds__(WAVES * 64) void wgemm_kernel(WgemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NT = WAVES * 64;
  // (one row: the register-staged prologue (EARLY); 2..16 rows (one m-tile): any prologue)
  // (the one-row form carries head dim 64 only, wgemm_fattn_ok: the KU 4 (head dim 128)
  // register-staged instantiation keeps the consumer's registers out)
  constexpr bool FATT = EPI == EPI_STORE && ASRC == A_LDS && WAVES == DEC_NW && KSW == KSPLIT &&
                        ((MT_MAX == 1 && EARLY && !FROWS && wgemm_fattn_d(KU) == 64) ||
                         (MT_MAX <= 2 && !EARLY && FROWS));
  // RMSNorm once per row (a.nrm_wgs): the grid's last workgroups (they wait on every other
  // block: the residual epilogues that publish the rows)
  constexpr bool NRM = EPI == EPI_RESID || (FATT && FROWS);
  if constexpr (NRM) {
    if (a.nrm_wgs && (int)blockIdx.x >= (int)gridDim.x - a.nrm_wgs) {
      norm_role<NT>(a, smem, (int)blockIdx.x - ((int)gridDim.x - a.nrm_wgs));
      return;
    }
  }
  const int nrm_wgs = NRM ? a.nrm_wgs : 0;
  // fused launch (a.fattn_wgs): the grid's projection / attention / o_proj workgroups
  // (WgemmArgs::fattn_first for the two orders)
  const int fo_wgs = (FATT && a.fattn_wgs && !a.fattn_first) ? a.fo_units : 0;  // o_proj workgroups (order 0)
  const int nproj = (int)gridDim.x - nrm_wgs - (FATT ? a.fattn_wgs : 0) - fo_wgs;
  if constexpr (FATT) {
    if (a.fattn_wgs) {
      const int cb = a.fattn_first ? (int)blockIdx.x : (int)blockIdx.x - nproj;
      if (cb >= 0 && cb < a.fattn_wgs) {
        fattn_consumer<NT, wgemm_fattn_d(KU)>(a, smem, cb);
        return;
      }
      if (!a.fattn_first && cb >= a.fattn_wgs) {  // (order 0) o_proj unit cb - fattn_wgs
        const int lane = threadIdx.x & 63;
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const size_t xs_bytes = (((size_t)a.M * (a.K + 8) * 2 + 15) & ~(size_t)15);
        if constexpr (FROWS) {
          fused_oproj_rows<KU, KSPLIT, R, MT_MAX>(a, (bf16_t*)smem, (float*)(smem + xs_bytes), wave, lane,
                                                  cb - a.fattn_wgs);
        } else {
          const uint32_t tag = ((uint32_t)a.fa.row_pos[0] << 6) | (uint32_t)a.fattn_layer;
          fused_oproj<KU, KSPLIT, R>(a, (bf16_t*)smem, (float*)(smem + xs_bytes), wave, lane, tag, cb - a.fattn_wgs);
        }
        return;
      }
    }
  }
  constexpr int UPW = WAVES / KSW;  // units processed concurrently by one workgroup
  constexpr int SL = KSPLIT / KSW;  // K slices over workgroups (grid.y)
  // this workgroup's index among the GEMM workgroups (the attention ones excluded)
  const int bx = (FATT && a.fattn_wgs && a.fattn_first) ? (int)blockIdx.x - a.fattn_wgs : (int)blockIdx.x;
  unsigned long long* stp = a.stamps ? a.stamps + (size_t)blockIdx.x * 32 : nullptr;
  TTS_STAMP(stp, 0);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kq = wave % KSW;  // k-part within the workgroup (split-K combine through LDS)
  const int kpart = (SL > 1 ? (int)blockIdx.y * KSW : 0) + kq;  // k-part of the layout
  const int ugrp = wave / KSW;
  const int M = a.M;
  const int mtn = (M + 15) >> 4;
  // column split (a.csplit = 2, store / residual epilogues): work unit u is half u & 1 of
  // layout unit u >> 1; its waves load only that half's 8 columns of every tile (the other
  // lanes re-read the same 128-B pieces, no extra HBM bytes), so a matrix of 128 units
  // streams on 256 workgroups
  const int cs2 = a.csplit == 2 ? 1 : 0;
  const int bunits = (a.N >> 4) / NG;  // layout units
  const int units = bunits << cs2;     // work units
  // K layout (StreamPlan::kc chunks, chunk-major): a wave's K part is kt_pc k-tiles of every
  // chunk; its stage st covers k-tiles kt(st) .. +KU-1 of chunk st / Sc.  K-sliced launches
  // (a.sliced) run chunk blockIdx.y only: a.K = one chunk, A = that chunk's columns.
  const int kc = a.kc;
  const int KT = a.sliced ? (a.K >> 5) * kc : (a.K >> 5) * SL;  // k-tiles of the whole matrix
  const int KTc = KT / kc;
  const int kt_pc = KTc / KSPLIT;
  const int Sc = kt_pc / KU;
  const int st_off = a.sliced ? blockIdx.y * Sc : 0;        // first (layout) stage of this launch
  const int kt_base = a.sliced ? blockIdx.y * KTc : (SL > 1 ? (int)blockIdx.y * (a.K >> 5) : 0);  // first k-tile in A
  const bf16_t* xg = a.x ? a.x + ((a.sliced || SL > 1) ? (size_t)blockIdx.y * a.K : 0) : nullptr;
  const int ldxs = a.K + 8;  // +16 B per row: the 16 A rows land on distinct LDS bank slots
  const int ustride = nproj * UPW;  // (the fused launch's attention / o_proj workgroups excluded)

  bf16_t* xs = (bf16_t*)smem;
  const size_t xs_bytes = (ASRC != A_GLOBAL) ? (((size_t)M * ldxs * 2 + 15) & ~(size_t)15) : 0;
  float* red = (float*)(smem + xs_bytes);  // split-K partials of waves kpart > 0, scratch

  // stage st of the wave's item of unit uu = NG*KU consecutive tiles from this tile index
  const int ur = a.ur;
  auto stile = [&](int uu, int st) -> long long {
    uu = min(uu, units - 1) >> cs2;
    const int r = uu / ur, ui = uu - r * ur;
    const int nr = min(ur, bunits - r * ur);
    return (long long)r * ur * KT * NG + (((long long)(st + st_off) * nr + ui) * KSPLIT + kpart) * NG * KU;
  };
  const int S = a.sliced ? Sc : kc * Sc;  // stages per item in this launch

  // ---- operands of the prologue and epilogue are loaded FIRST, the weight stream after:
  // vmcnt retires in issue order, so anything issued behind the stream could not be used
  // before the whole first weight stage had landed.
  const int tid = threadIdx.x;
  const int kch = a.K >> 3;  // 16-B chunks per A row
  // (2..16-row fused attention) the granule tags of the rows: each lane of wave 0 loads one
  // row's position here, ahead of every other load, and parks the tag in LDS after the
  // prologue's landing wait (the epilogue reads it there).  Computed from the load on the spot,
  // the tags would need a vmcnt(0) before the weight stream is even issued (the A rows' DMA is
  // still in flight), and held in registers through the stream they spilled.
  constexpr bool FTAGS = FATT && !EARLY;
  int ftag_pos = 0;
  if constexpr (FTAGS) {
    if (a.fattn_wgs) ftag_pos = a.fa.row_pos[min(lane & (16 * MT_MAX - 1), M - 1)];
  }
  // (a) A rows (+ RMSNorm weight) for the LDS prologue, EA chunks per thread at most
  constexpr int EA = wgemm_ea(WAVES);
  const int achunks = M * kch;
  const int a_nj = (achunks + NT - 1) / NT;
  constexpr bool early_a = EARLY && ASRC == A_LDS;  // (host: a_nj <= EA, kch % 64 == 0)
  u32x4_t xe[EA], ne[EA];
  if constexpr (early_a) {
    {
#pragma unroll
      for (int j = 0; j < EA; ++j) {  // all EA issued (clamped): a fixed load count keeps the
        const int c = min(tid + j * NT, achunks - 1);  // vmcnt waits below exact
        const int m = c / kch, k = (c - m * kch) * 8;
        xe[j] = *(const u32x4_t*)(xg + (size_t)m * a.ldx + k);
        if constexpr (NORM) ne[j] = *(const u32x4_t*)(a.normw + k);
      }
    }
  }
  // (a') rows too many for the early registers: LDS-DMA (global_load_lds, 1 KiB per wave
  //      instruction, one row piece each) straight into the padded LDS rows, and the RMSNorm
  //      weight into the (still unused) split-K scratch — no VGPRs, and issued ahead of the
  //      weight stream like every other operand
  // (the only LDS prologue besides the early one: the host sends rows whose K is not a
  // multiple of 512 through A_GLOBAL + a standalone RMSNorm instead (plan_wgemm).  A second,
  // runtime-selected prologue form would leave its loads "pending" at the join for the
  // compiler's wait insertion, i.e. a vmcnt(0) that drains the weight ring before the stream.)
  constexpr bool glds_ok = ASRC == A_LDS && !early_a;
  constexpr bool use_glds = glds_ok;
  if constexpr (glds_ok) {
    if (use_glds) {
      const int ppr = a.K >> 9;
      const int pieces = M * ppr;
      for (int p = wave; p < pieces; p += WAVES) {
        const int m = p / ppr, kp = p - m * ppr;
        __builtin_amdgcn_global_load_lds((gptr_t)(xg + (size_t)m * a.ldx + kp * 512 + lane * 8),
                                         (lptr_t)(xs + (size_t)m * ldxs + kp * 512), 16, 0, 0);
      }
      if constexpr (NORM) {
        for (int p = wave; p < ppr; p += WAVES)
          __builtin_amdgcn_global_load_lds((gptr_t)(a.normw + p * 512 + lane * 8), (lptr_t)((bf16_t*)red + p * 512),
                                           16, 0, 0);
      }
    }
  }
  // (c) epilogue operands of the wave's first unit: residual values / EOS mask + seen bits
  int u = bx * UPW + ugrp;
  const int u_first = min(u, units - 1);
  bf16_t rre[MT_MAX][4];
  int eosr[MT_MAX][4];
  uint32_t seen_cur[MT_MAX][4];
#pragma unroll
  for (int mt = 0; mt < MT_MAX; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // (no mt < mtn test: loads behind a branch cost exact vmcnt)
      const int m = min(mt * 16 + 4 * (lane >> 4) + r, M - 1);
      if constexpr (EPI == EPI_RESID) {
        rre[mt][r] = a.resid[(size_t)m * a.ldo + (u_first >> cs2) * 16 + (lane & 15)];
      }
      if constexpr (EPI == EPI_LOGITS) {
        eosr[mt][r] = a.eos_mask[m];
        seen_cur[mt][r] = a.seen[(size_t)m * a.seen_stride + (u_first >> 1)];
      }
    }

  uint32_t ftag = 0;  // fused attention: this launch's granule tag (row 0)
  if constexpr (FATT && EARLY) {
    if (a.fattn_wgs) ftag = ((uint32_t)a.fa.row_pos[0] << 6) | (uint32_t)a.fattn_layer;
  }

  // ---- then the weight stream
  // Buffer loads through one resource over the whole tiled matrix (32-bit offsets: no 64-bit
  // address per load).  A refill past the wave's last unit gets an offset beyond the
  // resource's range: the load returns zeros without touching memory, so every unit runs the
  // same consume-and-refill loop (no separate drain path) and the ring registers never need
  // path-merging copies (each such copy of an in-flight register is a vmcnt wait, i.e. the
  // ring drained at every unit boundary).
  const uint32_t wbytes = (uint32_t)((long long)(a.N >> 4) * KT * 1024);  // (<= kWgemmMaxBytes: launch-checked)
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, (short)0, (int)wbytes, 0x00020000);
  // byte offset of this lane's 16 B of stage st of the wave's item of unit uu (NG*KU tiles).
  // Past the wave's last unit: a sentinel the stage's tile offsets ((g*KU + kk) KiB, added in
  // uint32) cannot wrap back into the matrix — every piece of the refill stays beyond wbytes
  constexpr uint32_t kPast = kWgemmSentinel - (uint32_t)(NG * KU - 1) * 1024u;
  auto soff = [&](int uu, int st) -> uint32_t {
    const int ls = cs2 ? ((lane & ~8) | ((min(uu, units - 1) & 1) << 3)) : lane;
    return uu < units ? (uint32_t)stile(uu, st) * 1024u + (uint32_t)ls * 16u : kPast;
  };
  // Register ring of R stages (S = stages per item, S % R == 0): the first R stages of the
  // wave's stream are in flight before the prologue runs; consuming a slot refills it with
  // the stage R positions later (next unit's stages once this unit's are all issued).
  u32x4_t wr[R][KU][NG];
  // A_GLOBAL (rows that do not fit the LDS prologue): the A fragments of a stage ride in the
  // ring beside its weight tiles (L2 hits, issued with the stage), so no MFMA waits on an
  // L2 round trip; 1..2 m-tiles (MT_MAX 4 keeps the loads inside consume)
  constexpr bool AGR = ASRC == A_GLOBAL && MT_MAX <= 2;
  const int arow = lane & 15;
  const int akoff = 8 * (lane >> 4);
  u32x4_t ar[R][KU][AGR ? MT_MAX : 1];
  int pu = u, ps = 0;  // next stage to issue
  // The refills are unconditional (past the wave's last unit: the out-of-range offset): every
  // path then has a fixed load count and the compiler's vmcnt waits stay exact (a conditional
  // issue makes it merge paths pessimistically, i.e. drain the ring at every stage).
  auto issue = [&](u32x4_t (&dst)[KU][NG], u32x4_t (&adst)[KU][AGR ? MT_MAX : 1]) {
    const uint32_t q = soff(pu, ps);
#pragma unroll
    for (int kk = 0; kk < KU; ++kk)
#pragma unroll
      for (int g = 0; g < NG; ++g)  // (aux 2: the non-temporal policy: streamed once per step)
        dst[kk][g] = __builtin_amdgcn_raw_buffer_load_b128(wrsrc, (int)(q + (uint32_t)((g * KU + kk) * 1024)), 0, 2);
    if constexpr (AGR) {
      const int sg = ps + st_off, ch = kc == 1 ? 0 : sg / Sc;
      const int kt = ch * KTc + kpart * kt_pc + (sg - ch * Sc) * KU - kt_base;
#pragma unroll
      for (int kk = 0; kk < KU; ++kk)
#pragma unroll
        for (int mt = 0; mt < MT_MAX; ++mt) {
          const int m = min(mt * 16 + arow, M - 1);
          adst[kk][mt] = *(const u32x4_t*)(xg + (size_t)m * a.ldx + (kt + kk) * 32 + akoff);
        }
    }
    if (++ps == S) { ps = 0; pu += ustride; }
  };
  // every wave's operand loads enter the CU's memory pipeline ahead of any weight load; the
  // scheduling barrier stops the compiler sinking an operand load below the weight stream
  // (each prologue wait would then drain the primed stages too)
  __builtin_amdgcn_sched_barrier(0);
  if (a.diag & kWgemmDiagMask & 8) __syncthreads();
  // (unconditional: a wave with no unit issues out-of-range loads, never consumed.  A branch
  // here would make every prologue wait below drain the primed stages as well)
#pragma unroll
  for (int j = 0; j < R; ++j) issue(wr[j], ar[j]);
  __builtin_amdgcn_sched_barrier(0);

  // ---- prologue: A rows in LDS (plain, RMSNorm'ed, or combined from attention chunks)
  if (a.diag & kWgemmDiagMask & 1) {
  } else if constexpr (ASRC == A_LDS) {
   if constexpr (early_a) {
    // rows already in registers: RMSNorm statistics per 64-chunk wave segment (DPP), the
    // segments of a row summed in fixed order after one barrier
    if constexpr (NORM) {
#pragma unroll
      for (int j = 0; j < EA; ++j) {
        if (j < a_nj) {
          const float s = wave_sum_dpp(chunk_sumsq(xe[j]));
          const int c = tid + j * NT;
          if (lane == 0 && c < achunks) red[c >> 6] = s;
        }
      }
      lds_barrier();
    }
#pragma unroll
    for (int j = 0; j < EA; ++j) {
      if (j < a_nj) {
        const int c = tid + j * NT;
        if (c < achunks) {
          const int m = c / kch, k = (c - m * kch) * 8;
          u32x4_t v = xe[j];
          if constexpr (NORM) {
            const int seg0 = (m * kch) >> 6, nseg = kch >> 6;
            float ss = 0.f;
            for (int sg = 0; sg < nseg; ++sg) ss += red[seg0 + sg];
            const float r = 1.0f / sqrtf(ss / (float)a.K + a.eps);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              // (pack_bf2 rounds once: rounding the products first too would be a second,
              // redundant round trip through v_cvt_pk_bf16_f32 + unpack — the same bits)
              v[q] = pack_bf2(bf_lo(ne[j][q]) * rbf(bf_lo(v[q]) * r), bf_hi(ne[j][q]) * rbf(bf_hi(v[q]) * r));
            }
          }
          *(u32x4_t*)(xs + (size_t)m * ldxs + k) = v;
        }
      }
    }
    lds_barrier();
   } else if constexpr (use_glds) {
    // rows landed by LDS-DMA: wait for this wave's DMA only (the weight ring issued after
    // it stays in flight), then every wave's (raw barrier: __syncthreads would drain the ring)
    if (!(a.diag & kWgemmDiagMask & 32)) {
      __builtin_amdgcn_s_waitcnt(waitcnt_vm(R * KU * NG));
      __builtin_amdgcn_s_barrier();
    }
    TTS_STAMP(stp, 6);  // (A rows landed)
    if (a.diag & kWgemmDiagMask & 16) {
    } else if constexpr (NORM) {
      // RMSNorm of the landed rows, a wave per row (canonical order: chunk_sumsq + the wave
      // DPP tree per 512-value segment, segments in order).  Spreading the segment sums and the
      // scaling over every wave gave the same bits and was slower (round 5: TTS-1 8 rows qkv
      // 6.9 -> 9.8 us, profiles/r5h_ab_8.txt; round 4's four rewrites: neutral).
      // Four segments per batch: their LDS reads are issued together and their four DPP trees
      // interleave (one segment at a time was a chain of LDS-read latency + six dependent DPP
      // steps per 512 values); same sums, same order
      const bf16_t* gw = (const bf16_t*)red;
      // (one at a time where the weight ring's registers leave no room: the 2..16-row TTS-1
      // fused launch spilled with the batches)
      constexpr bool BATCH = !(FATT && KU < 4);
      if constexpr (!BATCH) {
        for (int m = wave; m < M; m += WAVES) {
          bf16_t* xr = xs + (size_t)m * ldxs;
          float ss = 0.f;
          for (int k0 = 0; k0 < a.K; k0 += 512)  // canonical order (chunk_sumsq)
            ss += wave_sum_dpp(chunk_sumsq(*(const u32x4_t*)(xr + k0 + lane * 8)));
          const float r = 1.0f / sqrtf(ss / (float)a.K + a.eps);
          for (int k = lane * 8; k < a.K; k += 512) {
            u32x4_t v = *(const u32x4_t*)(xr + k);
            const u32x4_t g = *(const u32x4_t*)(gw + k);
#pragma unroll
            for (int q = 0; q < 4; ++q)
              v[q] = pack_bf2(bf_lo(g[q]) * rbf(bf_lo(v[q]) * r), bf_hi(g[q]) * rbf(bf_hi(v[q]) * r));
            *(u32x4_t*)(xr + k) = v;
          }
        }
      } else {
        constexpr int NB = 4, SB = 2;
        const int k4 = a.K & ~(512 * NB - 1);
        for (int m = wave; m < M; m += WAVES) {
          bf16_t* xr = xs + (size_t)m * ldxs;
          float ss = 0.f;
          for (int k0 = 0; k0 < k4; k0 += 512 * NB) {  // canonical order (chunk_sumsq, segments in order)
            u32x4_t v[NB];
#pragma unroll
            for (int q = 0; q < NB; ++q) v[q] = *(const u32x4_t*)(xr + k0 + q * 512 + lane * 8);
            float sv[NB];
#pragma unroll
            for (int q = 0; q < NB; ++q) sv[q] = wave_sum_dpp(chunk_sumsq(v[q]));
#pragma unroll
            for (int q = 0; q < NB; ++q) ss += sv[q];
          }
          for (int k0 = k4; k0 < a.K; k0 += 512) ss += wave_sum_dpp(chunk_sumsq(*(const u32x4_t*)(xr + k0 + lane * 8)));
          const float r = 1.0f / sqrtf(ss / (float)a.K + a.eps);
          if (m == 0) TTS_STAMP(stp, 7);  // (wave 0: row 0's statistic)
          auto scale = [&](u32x4_t& v, const u32x4_t& g) {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              v[q] = pack_bf2(bf_lo(g[q]) * rbf(bf_lo(v[q]) * r), bf_hi(g[q]) * rbf(bf_hi(v[q]) * r));
          };
          const int ks = a.K & ~(512 * SB - 1);
          for (int k0 = 0; k0 < ks; k0 += 512 * SB) {  // (SB at a time: the ring's registers are live)
            u32x4_t v[SB], g[SB];
#pragma unroll
            for (int q = 0; q < SB; ++q) {
              v[q] = *(const u32x4_t*)(xr + k0 + q * 512 + lane * 8);
              g[q] = *(const u32x4_t*)(gw + k0 + q * 512 + lane * 8);
            }
#pragma unroll
            for (int q = 0; q < SB; ++q) {
              scale(v[q], g[q]);
              *(u32x4_t*)(xr + k0 + q * 512 + lane * 8) = v[q];
            }
          }
          for (int k = ks + lane * 8; k < a.K; k += 512) {
            u32x4_t v = *(const u32x4_t*)(xr + k);
            scale(v, *(const u32x4_t*)(gw + k));
            *(u32x4_t*)(xr + k) = v;
          }
        }
      }
      TTS_STAMP(stp, 24);  // (wave 0: its rows normalised, before the barrier)
#ifdef TTS_STAMPS
      // (diag 64: every wave's norm end, its SIMD (HW_ID bits 5:4) in the stamp's top bits)
      if ((a.diag & 64) && stp && lane == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        stp[8 + wave] = __builtin_amdgcn_s_memrealtime() | ((unsigned long long)((hw >> 4) & 3) << 60);
      }
#endif
      __builtin_amdgcn_s_waitcnt(waitcnt_lgkm0());
      __builtin_amdgcn_s_barrier();
    }
   }
  }
  TTS_STAMP(stp, 1);
  // (the tags' LDS slots: the last 16 floats of the scratch region's slack; read after the
  // split-K combine's barriers)
  uint32_t* ftag_lds = (uint32_t*)(red + wgemm_red_floats(WAVES, KSPLIT, NG, MT_MAX, M, a.K) - 32);
  if constexpr (FTAGS) {
    if (a.fattn_wgs && wave == 0 && lane < 16 * MT_MAX)
      ftag_lds[lane] = ((uint32_t)ftag_pos << 6) | (uint32_t)a.fattn_layer;
  }

  // per-lane running argmax (EPI_LOGITS): rows m = mt*16 + 4*(lane>>4) + r
  float best_v[MT_MAX][4];
  int best_i[MT_MAX][4];
#pragma unroll
  for (int mt = 0; mt < MT_MAX; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) { best_v[mt][r] = -INFINITY; best_i[mt][r] = 0x7fffffff; }

  bool first = true;
  // the unit body: `single` (compile-time) = every wave of the launch has at most one unit, so
  // the stream ends with the unit (no out-of-range refills, the last stages drained in place)
  auto unit_body = [&](int ubase, auto single) {
    u = ubase + ugrp;
    const bool active = u < units;
    uint32_t seen_nxt[MT_MAX][4];
    if constexpr (EPI == EPI_LOGITS) {  // next unit's penalty bits, in flight with this unit
      const int un = min(u + ustride, units - 1);
#pragma unroll
      for (int mt = 0; mt < MT_MAX; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = min(mt * 16 + 4 * (lane >> 4) + r, M - 1);
          seen_nxt[mt][r] = a.seen[(size_t)m * a.seen_stride + (un >> 1)];
        }
    }
    f32x4_t acc[NG][MT_MAX];
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int mt = 0; mt < MT_MAX; ++mt) acc[g][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    auto consume = [&](const u32x4_t (&src)[KU][NG], const u32x4_t (&asrc)[KU][AGR ? MT_MAX : 1], int stage) {
      const int sg = stage + st_off, ch = kc == 1 ? 0 : sg / Sc;
      const int kt = ch * KTc + kpart * kt_pc + (sg - ch * Sc) * KU - kt_base;  // A column tile
#pragma unroll
      for (int kk = 0; kk < KU; ++kk) {
        const int k = (kt + kk) * 32 + akoff;
#pragma unroll
        for (int mt = 0; mt < MT_MAX; ++mt) {  // (all MT_MAX tiles: no branch, exact vmcnt)
          const int m = min(mt * 16 + arow, M - 1);  // rows >= M: duplicates, never stored
          u32x4_t av;
          if constexpr (AGR) av = asrc[kk][mt];
          else if constexpr (ASRC != A_GLOBAL) av = *(const u32x4_t*)(xs + (size_t)m * ldxs + k);
          else av = *(const u32x4_t*)(xg + (size_t)m * a.ldx + k);
          const bf16x8_t af = as_bf16x8(av);
#pragma unroll
          for (int g = 0; g < NG; ++g) {
            acc[g][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, as_bf16x8(src[kk][g]), acc[g][mt], 0, 0, 0);
          }
        }
      }
    };
    // consume slot j, refill it
    auto step = [&](int j, int stage) {
      consume(wr[j], ar[j], stage);
      issue(wr[j], ar[j]);
    };
    if constexpr (decltype(single)::value) {  // the wave's only unit: refill while stages remain, then drain
      for (int st = 0; st + R < S; st += R) {
#pragma unroll
        for (int j = 0; j < R; ++j) step(j, st + j);
      }
#pragma unroll
      for (int j = 0; j < R; ++j) consume(wr[j], ar[j], S - R + j);
    } else {  // one loop for every unit (the last one's refills are the out-of-range loads)
      for (int st = 0; st < S; st += R) {
#pragma unroll
        for (int j = 0; j < R; ++j) step(j, st + j);
      }
    }

    if (first) {
      TTS_STAMP(stp, 2);
      if (!(a.diag & kWgemmDiagMask & 64)) TTS_STAMP_WAVE(stp, 8 + wave);
    }
    if (a.diag & kWgemmDiagMask & 2) {
      if (acc[0][0][0] == 1234.5f && a.out) a.out[0] = 0;
      return;
    }
    // ---- split-K combine through LDS, fixed order (deterministic)
    if constexpr (KSW > 1) {
      // slot of wave (ugrp, kq > 0): ugrp * (KSW-1) + kq - 1
      constexpr int PS = NG * MT_MAX * 4 * 64;
      // one 16-B LDS access per (tile, lane): the sums (fixed order, p ascending) are the
      // same as element-wise, and up to 16 reads of a lane are in flight at once
      if (kq > 0) {
        float* myred = red + (size_t)(ugrp * (KSW - 1) + kq - 1) * PS;
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
          for (int mt = 0; mt < MT_MAX; ++mt)
            if (MT_MAX == 1 || mt < mtn) *(f32x4_t*)(myred + ((g * MT_MAX + mt) * 64 + lane) * 4) = acc[g][mt];
      }
      lds_barrier();
      if (first) TTS_STAMP(stp, 4);
      if (kq == 0) {
        constexpr int NPV = (KSW - 1) * NG * MT_MAX;
        if constexpr (NPV <= 16) {  // every partial read issued before the first add
          f32x4_t pv[KSW > 1 ? KSW - 1 : 1][NG][MT_MAX];
#pragma unroll
          for (int p = 1; p < KSW; ++p)
#pragma unroll
            for (int g = 0; g < NG; ++g)
#pragma unroll
              for (int mt = 0; mt < MT_MAX; ++mt)
                pv[p - 1][g][mt] = *(const f32x4_t*)(red + (size_t)(ugrp * (KSW - 1) + p - 1) * PS +
                                                     ((g * MT_MAX + mt) * 64 + lane) * 4);
#pragma unroll
          for (int p = 1; p < KSW; ++p)
#pragma unroll
            for (int g = 0; g < NG; ++g)
#pragma unroll
              for (int mt = 0; mt < MT_MAX; ++mt) acc[g][mt] += pv[p - 1][g][mt];
        } else {
          // batches of HB k-parts, each batch's reads in flight before its adds (p ascending;
          // rows past M read duplicates, never stored: no per-tile branch around a read)
          constexpr int HB = 8 / (NG * MT_MAX) > 0 ? 8 / (NG * MT_MAX) : 1;
#pragma unroll
          for (int p0 = 1; p0 < KSW; p0 += HB) {
            f32x4_t pv[HB][NG][MT_MAX];
#pragma unroll
            for (int j = 0; j < HB; ++j)
#pragma unroll
              for (int g = 0; g < NG; ++g)
#pragma unroll
                for (int mt = 0; mt < MT_MAX; ++mt)
                  if (p0 + j < KSW)
                    pv[j][g][mt] = *(const f32x4_t*)(red + (size_t)(ugrp * (KSW - 1) + p0 + j - 1) * PS +
                                                     ((g * MT_MAX + mt) * 64 + lane) * 4);
#pragma unroll
            for (int j = 0; j < HB; ++j)
#pragma unroll
              for (int g = 0; g < NG; ++g)
#pragma unroll
                for (int mt = 0; mt < MT_MAX; ++mt)
                  if (p0 + j < KSW) acc[g][mt] += pv[j][g][mt];
          }
        }
      }
      if (first) TTS_STAMP(stp, 5);
      lds_barrier();
    }

    // ---- epilogue (lane owns column n, rows m = mt*16 + 4*(lane>>4) + r)
    if (kq == 0 && active && (!cs2 || ((lane >> 3) & 1) == (u & 1))) {
      const int n = (u >> cs2) * 16 + (lane & 15);
#pragma unroll
      for (int mt = 0; mt < MT_MAX; ++mt) {
        if (mt >= mtn) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = mt * 16 + 4 * (lane >> 4) + r;
          if (m >= M) continue;
          // (32-bit element offsets: 64-bit ones hoisted out of the unit loop cost registers)
          if constexpr (EPI == EPI_STORE) {
            if (a.part_out) a.part_out[((int)blockIdx.y * M + m) * a.ldo + n] = acc[0][mt][r];
            else a.out[m * a.ldo + n] = f2bf(acc[0][mt][r]);
          } else if constexpr (EPI == EPI_RESID) {
            bf16_t* p = a.resid + (m * a.ldo + n);
            const bf16_t ob = f2bf(bf2f(first ? rre[mt][r] : *p) + rbf(acc[0][mt][r]));
            *p = ob;
            // norm once per row: the pair (n, n ^ 1) of row m as a granule (the neighbour lane
            // holds the same row's other column and is in this branch with it)
            if (nrm_wgs)
              publish_pair(a.nw_gran + (size_t)m * (a.nw_hid / 2), n, ob, (*a.nw_epoch << 6) | (uint32_t)a.nw_layer, true);
          } else if constexpr (EPI == EPI_SWIGLU) {
            // unit u = (gate tile, up tile) pair for intermediate columns u*16 .. u*16+15
            const float gt = rbf(acc[0][mt][r]);
            const float up = rbf(acc[NG - 1][mt][r]);
            a.out[(size_t)m * a.ldo + n] = f2bf(rbf(silu_f(gt)) * up);
          } else if constexpr (EPI == EPI_LOGITS) {
            float v = rbf(acc[0][mt][r]);  // logits are materialised in bf16, then .float()
            const uint32_t bits = seen_cur[mt][r];
            if ((bits >> (n & 31)) & 1u) v = (v < 0.f) ? v * a.penalty : v / a.penalty;
            if (a.counts) v -= a.freq_penalty * (float)a.counts[(size_t)m * a.seen_stride * 32 + n];
            if (n == eosr[mt][r]) v = -INFINITY;
            if (a.logits_out) a.logits_out[(size_t)m * a.ldl + n] = v;
            argmax_merge(best_v[mt][r], best_i[mt][r], v, n);
          }
        }
      }
    }
    if constexpr (FATT) {  // publish the unit's 16 columns of every row as 8 granules per row
      if (kq == 0 && active && a.fattn_wgs) {
        if constexpr (EARLY) {  // (the one-row form: the register-staged prologue, host-checked)
          const uint32_t mine = (uint32_t)f2bf(acc[0][0][0]);
          const uint32_t other = (uint32_t)__shfl_xor((int)mine, 1, 64);
          if (lane < 16 && !(lane & 1)) {
            const int n = u * 16 + lane;
            const uint64_t g = ((uint64_t)ftag << 32) | (other << 16) | mine;
            __hip_atomic_store(a.gran + n / 2, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        } else {  // lane holds rows mt * 16 + 4 (lane >> 4) + r of column u * 16 + (lane & 15)
#pragma unroll
          for (int mt = 0; mt < MT_MAX; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t mine = (uint32_t)f2bf(acc[0][mt][r]);
            const uint32_t other = (uint32_t)__shfl_xor((int)mine, 1, 64);
            const int m = mt * 16 + 4 * (lane >> 4) + r;
            if (!(lane & 1) && m < M) {
              const int n = u * 16 + (lane & 15);
              const uint64_t g = ((uint64_t)ftag_lds[m] << 32) | (other << 16) | mine;
              __hip_atomic_store(a.gran + (m * (a.N >> 1) + (n >> 1)), g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
        }
      }
    }
    if (first) TTS_STAMP(stp, 3);
    first = false;
    if constexpr (EPI == EPI_LOGITS) {
#pragma unroll
      for (int mt = 0; mt < MT_MAX; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) seen_cur[mt][r] = seen_nxt[mt][r];
    }
  };
  if (units <= ustride) {
    unit_body(bx * UPW, std::true_type{});
  } else {
    for (int ubase = bx * UPW; ubase < units; ubase += ustride) unit_body(ubase, std::false_type{});
  }

  if constexpr (FATT) {
    if (a.fattn_wgs && a.fattn_first && a.fo_units > 0 && bx < a.fo_units) {
      lds_barrier();  // (every wave past the QKV unit's LDS use)
      fused_oproj<KU, KSPLIT, R>(a, xs, red, wave, lane, ftag, bx);
    }
  }
  if constexpr (EPI == EPI_LOGITS) {
    // lanes sharing (lane >> 4) hold the same rows: butterfly over the 16 columns
#pragma unroll
    for (int mt = 0; mt < MT_MAX; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          const float v2 = __shfl_xor(best_v[mt][r], o, 64);
          const int i2 = __shfl_xor(best_i[mt][r], o, 64);
          argmax_merge(best_v[mt][r], best_i[mt][r], v2, i2);
        }
    // across the unit-groups of the workgroup (only kpart==0 waves hold results)
    float* rv = red;
    int* ri = (int*)(red + UPW * MT_MAX * 16);
    lds_barrier();
    if (kq == 0 && (lane & 15) == 0) {
#pragma unroll
      for (int mt = 0; mt < MT_MAX; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = mt * 16 + 4 * (lane >> 4) + r;
          rv[ugrp * MT_MAX * 16 + m] = best_v[mt][r];
          ri[ugrp * MT_MAX * 16 + m] = best_i[mt][r];
        }
    }
    lds_barrier();
    for (int m = threadIdx.x; m < M; m += NT) {
      float v = rv[m];
      int i = ri[m];
      for (int g = 1; g < UPW; ++g) argmax_merge(v, i, rv[g * MT_MAX * 16 + m], ri[g * MT_MAX * 16 + m]);
      a.part_val[(size_t)m * a.part_stride + blockIdx.x] = v;
      a.part_idx[(size_t)m * a.part_stride + blockIdx.x] = i;
    }
  }
}

// ---------------------------------------------------------------- host dispatch -------
// Launch shapes (WAVES, KU, KSPLIT, ring depth R) = the stream plans a matrix can have.
struct Shape3 { int waves, ku, ksplit, r; bool ng2; };
inline constexpr Shape3 kShapes[] = {
    {4, 8, 1, 2, false},    // 0  lm_head
    {8, 4, 8, 2, false},    // 1  fallback for short K
    {16, 2, 16, 2, false},  // 2  qkv / o_proj
    {16, 4, 16, 2, false},  // 3  down
    {8, 4, 4, 2, true},     // 4  (NG = 2)
    {8, 2, 4, 2, true},     // 5  gate/up (NG = 2)
    {16, 2, 8, 2, true},    // 6  (NG = 2)
};
inline constexpr int kNumShapes = sizeof(kShapes) / sizeof(kShapes[0]);
inline bool shape_ng2(int c) { return kShapes[c].ng2; }

// the instantiation a launch runs (the dry run's record; the order of wgemm_kernel's parameters)
inline std::string wgemm_inst_name(int waves, int ku, int mt, int ng, int ksplit, int asrc, bool norm, int epi, int r,
                                   bool early, int ksw, bool frows) {
  char b[128];
  snprintf(b, sizeof b, "wgemm_kernel<%d, %d, %d, %d, %d, %d, %s, %d, %d, %s, %d, %s>", waves, ku, mt, ng, ksplit, asrc,
           norm ? "true" : "false", epi, r, early ? "true" : "false", ksw, frows ? "true" : "false");
  return b;
}

template <int WAVES, int KU, int NG, int KSPLIT, int ASRC, bool NORM, int EPI, int R, bool EARLY>
static void launch_one_e(const WgemmArgs& a, int grid, hipStream_t s) {
  const int mt = a.M <= 16 ? 1 : (a.M <= 32 ? 2 : 4);
  if (dry_launches()) {  // (the branches below, without the launch)
    const bool frows = mt <= 2 && !EARLY && a.fattn_wgs && a.M > 1;
    dry_record(wgemm_inst_name(WAVES, KU, mt, NG, KSPLIT, ASRC, NORM, EPI, R, mt == 1 && EARLY && !frows, KSPLIT, frows));
    return;
  }
  size_t lds = (ASRC != A_GLOBAL) ? (((size_t)a.M * (a.K + 8) * 2 + 15) & ~(size_t)15) : 0;
  lds += (size_t)wgemm_red_floats(WAVES, KSPLIT, NG, mt, a.M, a.K) * sizeof(float);
  if (a.fattn_wgs) {  // QKV + fused decode attention (1..16 rows, D 64 / 128, 16-wave workgroups)
    if (!(EPI == EPI_STORE && ASRC == A_LDS && a.M >= 1 && a.M <= 32 && a.fa.D == wgemm_fattn_d(KU) &&
          WAVES == DEC_NW && a.gran && a.fattn_err && !a.sliced && a.csplit == 1 && a.fattn_wgs == a.M * a.fa.KVH))
      throw std::runtime_error("wgemm: fused attention needs a 1..32-row 16-wave QKV launch (D 64 or 128)");
    if ((a.M == 1) != EARLY)
      throw std::runtime_error("wgemm: fused attention: one row = the register-staged prologue, 2..16 rows = not");
    if (a.M == 1 && a.fa.D != 64)
      throw std::runtime_error("wgemm: fused one-row attention: head dim 64 only");
    if (a.M > 1 && a.fattn_first)
      throw std::runtime_error("wgemm: multi-row fused attention: producer-first grid order only");
    if (a.fo_units && a.M > 1) {  // fused o_proj behind the 2..16-row attention (order 0)
      const int HD = a.fa.H * a.fa.D;
      const int S = (HD / 32) / (KSPLIT * KU);
      if (!(a.fo_w && a.fo_resid && a.fo_units <= a.fo_ur && S == R && KSPLIT == WAVES && HD == a.K && a.fo_kc >= 1 &&
            (HD / 32) % (a.fo_kc * KSPLIT * KU) == 0 && R * KU % 4 == 0 && R * KU >= 4))
        throw std::runtime_error("wgemm: fused multi-row o_proj shape mismatch");
    } else if (a.fo_units) {  // fused o_proj: one unit per o_proj (order 1: projection) workgroup, one granule per lane
      const int S = (a.fa.H * a.fa.D / 32) / (KSPLIT * KU);
      if (!(a.fo_w && a.fo_resid && (!a.fattn_first || a.fo_units <= grid) && a.fo_units <= a.fo_ur && S == R &&
            a.fa.H * a.fa.D == KSPLIT * 128 && KSPLIT == WAVES && (size_t)a.M * (a.K + 8) * 2 >= (size_t)KSPLIT * 256))
        throw std::runtime_error("wgemm: fused o_proj shape mismatch");
    }
    lds = std::max(lds, a.fa.D == 64 ? fattn_lds_bytes<64>() : fattn_lds_bytes<128>());
    grid += a.fattn_wgs + (a.fattn_first ? 0 : a.fo_units);
    if (a.fattn_first) {
      // order 1: the attention workgroups spin on the projection workgroups' granules and
      // those (o_proj fused) on the attention's: every workgroup must be resident at once.
      // A 16-wave workgroup at 128 VGPRs fills a CU's register file (one per CU), so
      // grid <= CUs is required — and still not sufficient when other work shares the GPU
      static const int cus = [] {
        int n = 0;
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n;
      }();
      if (grid > cus) throw std::runtime_error("wgemm: fused attention grid exceeds one workgroup per CU");
    }
  }
  if (a.nrm_wgs) {  // RMSNorm once per row: M workgroups appended last (norm_role)
    const bool producer = EPI == EPI_RESID || (a.fattn_wgs && a.fo_units && a.M > 1 && !EARLY);
    if (!(producer && a.nrm_wgs == a.M && (EPI != EPI_RESID || a.M <= 16) && a.nw_w && a.nw_out && a.nw_gran && a.nw_epoch && a.nw_hid % 512 == 0 &&
          a.nw_hid <= 8192 && a.nw_hid == (EPI == EPI_RESID ? a.N : a.fo_units * 16) && !a.sliced &&
          (WAVES * 64) * (8192 / 2 / (WAVES * 64) > 0 ? 8192 / 2 / (WAVES * 64) : 1) * 2 >= a.nw_hid))
      throw std::runtime_error("wgemm: norm-once workgroups need a residual launch over hid % 512 == 0 columns");
    lds = std::max(lds, (((size_t)a.nw_hid * 2 + 15) & ~(size_t)15) + (size_t)(a.nw_hid / 512) * 4 + 64);
    grid += a.nrm_wgs;
  }
  if (lds > 160 * 1024) throw std::runtime_error("wgemm: LDS request above 160 KiB");
  if ((unsigned long long)a.N * (unsigned long long)(a.sliced ? (size_t)a.K * a.kc : (size_t)a.K) * 2ull > kWgemmMaxBytes)
    throw std::runtime_error("wgemm: tiled weight matrix above the 32-bit buffer range");
  if (ASRC == A_LDS && !EARLY && a.K % 512 != 0)
    throw std::runtime_error("wgemm: the LDS-DMA prologue needs K a multiple of 512 (plan_wgemm: A_GLOBAL)");
  const dim3 g(grid, a.sliced ? a.kc : 1);
  if (mt <= 2 && !EARLY && a.fattn_wgs && a.M > 1) {  // (FROWS: 2..32 rows)
    if constexpr (EPI == EPI_STORE && ASRC == A_LDS && WAVES == DEC_NW) {
      if (mt == 1)
        hipLaunchKernelGGL((wgemm_kernel<WAVES, KU, 1, NG, KSPLIT, ASRC, NORM, EPI, R, false, KSPLIT, true>), g,
                           dim3(WAVES * 64), lds, s, a);
      else
        hipLaunchKernelGGL((wgemm_kernel<WAVES, KU, 2, NG, KSPLIT, ASRC, NORM, EPI, R, false, KSPLIT, true>), g,
                           dim3(WAVES * 64), lds, s, a);
    }
  } else if (mt == 1)
    hipLaunchKernelGGL((wgemm_kernel<WAVES, KU, 1, NG, KSPLIT, ASRC, NORM, EPI, R, EARLY>), g,
                       dim3(WAVES * 64), lds, s, a);
  else if (mt == 2)
    hipLaunchKernelGGL((wgemm_kernel<WAVES, KU, 2, NG, KSPLIT, ASRC, NORM, EPI, R, false>), g,
                       dim3(WAVES * 64), lds, s, a);
  else
    hipLaunchKernelGGL((wgemm_kernel<WAVES, KU, 4, NG, KSPLIT, ASRC, NORM, EPI, R, false>), g,
                       dim3(WAVES * 64), lds, s, a);
}

// ring depth: the shape's R when it divides the item's stage count S, else 2 or 1
// early (register-staged) prologue when the rows fit the early registers (decode)
template <int WAVES, int KU, int NG, int KSPLIT, int ASRC, bool NORM, int EPI, int R>
static void launch_one(const WgemmArgs& a, int grid, hipStream_t s) {
  bool early = false;
  if (a.M <= 16 && !(a.fattn_wgs && a.M > 1)) {  // (multi-row fused attention: the LDS prologue form)
    const int kch = a.K / 8, NT = WAVES * 64;
    if (ASRC == A_LDS) early = (kch % 64 == 0) && (a.M * kch + NT - 1) / NT <= wgemm_ea(WAVES);
  }
  if constexpr (ASRC == A_GLOBAL) launch_one_e<WAVES, KU, NG, KSPLIT, ASRC, NORM, EPI, R, false>(a, grid, s);
  else if (early) launch_one_e<WAVES, KU, NG, KSPLIT, ASRC, NORM, EPI, R, true>(a, grid, s);
  else launch_one_e<WAVES, KU, NG, KSPLIT, ASRC, NORM, EPI, R, false>(a, grid, s);
}

template <int C, int NG, int ASRC, bool NORM, int EPI>
static void launch_shape(const WgemmArgs& a, int grid, hipStream_t s) {
  constexpr Shape3 h = kShapes[C];
  const int S = (a.K / 32) / (h.ksplit * h.ku);  // (sliced: stages of one chunk)
  // (A_GLOBAL rides A fragments in the ring: one stage deep where two would spill — KU 4, or
  // two m-tiles at KU > 2)
  const bool agr_r1 = ASRC == A_GLOBAL && (h.ku >= 4 || (a.M > 16 && h.ku > 2));
  if constexpr (NG == 2 && ASRC == A_LDS && h.ku == 2 && h.waves == 8) {
    // 4..16 rows, gate/up (8-wave workgroups: 256 registers a lane): a four-stage ring, so
    // the stream keeps going through the longer LDS prologue (rows landed + RMSNorm of every
    // row) instead of stalling once two stages have landed: TTS-1-Max 8 rows 3,380 -> 3,370 us,
    // TTS-1 8 rows 808 -> 806 us, same ids (profiles/r4r_ab_ring4_*).  TTS_RING4=0: off
    static const bool ring4 = !(getenv("TTS_RING4") && !atoi(getenv("TTS_RING4")));
    // 17..32 rows too (two m-tiles, 164 registers, no spill): gate/up 17.42 -> 17.14 us, step
    // 993.4 -> 989.5 us at 32 rows, same ids (profiles/r5ring32_*).  TTS_RING4_32=0: 4..16 only
    static const bool ring4_32 = !(getenv("TTS_RING4_32") && !atoi(getenv("TTS_RING4_32")));
    if (ring4 && a.M >= 4 && a.M <= (ring4_32 ? 32 : 16) && S % 4 == 0) {
      launch_one<h.waves, h.ku, NG, h.ksplit, ASRC, NORM, EPI, 4>(a, grid, s);
      return;
    }
  }
  if (h.r >= 2 && S % 2 == 0 && !agr_r1) launch_one<h.waves, h.ku, NG, h.ksplit, ASRC, NORM, EPI, 2>(a, grid, s);
  else launch_one<h.waves, h.ku, NG, h.ksplit, ASRC, NORM, EPI, 1>(a, grid, s);
}

template <int NG, int ASRC, bool NORM, int EPI>
static void launch_cfg(const WgemmArgs& a, int cfg, int grid, hipStream_t s) {
  if constexpr (NG == 2) {
    switch (cfg) {
      case 4: launch_shape<4, NG, ASRC, NORM, EPI>(a, grid, s); break;
      case 6: launch_shape<6, NG, ASRC, NORM, EPI>(a, grid, s); break;
      default: launch_shape<5, NG, ASRC, NORM, EPI>(a, grid, s); break;
    }
  } else {
    switch (cfg) {
      case 1: launch_shape<1, NG, ASRC, NORM, EPI>(a, grid, s); break;
      case 2: launch_shape<2, NG, ASRC, NORM, EPI>(a, grid, s); break;
      case 3: launch_shape<3, NG, ASRC, NORM, EPI>(a, grid, s); break;
      default: launch_shape<0, NG, ASRC, NORM, EPI>(a, grid, s); break;
    }
  }
}

// per-epilogue launchers (one translation unit each)
void launch_wgemm_store(const WgemmArgs& a, const WgemmPlan& p, bool norm, hipStream_t s);
void launch_wgemm_resid(const WgemmArgs& a, const WgemmPlan& p, bool norm, hipStream_t s);
void launch_wgemm_swiglu(const WgemmArgs& a, const WgemmPlan& p, bool norm, hipStream_t s);
void launch_wgemm_logits(const WgemmArgs& a, const WgemmPlan& p, bool norm, hipStream_t s);

}  // namespace tts
