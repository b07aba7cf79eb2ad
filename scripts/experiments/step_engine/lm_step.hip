// lm_step.hip — the one-row decode step's transformer stack as ONE persistent launch on a
// weight-streaming engine (TTS-1 geometry: hidden 2048, 32 q / 8 kv heads of 64, ffn 8192,
// 256 CUs).  Reference semantics: transformers LlamaDecoderLayer (modeling_llama.py:284-326)
// at decode time, as the launch path restates it (lm_gemm.hip header, lm_attn.hip).
//
// Why one launch: as a chain of dependent launches a batch-1 layer pays, per launch, the
// ramp of a fresh weight stream after its inputs are ready (MI355X_MICROARCH.md, price list
// rows launches-baseline / engine-vs-launches / prefetch-credit).  Here every CU runs one
// 8-wave workgroup for all layers:
//   * wave 0 is the LOADER: it streams this CU's share of every weight matrix, in the order
//     the step consumes them (qkv, o, gate/up, down of layer 0, then layer 1, ...), through
//     an LDS ring of 16 KiB slots by LDS-DMA (global_load_lds nt), FLY slots in flight, and
//     never waits for a data dependency — only for a free slot.  While the CU waits for a
//     vector from the other CUs, its ring keeps filling with the weights it will multiply
//     next.
//   * waves 1..7 are CONSUMERS: slot s of the step goes to consumer s % 7; a slot is a
//     self-contained piece of work (4 whole rows of a K = 2048 matrix, or 8 rows of the
//     down projection over a 1024-wide k chunk), multiplied on the VALU (v_dot2_f32_bf16)
//     against the op's input vector once it is there.
// Every CU owns a fixed slice of each matrix: qkv outputs 12c .. 12c+11, o outputs 8c ..
// 8c+7, gate/up outputs (= act) 32c .. 32c+31 and down outputs 8c .. 8c+7 (the whole
// K = 8192: down slot t covers k = 1024t .. +1023 and gathers just that act chunk, made by CUs
// 32t .. 32t+31, so it neither waits for every CU nor needs a cross-CU partial reduction).
// Vectors move between CUs as 8-byte granules {payload, tag} written by ONE agent-scope
// store each (tag = the step's sequence number: a granule left by an earlier step never
// matches) and gathered by one wave per vector per CU (MI355X_MICROARCH.md: granule,
// allgather).  Attention runs on CUs 0..7 (one per kv head): their 7 consumer waves hold
// the kv head's K rows / V^T columns in registers from the start of the layer
// (lm_attn_core.h), gather q / k / v, and publish the head group's bf16 output.
//
// Arithmetic: the reference's roundings at every op boundary (bf16 RMSNorm, projections
// rounded once to bf16, bf16 residual adds, SiLU(gate)*up in bf16, flash-numerics attention
// with the global maximum); fp32 sums in this engine's own fixed order (deterministic, not
// bit-identical to the launch path's split-K order).  Every wait is bounded: a timeout sets
// err and every wave drains (the host reports the failure; tests/test_gpu_step.py).
#include <cstdio>
#include <stdexcept>

#include "hip_common.h"
#include "lm_kernels.h"
#include "lm_attn_core.h"

namespace tts {

namespace {

constexpr int NCU = 256, NWV = 8, NCONS = NWV - 1;
constexpr int HID = 2048, QKVN = 3072, FFN = 8192, NH = 32, NKV = 8, HDIM = 64, GQ = NH / NKV;
constexpr int SLOT = 16384;                    // bytes per ring slot
constexpr int NS = 8;                          // ring slots
constexpr int FLY = 3;                         // slots the loader keeps in flight
constexpr int S_QKV = 3, S_O = 2, S_GU = 16, S_D = 8;
constexpr int O_QKV = 0, O_O = S_QKV, O_GU = O_O + S_O, O_D = O_GU + S_GU, S_LAYER = O_D + S_D;  // 29
constexpr int PW = 64;                         // attention positions per consumer wave and pass
constexpr int MAX_SPINS = 1 << 17;
constexpr int NEV = kStepEvents;

// diagnostics (StepArgs::trace): a 100 MHz stamp of event ev of layer l on this CU
TTS_DEV void stamp(unsigned long long* tr, int l, int c, int ev) {
  if (tr) tr[((size_t)l * NCU + c) * NEV + ev] = __builtin_amdgcn_s_memrealtime();
}

// granule area of one layer (u64 {payload, tag})
constexpr int G_X = 0;                   // layer output x_{l+1}: bf16 pairs [HID/2]
constexpr int G_QKV = G_X + HID / 2;     // q | k | v before RoPE: bf16 pairs [QKVN/2]
constexpr int G_ATT = G_QKV + QKVN / 2;  // attention output: bf16 pairs [HID/2]
constexpr int G_H = G_ATT + HID / 2;     // residual after attention: bf16 pairs [HID/2]
constexpr int G_ACT = G_H + HID / 2;     // SiLU(gate) * up: bf16 pairs [FFN/2]
constexpr int G_LAYER = G_ACT + FFN / 2;

// LDS carve-up (bytes)
constexpr int L_RING = 0;
constexpr int L_X = L_RING + NS * SLOT;       // x_l (bf16 [HID])
constexpr int L_H = L_X + HID * 2;            // h (bf16 [HID])
constexpr int L_A = L_H + HID * 2;            // attention output (bf16 [HID])
constexpr int L_DP = L_A + HID * 2;           // down: the 8 slots' row sums (f32 [S_D][8])
constexpr int L_QS = L_DP + S_D * 8 * 4;      // attention: roped q [GQ][HDIM] f32
constexpr int L_RAW = L_QS + GQ * HDIM * 4;   // attention: gathered q | k | v pairs (u32)
constexpr int L_KN = L_RAW + (GQ * HDIM / 2 + HDIM) * 4;  // new k, new v (bf16 [HDIM] each)
constexpr int L_AO = L_KN + 2 * HDIM * 2;     // attention output of the group (bf16 [GQ*HDIM])
constexpr int L_RED = L_AO + GQ * HDIM * 2;   // attention merge scratch
constexpr int L_FLAGS = L_RED + dec_red_floats<HDIM, NCONS>() * 4;
constexpr int F_FULL = 0, F_FREE = NS, F_RX = 2 * NS, F_RA = F_RX + 1, F_RH = F_RX + 2, F_BAR = F_RX + 3,
              F_DS = F_RX + 4, F_XP = F_RX + 5, F_GU = F_RX + 6, F_GATH = F_RX + 7, F_N = F_RX + 8;
constexpr int LDS_BYTES = L_FLAGS + F_N * 4;
static_assert(LDS_BYTES <= 160 * 1024, "decode step LDS");

// explicit address spaces: LDS flags as ds_* and granules as global_* instructions (a generic
// pointer would compile to flat_* instructions, which count on both waitcnt queues)
typedef __attribute__((address_space(3))) int lint;
typedef __attribute__((address_space(1))) uint64_t g64;
typedef __attribute__((address_space(1))) int gint;
TTS_DEV lint* lflags(char* smem) { return (lint*)(smem + L_FLAGS); }
TTS_DEV int lds_ld(lint* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
TTS_DEV void lds_st(lint* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
TTS_DEV int lds_add(lint* p, int v) { return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
TTS_DEV uint64_t gld(const uint64_t* p) {
  return __hip_atomic_load((const g64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
TTS_DEV void gst(uint64_t* p, uint32_t payload, uint32_t tag) {
  __hip_atomic_store((g64*)p, ((uint64_t)tag << 32) | payload, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
TTS_DEV int gerr(const int* e) { return __hip_atomic_load((const gint*)e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
TTS_DEV void set_err(int* e) { __hip_atomic_store((gint*)e, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// The loader's flag accesses as inline asm: the compiler treats any LDS access after an
// LDS-DMA load as a possible alias of the DMA destination and drains every load in flight
// (s_waitcnt vmcnt(0)) before it, which would leave one slot in flight.  The ring protocol
// orders them instead (counted vmcnt before FULL, FREE read before the slot is refilled).
TTS_DEV int lds_ld_dma(lint* p) {
  int v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(size_t)p) : "memory");
  return v;
}
TTS_DEV void lds_st_dma(lint* p, int v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"((uint32_t)(size_t)p), "v"(v) : "memory");
}

// wave-uniform wait until the LDS word reaches v (bounded; err drains every wave)
TTS_DEV void lds_spin_ge(lint* p, int v, int* err) {
  int spins = 0;
  while (lds_ld(p) < v) {
    if (++spins > MAX_SPINS || ((spins & 255) == 0 && gerr(err))) {
      set_err(err);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
TTS_DEV void lds_wait_ge(lint* p, int v, int* err) {
  if (lds_ld(p) < v) lds_spin_ge(p, v, err);
}

// one granule's payload once its tag is this step's (bounded)
TTS_DEV uint32_t gwait(const uint64_t* p, uint32_t tag, int* err, bool any = false) {
  uint64_t v = gld(p);
  if (any) return (uint32_t)v;
  int spins = 0;
  while ((uint32_t)(v >> 32) != tag) {
    if (++spins > MAX_SPINS || ((spins & 255) == 0 && gerr(err))) {
      set_err(err);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    v = gld(p);
  }
  return (uint32_t)v;
}

// One wave gathers a bf16 vector of HID values (HID/2 granules, 16 per lane) into LDS: one
// sweep issues every load, then only the granules still stale are re-read, all of them per
// re-sweep (never one round trip per granule).
TTS_DEV void gather_vec(const uint64_t* g, uint32_t tag, bf16_t* dst, int lane, int* err, bool any) {
  constexpr int PER = HID / 2 / 64;
  uint64_t v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) v[i] = gld(g + lane + 64 * i);
  uint32_t pending = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    if (any || (uint32_t)(v[i] >> 32) == tag) ((uint32_t*)dst)[lane + 64 * i] = (uint32_t)v[i];
    else pending |= 1u << i;
  }
  int spins = 0;
  while (pending) {
    if (++spins > MAX_SPINS || ((spins & 255) == 0 && gerr(err))) {
      set_err(err);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (pending & (1u << i)) v[i] = gld(g + lane + 64 * i);
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if ((pending & (1u << i)) && (uint32_t)(v[i] >> 32) == tag) {
        ((uint32_t*)dst)[lane + 64 * i] = (uint32_t)v[i];
        pending &= ~(1u << i);
      }
  }
}

TTS_DEV float dot8(u32x4_t a, u32x4_t b, float acc) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
  {
    // element copies first: __builtin_bit_cast of a vector subscript reads element 0
    const uint32_t aq = a[q], bq = b[q];
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_cvt_t, aq), __builtin_bit_cast(bf16x2_cvt_t, bq), acc,
                                          false);
  }
  return acc;
}

// this lane's 32 values of RMSNorm(v) (LlamaRMSNorm: fp32 mean of squares in the canonical
// order of the launch path, x * r rounded to bf16, times the weight rounded to bf16), at
// k = 8 lane + 512 j; v (LDS bf16 [HID]), w (global bf16 [HID])
TTS_DEV void norm_chunks(const bf16_t* v, const bf16_t* w, float eps, int lane, u32x4_t (&xn)[4]) {
  u32x4_t x[4], g[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    g[j] = *(const u32x4_t*)(w + 8 * lane + 512 * j);
    x[j] = *(const u32x4_t*)(v + 8 * lane + 512 * j);
  }
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) ss += wave_sum_dpp(chunk_sumsq(x[j]));  // per 512-value segment, in order
  const float r = 1.0f / sqrtf(ss / (float)HID + eps);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      xn[j][q] = pack_bf2(rbf(bf_lo(g[j][q]) * rbf(bf_lo(x[j][q]) * r)), rbf(bf_hi(g[j][q]) * rbf(bf_hi(x[j][q]) * r)));
}
TTS_DEV void plain_chunks(const bf16_t* v, int lane, u32x4_t (&xn)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) xn[j] = *(const u32x4_t*)(v + 8 * lane + 512 * j);
}

// the 4 rows of a K = 2048 slot against the lane's chunks: wave-uniform fp32 results
TTS_DEV void rows4(const char* slot, const u32x4_t (&xn)[4], int lane, float (&y)[4]) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {  // two rows at a time: 8 LDS reads in flight before the products
    u32x4_t w[2][4];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) w[r][j] = *(const u32x4_t*)(slot + (2 * h + r) * 4096 + j * 1024 + lane * 16);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = dot8(w[r][j], xn[j], acc);
      y[2 * h + r] = wave_sum_dpp(acc);
    }
  }
}

// Attention of kv head c (CUs 0..7) by the 7 consumer waves: q of heads 4c..4c+3 and the
// new k, v gathered from the qkv granules -> RoPE -> lm_attn_core.h dec_attend_w (global max,
// bf16 P.V, wave-order merge) -> the group's 4 heads published; the new K row / V^T column to
// the cache.
TTS_DEV void step_attention(const StepArgs& a, char* smem, uint64_t* G, uint32_t tag,
                                                         int c, int cw, int ctid, int lane, int l, int pos, int ctx,
                                                         size_t kvl, size_t kvbase, int& nbar) {
  lint* fl = lflags(smem);
  auto cbar = [&]() {  // barrier over the consumer waves (LDS counter)
    ++nbar;
    if (lane == 0) lds_add(fl + F_BAR, 1);
    lds_wait_ge(fl + F_BAR, NCONS * nbar, a.err);
  };
  const bf16_t* kc = a.kv + 2 * kvl + kvbase;                // K rows of (slot, kv head c)
  const bf16_t* vtc = a.kv + 2 * kvl + a.kv_layer + kvbase;  // V^T columns
  // this wave's first-pass K / V^T fragments, in flight while q / k / v are gathered (loading
  // them earlier, at the top of the layer, keeps them live across the slot math: spills)
  using C = DecShape<HDIM, PW>;
  u32x4_t kf[C::MT][C::KS], vf[C::PS][C::DT];
  if (cw * PW < ctx) {
    dec_load_k<HDIM, PW>(kc, cw * PW, ctx, lane, kf);
    dec_load_v<HDIM, PW>(vtc, a.kv_stride, cw * PW, lane, vf);
  }
  float* qs = (float*)(smem + L_QS);
  uint32_t* raw = (uint32_t*)(smem + L_RAW);
  const bf16_t* rawb = (const bf16_t*)raw;
  bf16_t* knew = (bf16_t*)(smem + L_KN);
  bf16_t* vnew = knew + HDIM;
  bf16_t* ao = (bf16_t*)(smem + L_AO);
  // the RoPE table entries too (a dependent global load after the gather would sit on the
  // critical path)
  const int qd = ctid % HDIM;
  const float qc = bf2f(a.rope_cos[(size_t)pos * HDIM + qd]), qsn = bf2f(a.rope_sin[(size_t)pos * HDIM + qd]);
  constexpr int NQ = GQ * HDIM / 2, NG = NQ + HDIM;
  if (ctid < NG) {
    int col;
    if (ctid < NQ) col = c * GQ * HDIM + 2 * ctid;
    else if (ctid < NQ + HDIM / 2) col = NH * HDIM + c * HDIM + 2 * (ctid - NQ);
    else col = NH * HDIM + NKV * HDIM + c * HDIM + 2 * (ctid - NQ - HDIM / 2);
    raw[ctid] = gwait(G + G_QKV + col / 2, tag, a.err, a.nodeps);
  }
  cbar();
  if (cw == 0 && lane == 0) stamp(a.trace, l, c, 14);
  constexpr int H2 = HDIM / 2;
  if (ctid < GQ * HDIM) {
    const int g = ctid / HDIM;
    qs[ctid] = rope_elem(rawb[ctid], rawb[g * HDIM + (qd < H2 ? qd + H2 : qd - H2)], qd < H2, qc, qsn);
  } else if (ctid < GQ * HDIM + HDIM) {
    const int d = ctid - GQ * HDIM;
    knew[d] = f2bf(rope_elem(rawb[GQ * HDIM + d], rawb[GQ * HDIM + (d < H2 ? d + H2 : d - H2)], d < H2, qc, qsn));
    vnew[d] = rawb[GQ * HDIM + HDIM + d];
  }
  cbar();
  dec_attend_w<HDIM, PW, NCONS>(kc, vtc, a.kv_stride, ctx, a.scale, qs, knew, vnew, (float*)(smem + L_RED), kf, vf,
                                ao, cw, ctid, cbar);
  cbar();
  if (cw == 0 && lane == 0) stamp(a.trace, l, c, 15);
  if (ctid < GQ * HDIM / 2) gst(G + G_ATT + c * GQ * HDIM / 2 + ctid, ((const uint32_t*)ao)[ctid], tag);
  if (ctid < HDIM) {  // the new position into the cache (no other CU reads this (slot, kv head))
    bf16_t* kw = a.kv + 2 * kvl + kvbase;
    kw[(size_t)pos * HDIM + ctid] = knew[ctid];
    kw[a.kv_layer + (size_t)ctid * a.kv_stride + pos] = vnew[ctid];
  }
}

// The loader wave: this CU's weight stream through the LDS ring (see the header).
__attribute__((noinline)) __device__ void step_loader(const void* stream, char* smem, int c, int lane, int s_begin,
                                                      int total, int* err, unsigned long long* tr) {
  lint* fl = lflags(smem);
  // slot-major stream [slot][CU][16 KiB]: at any moment the 256 loaders read one contiguous
  // 4 MiB window (few pages, few DRAM rows) instead of 256 scattered per-CU regions
  const char* src = (const char*)stream + (size_t)c * SLOT;
  int pub = s_begin;  // first slot not yet published (slots pub .. s-1 are in flight)
  int spins = 0;
  bool bad = false;
#pragma unroll 1
  for (int s = s_begin; s < total; ++s) {
    const int r = s % NS;
    if (tr && lane == 0 && s % S_LAYER == 0) stamp(tr, s / S_LAYER, c, 12);
    // ring full: while the slot is still being read, publish the in-flight slots as they land
    // (oldest first, the newer ones stay in flight)
    while (lds_ld_dma(fl + F_FREE + r) != s - NS) {
      const int inflight = s - pub;
      if (inflight > 0) {
        if (inflight >= 3) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        else if (inflight == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_st_dma(fl + F_FULL + pub % NS, pub);
        ++pub;
        continue;
      }
      if (tr && lane == 0) stamp(tr, s / S_LAYER, c, 13);
      if (++spins > MAX_SPINS || ((spins & 255) == 0 && gerr(err))) {
        set_err(err);
        bad = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (bad) break;
    spins = 0;
    const char* gs = src + (size_t)s * NCU * SLOT + lane * 16;
    char* ls = smem + L_RING + r * SLOT;
#pragma unroll
    for (int p = 0; p < SLOT / 1024; ++p)
      __builtin_amdgcn_global_load_lds((gptr_t)(gs + p * 1024), (lptr_t)(ls + p * 1024), 16, 0, 2 /* nt */);
    if (lds_ld_dma(fl + F_GATH) > 0) {
      // a wave of this CU is sweeping granules: thin the stream to this one slot in flight so
      // the sweep's loads do not queue behind a refill burst (MI355X_MICROARCH.md gather-pass)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      for (; pub < s; ++pub) lds_st_dma(fl + F_FULL + pub % NS, pub);
    } else if (s - pub + 1 > FLY) {  // the oldest in-flight slot has landed once FLY newer ones remain
      asm volatile("s_waitcnt vmcnt(48)" ::: "memory");  // = FLY * 16 loads
      lds_st_dma(fl + F_FULL + pub % NS, pub);
      ++pub;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (; pub < total; ++pub) lds_st_dma(fl + F_FULL + pub % NS, pub);
}

}  // namespace

__global__ __launch_bounds__(NWV * 64) void decode_step_kernel(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  lint* fl = lflags(smem);
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = a.L;
  const int total = S_LAYER * L;
  const uint32_t tag = (uint32_t)__hip_atomic_load(a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // ring flags: full[r] / free[r] = the last slot published / released at ring position r
  // (initially the slot NS before the first one there); counters 0
  if (tid < F_N) fl[tid] = (tid < F_FREE + NS) ? (tid % NS) - NS : 0;
  __syncthreads();  // (the only workgroup barrier: the loader runs free from here on)

  if (wave == 0) {
    step_loader(a.stream, smem, c, lane, 0, total, a.err, a.trace);
    return;
  }

  // -------------------------------------------------------------------- consumers -------
  const int cw = wave - 1;       // consumer index 0..14
  bf16_t* xs = (bf16_t*)(smem + L_X);
  bf16_t* hs = (bf16_t*)(smem + L_H);
  bf16_t* as = (bf16_t*)(smem + L_A);
  const bool attn_cu = c < NKV;  // kv head c
  const int pos = a.row_pos[0], ctx = pos + 1, slot_kv = a.row_slot[0];
  int nbar = 0;
  unsigned long long* const tr = a.trace;
#define EV(e)                                  \
  do {                                         \
    if (tr && lane == 0) stamp(tr, l, c, (e)); \
  } while (0)
  auto cbar = [&]() {  // barrier over the consumer waves (LDS counter)
    ++nbar;
    if (lane == 0) lds_add(fl + F_BAR, 1);
    lds_wait_ge(fl + F_BAR, NCONS * nbar, a.err);
  };
  // wait for ring slot s, run f on it, free it
  auto on_slot = [&](int s, auto f) {
    const int r = s % NS;
    lds_wait_ge(fl + F_FULL + r, s, a.err);  // (full[r] holds the last slot published there)
    f(smem + L_RING + r * SLOT);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) lds_st(fl + F_FREE + r, s);
  };

#pragma unroll 1
  for (int l = 0; l < L; ++l) {
    // lane-derived addresses are recomputed per layer instead of being hoisted out of the
    // loop (live across it they would crowd the registers the attention and slot math need)
    int lane = tid & 63, ctid = tid - 64;
    asm volatile("" : "+v"(lane), "+v"(ctid));
    uint64_t* G = a.gran + (size_t)l * G_LAYER;
    const uint64_t* Gprev = a.gran + (size_t)(l > 0 ? l - 1 : 0) * G_LAYER;
    const int base = S_LAYER * l;
    const size_t kvl = (size_t)l * a.kv_layer;
    const size_t kvbase = ((size_t)slot_kv * NKV + c) * a.kv_stride * HDIM;

    if (a.nodeps == 2) {  // diagnostics: the loader's own pace (slots released unread)
      if (cw == 0) EV(0);
#pragma unroll 1
      for (int t = 0; t < S_LAYER; ++t)
        if ((base + t) % NCONS == cw) on_slot(base + t, [](const char*) {});
      continue;
    }
    // 1. x_l: the token embedding (layer 0, written by the previous step's finalize) or the
    //    previous layer's output granules
    if (cw == 0) {
      EV(0);
      if (l == 0) {
#pragma unroll
        for (int i = 0; i < HID / 512; ++i) *(u32x4_t*)(xs + 8 * lane + 512 * i) = *(const u32x4_t*)(a.x + 8 * lane + 512 * i);
      } else {
        // sweep once this CU's own part of x_l is out: by then the other CUs' parts are
        // close, and the sweep's loads no longer queue beside this CU's down stream
        lds_wait_ge(fl + F_XP, l, a.err);
        if (lane == 0) lds_add(fl + F_GATH, 1);
        gather_vec(Gprev + G_X, tag, xs, lane, a.err, a.nodeps);
        if (lane == 0) lds_add(fl + F_GATH, -1);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) lds_st(fl + F_RX, l + 1);
      EV(1);
    }
    // 2. qkv slots: outputs 12c + 4t .. +3, RMSNorm(x, ln1) on the fly
    {
      bool have = false;
      u32x4_t xn[4];
#pragma unroll 1
      for (int t = 0; t < S_QKV; ++t) {
        const int s = base + O_QKV + t;
        if (s % NCONS != cw) continue;
        lds_wait_ge(fl + F_RX, l + 1, a.err);
        if (!have) { norm_chunks(xs, a.ln1 + l * a.ln_stride, a.eps, lane, xn); have = true; }
        on_slot(s, [&](const char* sl) {
          float y[4];
          rows4(sl, xn, lane, y);
          if (lane < 2) gst(G + G_QKV + (12 * c + 4 * t) / 2 + lane, pack_bf2(y[2 * lane], y[2 * lane + 1]), tag);
        });
        if (t == S_QKV - 1) EV(2);
      }
    }
    // 3. attention (CUs 0..7: kv head c): q of heads 4c..4c+3, the new k and v -> RoPE ->
    //    the same per-wave / global-max arithmetic as attn_decode_kernel -> 4 heads' output
    if (attn_cu) {
      step_attention(a, smem, G, tag, c, cw, ctid, lane, l, pos, ctx, kvl, kvbase, nbar);
      if (cw == 0) EV(3);
    }
    // 4. the attention output of all heads
    if (cw == 1) {
      if (lane == 0) lds_add(fl + F_GATH, 1);
      gather_vec(G + G_ATT, tag, as, lane, a.err, a.nodeps);
      if (lane == 0) lds_add(fl + F_GATH, -1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) lds_st(fl + F_RA, l + 1);
      EV(4);
    }
    // 5. o slots: outputs 8c + 4t .. +3, then h = x + o (bf16) published
    {
      bool have = false;
      u32x4_t xn[4];
#pragma unroll 1
      for (int t = 0; t < S_O; ++t) {
        const int s = base + O_O + t;
        if (s % NCONS != cw) continue;
        lds_wait_ge(fl + F_RA, l + 1, a.err);
        if (!have) { plain_chunks(as, lane, xn); have = true; }
        on_slot(s, [&](const char* sl) {
          float y[4];
          rows4(sl, xn, lane, y);
          if (lane < 2) {
            const int n = 8 * c + 4 * t + 2 * lane;
            const float h0 = rbf(bf2f(xs[n]) + rbf(y[2 * lane])), h1 = rbf(bf2f(xs[n + 1]) + rbf(y[2 * lane + 1]));
            gst(G + G_H + n / 2, pack_bf2(h0, h1), tag);
          }
        });
        if (t == S_O - 1) EV(5);
      }
    }
    // 6. h of all columns
    if (cw == 2) {
      if (lane == 0) lds_add(fl + F_GATH, 1);
      gather_vec(G + G_H, tag, hs, lane, a.err, a.nodeps);
      if (lane == 0) lds_add(fl + F_GATH, -1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) lds_st(fl + F_RH, l + 1);
      EV(6);
    }
    // 7. gate/up slots: act 32c + 2t, +1 = SiLU(gate) * up (bf16), RMSNorm(h, ln2) on the fly,
    //    published for the down slots of every CU
    {
      bool have = false;
      u32x4_t xn[4];
#pragma unroll 1
      for (int t = 0; t < S_GU; ++t) {
        const int s = base + O_GU + t;
        if (s % NCONS != cw) continue;
        lds_wait_ge(fl + F_RH, l + 1, a.err);
        if (!have) { norm_chunks(hs, a.ln2 + l * a.ln_stride, a.eps, lane, xn); have = true; }
        on_slot(s, [&](const char* sl) {
          float y[4];  // gate 2t, gate 2t+1, up 2t, up 2t+1
          rows4(sl, xn, lane, y);
          if (lane == 0) {
            const float a0 = rbf(rbf(silu_f(rbf(y[0]))) * rbf(y[2])), a1 = rbf(rbf(silu_f(rbf(y[1]))) * rbf(y[3]));
            gst(G + G_ACT + 16 * c + t, pack_bf2(a0, a1), tag);
          }
        });
        if (lane == 0) lds_add(fl + F_GU, 1);
        if (t == S_GU - 1) EV(7);
      }
    }
    // 8. down slots: slot t = this CU's 8 output rows 8c .. 8c+7 over k = 1024 t .. +1023;
    //    its act chunk (produced by CUs 32t .. 32t+31) gathered straight into registers while
    //    the slot itself is already in the ring.  The last slot to finish sums the 8 chunks in
    //    order, adds h and publishes this CU's part of x_{l+1}.
    {
#pragma unroll 1
      for (int t = 0; t < S_D; ++t) {
        const int s = base + O_D + t;
        if (s % NCONS != cw) continue;
        // sweep once this CU's own gate/up slots are done (the other CUs' are then close, and
        // the sweep no longer queues beside this CU's gate/up stream)
        lds_wait_ge(fl + F_GU, S_GU * (l + 1), a.err);
        if (t == 0) EV(8);
        // act k = 1024 t + 8 lane + 512 j + e  ->  granule 512 t + 4 lane + 256 j + e / 2
        const uint64_t* ga = G + G_ACT + 512 * t + 4 * lane;
        if (lane == 0) lds_add(fl + F_GATH, 1);
        uint64_t gv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) gv[k] = gld(ga + 256 * (k >> 2) + (k & 3));
        uint32_t pending = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) pending |= ((uint32_t)(gv[k] >> 32) != tag && !a.nodeps) ? 1u << k : 0u;
        int spins = 0;
        while (pending) {
          if (++spins > MAX_SPINS || ((spins & 255) == 0 && gerr(a.err))) {
            set_err(a.err);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (pending & (1u << k)) gv[k] = gld(ga + 256 * (k >> 2) + (k & 3));
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if ((uint32_t)(gv[k] >> 32) == tag) pending &= ~(1u << k);
        }
        if (lane == 0) lds_add(fl + F_GATH, -1);
        u32x4_t av[2];
#pragma unroll
        for (int k = 0; k < 8; ++k) av[k >> 2][k & 3] = (uint32_t)gv[k];
        float* dp = (float*)(smem + L_DP);
        on_slot(s, [&](const char* sl) {  // slot layout [row 8][k 1024]
          u32x4_t w[8][2];
#pragma unroll
          for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int j = 0; j < 2; ++j) w[r][j] = *(const u32x4_t*)(sl + r * 2048 + j * 1024 + lane * 16);
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const float y = wave_sum_dpp(dot8(w[r][1], av[1], dot8(w[r][0], av[0], 0.f)));
            if (lane == 0) dp[8 * t + r] = y;
          }
        });
        if (lane == 0) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          if (lds_add(fl + F_DS, 1) == S_D * (l + 1) - 1) {  // the last slot: x_{l+1} = h + down
            EV(11);
            for (int k = 0; k < 4; ++k) {
              float xv[2];
              for (int e = 0; e < 2; ++e) {
                const int r = 2 * k + e;
                float d = 0.f;
                for (int u = 0; u < S_D; ++u) d += dp[8 * u + r];
                xv[e] = rbf(bf2f(hs[8 * c + r]) + rbf(d));
              }
              gst(G + G_X + 4 * c + k, pack_bf2(xv[0], xv[1]), tag);
              if (l == L - 1) ((uint32_t*)a.x)[4 * c + k] = pack_bf2(xv[0], xv[1]);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            lds_add(fl + F_XP, 1);
          }
        }
        if (t == S_D - 1) EV(9);
      }
    }
    if (gerr(a.err)) break;
  }
#undef EV
  // the last CU out advances the step tag for the next replay
  if (tid == 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (__hip_atomic_fetch_add(a.done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == NCU - 1) {
      __hip_atomic_store(a.done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.seq, (int)(tag + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------------------------------ MLP block ---------
// The MLP half of ONE layer of the one-row decode as one launch on the same engine and weight
// stream (the per-layer launch path's gate/up + down pair): h = the residual after attention
// (row 0 of a.x, written by the o_proj launch before this one), RMSNorm(h, ln2) -> gate/up
// slots -> act granules -> down slots (each gathers its act chunk from 32 CUs while its
// weights are already in the ring) -> x = h + down written back over h.  In place is safe:
// a CU writes its 8 outputs only after it has gathered act from every CU, and every CU read
// all of h before it published act.  The launch boundary carries x to the next layer (no
// granule all-gather), and the down weights stream in while act is exchanged.
__global__ __launch_bounds__(NWV * 64) void mlp_block_kernel(StepArgs a, int l) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  lint* fl = lflags(smem);
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int s_begin = S_LAYER * l + O_GU, s_end = S_LAYER * l + S_LAYER;
  const uint32_t tag = (uint32_t)__hip_atomic_load(a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tid < F_N) {  // full / free of ring position r: the slot NS before the first one there
    int v = 0;
    if (tid < 2 * NS) {
      const int r = tid % NS;
      v = s_begin + ((r - s_begin % NS) + NS) % NS - NS;
    }
    fl[tid] = v;
  }
  __syncthreads();
  if (wave == 0) {
    step_loader(a.stream, smem, c, lane, s_begin, s_end, a.err, nullptr);
    return;
  }
  const int cw = wave - 1;
  uint64_t* G = a.gran + (size_t)l * G_LAYER;
  const bf16_t* h = a.x;
  auto on_slot = [&](int s, auto f) {
    const int r = s % NS;
    lds_wait_ge(fl + F_FULL + r, s, a.err);
    f(smem + L_RING + r * SLOT);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) lds_st(fl + F_FREE + r, s);
  };
  // gate/up slots: act 32c + 2t, +1
  {
    bool have = false;
    u32x4_t xn[4];
#pragma unroll 1
    for (int t = 0; t < S_GU; ++t) {
      const int s = s_begin + t;
      if (s % NCONS != cw) continue;
      if (!have) { norm_chunks(h, a.ln2 + l * a.ln_stride, a.eps, lane, xn); have = true; }
      on_slot(s, [&](const char* sl) {
        float y[4];
        rows4(sl, xn, lane, y);
        if (lane == 0) {
          const float a0 = rbf(rbf(silu_f(rbf(y[0]))) * rbf(y[2])), a1 = rbf(rbf(silu_f(rbf(y[1]))) * rbf(y[3]));
          gst(G + G_ACT + 16 * c + t, pack_bf2(a0, a1), tag);
        }
      });
      if (lane == 0) lds_add(fl + F_GU, 1);
    }
  }
  // down slots (as in decode_step_kernel), x written back over h
  float hres[8];
#pragma unroll 1
  for (int t = 0; t < S_D; ++t) {
    const int s = s_begin + (O_D - O_GU) + t;
    if (s % NCONS != cw) continue;
    lds_wait_ge(fl + F_GU, S_GU, a.err);
    const uint64_t* ga = G + G_ACT + 512 * t + 4 * lane;
    uint64_t gv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) gv[k] = gld(ga + 256 * (k >> 2) + (k & 3));
    uint32_t pending = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) pending |= ((uint32_t)(gv[k] >> 32) != tag) ? 1u << k : 0u;
    int spins = 0;
    while (pending) {
      if (++spins > MAX_SPINS || ((spins & 255) == 0 && gerr(a.err))) {
        set_err(a.err);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (pending & (1u << k)) gv[k] = gld(ga + 256 * (k >> 2) + (k & 3));
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if ((uint32_t)(gv[k] >> 32) == tag) pending &= ~(1u << k);
    }
    u32x4_t av[2];
#pragma unroll
    for (int k = 0; k < 8; ++k) av[k >> 2][k & 3] = (uint32_t)gv[k];
    float* dp = (float*)(smem + L_DP);
    on_slot(s, [&](const char* sl) {
      u32x4_t w[8][2];
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int j = 0; j < 2; ++j) w[r][j] = *(const u32x4_t*)(sl + r * 2048 + j * 1024 + lane * 16);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const float y = wave_sum_dpp(dot8(w[r][1], av[1], dot8(w[r][0], av[0], 0.f)));
        if (lane == 0) dp[8 * t + r] = y;
      }
    });
    if (lane == 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lds_add(fl + F_DS, 1) == S_D - 1) {
#pragma unroll
        for (int r = 0; r < 8; ++r) hres[r] = bf2f(h[8 * c + r]);
        for (int k = 0; k < 4; ++k) {
          float xv[2];
          for (int e = 0; e < 2; ++e) {
            const int r = 2 * k + e;
            float d = 0.f;
            for (int u = 0; u < S_D; ++u) d += dp[8 * u + r];
            xv[e] = rbf(hres[r] + rbf(d));
          }
          ((uint32_t*)a.x)[4 * c + k] = pack_bf2(xv[0], xv[1]);
        }
      }
    }
  }
  if (tid == 64) {  // the last CU out advances the tag
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (__hip_atomic_fetch_add(a.done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == NCU - 1) {
      __hip_atomic_store(a.done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.seq, (int)(tag + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

bool step_supported(int hidden, int heads, int kv_heads, int head_dim, int ffn, int layers, int num_cu) {
  return hidden == HID && heads == NH && kv_heads == NKV && head_dim == HDIM && ffn == FFN && layers >= 1 &&
         layers <= StepArgs::kMaxLayers && num_cu == NCU;
}
size_t step_stream_bytes(int layers) { return (size_t)NCU * S_LAYER * layers * SLOT; }
size_t step_gran_elems(int layers) { return (size_t)G_LAYER * layers; }

void launch_decode_step(const StepArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(decode_step_kernel, dim3(NCU), dim3(NWV * 64), LDS_BYTES, s, a);
}
void launch_mlp_block(const StepArgs& a, int layer, hipStream_t s) {
  hipLaunchKernelGGL(mlp_block_kernel, dim3(NCU), dim3(NWV * 64), LDS_BYTES, s, a, layer);
}

// ------------------------------------------------------------------ weight stream ------
// Row-major W of one layer's matrix -> this engine's slots (every CU's share, in stream
// order).  kind 0 qkv [3072][2048], 1 o [2048][2048], 2 gate [8192][2048], 3 up, 4 down
// [2048][8192].  One thread = 16 bytes.
__global__ void step_pack_kernel(const bf16_t* __restrict__ w, char* __restrict__ stream, int kind, int layer, int L) {
  const long long n16 = (kind == 0) ? (long long)QKVN * HID / 8 : (kind == 1) ? (long long)HID * HID / 8
                        : (kind == 4) ? (long long)HID * FFN / 8 : (long long)FFN * HID / 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n16; i += (long long)gridDim.x * blockDim.x) {
    int cu, s, off;
    if (kind == 4) {  // Wd[n][k]: CU = n / 8, slot t = k / 1024, layout [row n % 8][k % 1024]
      const int n = (int)(i / (FFN / 8)), k = (int)(i % (FFN / 8)) * 8;
      cu = n / 8;
      s = O_D + k / 1024;
      off = (n % 8) * 2048 + (k % 1024) * 2;
    } else {
      const int row = (int)(i / (HID / 8)), k = (int)(i % (HID / 8)) * 8;
      int t, r;
      if (kind == 0) { cu = row / 12; t = (row % 12) / 4; r = row % 4; s = O_QKV + t; }
      else if (kind == 1) { cu = row / 8; t = (row % 8) / 4; r = row % 4; s = O_O + t; }
      else {  // gate / up row j: CU j / 32, slot (j % 32) / 2, rows gate 2t, gate 2t+1, up 2t, up 2t+1
        cu = row / 32;
        t = (row % 32) / 2;
        r = (kind == 2 ? 0 : 2) + (row % 2);
        s = O_GU + t;
      }
      off = r * 4096 + k * 2;
    }
    char* dst = stream + (((size_t)S_LAYER * layer + s) * NCU + cu) * SLOT + off;
    *(u32x4_t*)dst = *(const u32x4_t*)(w + i * 8);
  }
}

void launch_step_pack(const bf16_t* w, void* stream, int kind, int layer, int L, hipStream_t s) {
  hipLaunchKernelGGL(step_pack_kernel, dim3(4096), dim3(256), 0, s, w, (char*)stream, kind, layer, L);
}

}  // namespace tts
