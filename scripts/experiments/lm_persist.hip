// lm_persist.hip — the one-row decode step's whole transformer stack as ONE persistent
// launch (TTS-1 geometry: hidden 2048, 32 q / 8 kv heads of 64, ffn 8192; 256 CUs).
//
// Why: as a chain of dependent launches a batch-1 layer costs ~40 us although its weights
// stream in ~19 us at 6.5 TB/s — every launch pays its ramp, its dependent prologue and its
// tail while HBM idles (scripts/chain_probe.hip: four dependent launches per layer cost
// 21 us with no weight bytes at all).  Here every CU runs one 16-wave workgroup for the
// whole step; each wave streams its static sequence of 1 KiB weight tiles (qkv / o / gate-up
// / down tiles of every layer, in order) through a private LDS-DMA ring that stays D tiles
// ahead of its consumer, ACROSS phase and layer boundaries: while a workgroup waits for the
// vector its next phase needs, its ring keeps loading the tiles that phase (and the next)
// will multiply.  Vectors move between workgroups as 8-byte granules {payload, tag}
// (one agent-scope store each; tag = the step's sequence number, so a stale granule never
// matches) plus one flag word per producing unit that a single consumer wave polls.
//
// Arithmetic is bit-identical to the launch path at one row (lm_gemm_kernel.h): the same
// split-K partition per matrix (qkv / o / down: 16 K parts of contiguous k-tiles, gate/up:
// 4), the same MFMA accumulation order inside a part, the partials summed in part order,
// the same RMSNorm segment order, the same attention chunk math (lm_attn_chunk.h) and the
// o_proj prologue's chunk-merge grouping.  tests/test_gpu_persist.py compares the two paths
// id for id.
//
// Workgroup roles (per layer; b = workgroup):
//   A  b <   128 : gate/up units 2b, 2b+1; down unit b
//   B  b in [128,192): qkv units b-128 and b; o unit b-128; gate/up
//   C  b in [192,256): qkv unit b-128; o unit b-128; gate/up; attention task b-192
//                      (kv head (b-192) % 8, chunk slot (b-192) / 8); slot 0 merges its
//                      kv head's chunks into the attention output
// Reference semantics: transformers LlamaDecoderLayer (modeling_llama.py:284-326) as the
// launch path restates it (see lm_gemm.hip header).
#include <algorithm>
#include <cstdio>
#include <stdexcept>

#include "hip_common.h"
#include "lm_attn_chunk.h"
#include "lm_kernels.h"
#include "lm_persist.h"

namespace tts {

namespace {

constexpr int PW = 16, PNT = PW * 64;
constexpr int HID = 2048, NH = 32, NKV = 8, HDIM = 64, QKVN = (NH + 2 * NKV) * HDIM, FFN = 8192;
constexpr int GQ = NH / NKV;           // q heads per kv head
constexpr int SPLIT = 128;             // decode attention chunk (decode_split(64))
constexpr int NSLOT_ATT = 8;           // chunk slots per kv head (chunk c -> slot c % 8)
constexpr int NSMAX = 8;               // chunks per row (max_seq <= 1024)
constexpr int NWG = 256;
constexpr int MAX_SPINS = 1 << 16;

// granule slab of one layer (u64 {payload, tag})
constexpr int G_X = 0;                           // layer input (bf16 pairs; previous layer's down)
constexpr int G_QKV = G_X + HID / 2;             // q | k | v before RoPE (bf16 pairs)
constexpr int G_AO = G_QKV + QKVN / 2;           // merged attention output (bf16 pairs)
constexpr int G_H = G_AO + HID / 2;              // residual after attention (bf16 pairs)
constexpr int G_ACT = G_H + HID / 2;             // SwiGLU output (bf16 pairs)
constexpr int G_PO = G_ACT + FFN / 2;            // chunk partial o [NH][NSMAX][HDIM] (f32)
constexpr int G_PML = G_PO + NH * NSMAX * HDIM;  // chunk (m, l) [NH][NSMAX][2] (f32)
constexpr int G_SLAB = G_PML + NH * NSMAX * 2;
// flag slab of one layer: one word per producing unit, = the step's tag once published
constexpr int F_X = 0;              // 128 down units
constexpr int F_QKV = F_X + 128;    // 192 qkv units
constexpr int F_PART = F_QKV + 192; // 64 attention tasks (kv head, chunk slot)
constexpr int F_AO = F_PART + 64;   // 8 merges (kv heads)
constexpr int F_H = F_AO + 8;       // 128 o units
constexpr int F_ACT = F_H + 128;    // 256 gate/up workgroups (units 2b, 2b+1 = act k-tile b)
constexpr int F_SLAB = F_ACT + 256 + 8;

enum { MAT_QKV = 0, MAT_O = 1, MAT_GU = 2, MAT_D = 3 };
enum { ROLE_A = 0, ROLE_B = 1, ROLE_C = 2 };

// LDS carve-up (bytes)
constexpr int L_V = 4096;                     // one bf16 vector of HID
constexpr int L_RED = 16 * 16 * 4;            // split-K partials (row 0 of each wave's tile)
constexpr int L_MISC = 64 + 4 * 8 * 2 * 4;    // RMSNorm segment sums, merge (m, l)
constexpr int L_ACT = FFN * 2;                // role A: the act vector (each wave its slice)
constexpr int ATT_KROW = HDIM + 8;
constexpr int L_ATT = 2 * SPLIT * ATT_KROW * 2 + GQ * HDIM * 4 + GQ * SPLIT * 4 + (GQ * HDIM / 2 + HDIM) * 4 +
                      HDIM * 2;
constexpr int ring_slots(int role) { return role == ROLE_C ? 6 : 8; }
constexpr int lds_bytes(int role) {
  return PW * ring_slots(role) * 1024 + 2 * L_V + L_RED + L_MISC +
         (role == ROLE_A ? L_ACT : 0) + (role == ROLE_C ? L_ATT : 0);
}
static_assert(lds_bytes(ROLE_A) <= 160 * 1024 && lds_bytes(ROLE_B) <= 160 * 1024 &&
              lds_bytes(ROLE_C) <= 160 * 1024, "persistent step LDS");

TTS_DEV uint64_t gload(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
TTS_DEV void gstore(uint64_t* p, uint32_t payload, uint32_t tag) {
  __hip_atomic_store(p, ((uint64_t)tag << 32) | payload, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
TTS_DEV int fload(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
TTS_DEV void fstore(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
TTS_DEV void raise_err(int* err) { __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// granule payload once its tag is this step's (bounded: sets err and returns what is there)
TTS_DEV uint32_t gwait(const uint64_t* p, uint32_t tag, int* err) {
  uint64_t v = gload(p);
  int spins = 0;
  while ((uint32_t)(v >> 32) != tag) {
    if (++spins > MAX_SPINS || ((spins & 63) == 0 && fload(err))) {
      raise_err(err);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
    v = gload(p);
  }
  return (uint32_t)v;
}

// one wave waits until flags[i] == tag for i < n (lane i, i + 64, ...); uniform return
TTS_DEV void wave_wait_flags(const int* flags, int n, int tag, int* err, int lane) {
  int spins = 0;
  while (true) {
    bool ok = true;
    for (int i = lane; i < n; i += 64) ok = ok && (fload(flags + i) == tag);
    if (__builtin_amdgcn_ballot_w64(!ok) == 0) return;
    if (++spins > MAX_SPINS || ((spins & 63) == 0 && fload(err))) {
      if (lane == 0) raise_err(err);
      return;
    }
    __builtin_amdgcn_s_sleep(4);
  }
}

// diagnostics (PersistArgs::trace): thread 0 of each workgroup stamps the 100 MHz clock
// at the phase points of each layer: trace[(b * L + l) * 32 + ev]
TTS_DEV void stamp(const PersistArgs& a, int b, int l, int ev) {
  if (a.trace && threadIdx.x == 0) a.trace[((size_t)b * a.L + l) * 32 + ev] = __builtin_amdgcn_s_memrealtime();
}

TTS_DEV void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(waitcnt_lgkm0());
  __builtin_amdgcn_s_barrier();
}

struct PCtx {
  const PersistArgs* a;
  char* smem;
  int b, tid, lane, wave;
  uint32_t tag;
  // LDS regions
  bf16_t *v1, *v2, *act;
  float* red;
  float* misc;
  char* ring;
  char* att;
};

// ------------------------------------------------------------------ weight ring -----
// segment descriptor of (matrix, unit, member g, K part) in the wave's sequence: tile i is
// base + (i >> kus) * stride + (i & (ku - 1)) of the matrix's stream-plan layout
struct Seg { int mat, kus, cnt, base, stride; };
TTS_DEV Seg make_seg(const PersistArgs& a, int mat, int u, int g, int kp) {
  int ng = 1, ks = 16, ku = 2, ur = a.ur_qkv, units = QKVN / 16, KT = HID / 32, kc = 1, cnt = 4;
  if (mat == MAT_O) { ur = a.ur_o; units = HID / 16; }
  if (mat == MAT_GU) { ng = 2; ks = 4; ur = a.ur_gu; units = FFN / 16; cnt = 16; }
  if (mat == MAT_D) { ku = 4; ur = a.ur_d; units = HID / 16; KT = FFN / 32; kc = 4; cnt = 16; }
  const int KTc = KT / kc, kt_pc = KTc / ks, Sc = kt_pc / ku;
  auto kt_of = [&](int i) { const int st = i / ku, ch = st / Sc; return ch * KTc + kp * kt_pc + (st - ch * Sc) * ku + i % ku; };
  const long long b0 = plan_tile(ng, ks, ku, ur, units, KT, kc, u * ng + g, kt_of(0));
  const long long b1 = plan_tile(ng, ks, ku, ur, units, KT, kc, u * ng + g, kt_of(ku));
  Seg r;
  r.mat = mat; r.kus = ku == 4 ? 2 : 1; r.cnt = cnt; r.base = (int)b0; r.stride = (int)(b1 - b0);
  return r;
}

// The wave's tile sequence per layer, by role (phase order):
//   A: qkv (unit b+64, K part w), gate/up (unit 2b + w/8, member (w/4)&1, K part w&3), down (unit b, part w)
//   B: qkv (unit b-128, part w), o (unit b-128, part w), gate/up
//   C: o (unit b-128, part w), gate/up   (+ the attention task b-192)
template <int ROLE>
TTS_DEV Seg role_seg(const PersistArgs& a, int b, int w, int s) {
  const int gu_u = 2 * b + (w >> 3), gu_g = (w >> 2) & 1, gu_kp = w & 3;
  if (ROLE == ROLE_A) {
    if (s == 0) return make_seg(a, MAT_QKV, b + 64, 0, w);
    if (s == 1) return make_seg(a, MAT_GU, gu_u, gu_g, gu_kp);
    return make_seg(a, MAT_D, b, 0, w);
  }
  if (ROLE == ROLE_B) {
    if (s == 0) return make_seg(a, MAT_QKV, b - 128, 0, w);
    if (s == 1) return make_seg(a, MAT_O, b - 128, 0, w);
    return make_seg(a, MAT_GU, gu_u, gu_g, gu_kp);
  }
  if (s == 0) return make_seg(a, MAT_O, b - 128, 0, w);
  return make_seg(a, MAT_GU, gu_u, gu_g, gu_kp);
}
template <int ROLE>
constexpr int role_nseg() { return ROLE == ROLE_C ? 2 : 3; }

// Per-wave LDS-DMA ring: D tiles in flight, D + 1 slots (the refill lands in the slot read
// by the previous step).  Waits are counted on vmcnt: a wave's loads retire in order, so
// "at most D - 1 younger loads outstanding" means the oldest tile has landed (any younger
// non-ring load only makes the wait stricter).
template <int ROLE, int D>
struct Ring {
  static constexpr int NS = D + 1;
  const PersistArgs* a;
  char* base;  // this wave's slots (LDS)
  int lane, b, w;
  int l_iss = 0, s_iss = 0, i_iss = 0, n_iss = 0, n_con = 0;
  Seg cur;
  const bf16_t* cur_w = nullptr;

  TTS_DEV void load_seg() {
    cur = role_seg<ROLE>(*a, b, w, s_iss);
    cur_w = a->w[l_iss][cur.mat];
  }
  TTS_DEV void issue() {
    if (l_iss >= a->L) return;
    const int off = cur.base + (i_iss >> cur.kus) * cur.stride + (i_iss & ((1 << cur.kus) - 1));
    const bf16_t* src = cur_w + (size_t)off * 512 + lane * 8;
    __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(base + (n_iss % NS) * 1024), 16, 0, 2 /* nt */);
    ++n_iss;
    if (++i_iss == cur.cnt) {
      i_iss = 0;
      if (++s_iss == role_nseg<ROLE>()) {
        s_iss = 0;
        ++l_iss;
      }
      if (l_iss < a->L) load_seg();
    }
  }
  TTS_DEV void prime() {
    load_seg();
#pragma unroll
    for (int j = 0; j < D; ++j) issue();
  }
  // B fragment of the next tile (waits for its DMA)
  TTS_DEV u32x4_t next() {
    if (n_iss - n_con - 1 >= D - 1) __builtin_amdgcn_s_waitcnt(waitcnt_vm(D - 1));
    else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    const u32x4_t v = *(const u32x4_t*)(base + (n_con % NS) * 1024 + lane * 16);
    ++n_con;
    return v;
  }
};

TTS_DEV f32x4_t mfma_step(u32x4_t a, u32x4_t b, f32x4_t acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                acc, 0, 0, 0);
}

// one tile: B from the ring, A = the LDS vector's k-tile kt (all 16 A rows = row 0, as the
// launch path's duplicated rows), refill; the scheduling barrier keeps the next step's LDS
// reads from being hoisted (their registers would spill)
template <class R>
TTS_DEV f32x4_t tile_step(R& ring, const bf16_t* vec, int kt, int lane, f32x4_t acc) {
  const u32x4_t bw = ring.next();
  const u32x4_t av = *(const u32x4_t*)(vec + kt * 32 + 8 * (lane >> 4));
  acc = mfma_step(av, bw, acc);
  ring.issue();
  __builtin_amdgcn_sched_barrier(0);
  return acc;
}

// attn_chunk_softmax (lm_attn_chunk.h) with the same arithmetic, the query re-read from
// LDS for each lane position (a compiler barrier between the two): the launch path's form
// keeps the whole query (64 floats) in registers across both, which this kernel's register
// budget (the weight ring, 16 waves) cannot hold
template <int D, int SPLIT_>
TTS_DEV void chunk_softmax_lean(const bf16_t* Ks, const float* qg, int n, float scale, int lane, float* psg,
                                float& m_out, float& l_out) {
  constexpr int KROW = D + 8, CH = D / 8, PPL = SPLIT_ / 64;
  float sc[PPL];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const float* qj = qg;
    asm volatile("" : "+v"(qj));  // (a fresh pointer per position: the query is re-read)
    const int tl = lane + 64 * j;
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const u32x4_t kv = *(const u32x4_t*)(Ks + tl * KROW + c * 8);
      const float4 q0 = *(const float4*)(qj + c * 8);
      const float4 q1 = *(const float4*)(qj + c * 8 + 4);
      acc += q0.x * bf_lo(kv[0]) + q0.y * bf_hi(kv[0]) + q0.z * bf_lo(kv[1]) + q0.w * bf_hi(kv[1]) +
             q1.x * bf_lo(kv[2]) + q1.y * bf_hi(kv[2]) + q1.z * bf_lo(kv[3]) + q1.w * bf_hi(kv[3]);
    }
    sc[j] = (tl < n) ? acc * scale : -INFINITY;
    mx = fmaxf(mx, sc[j]);
  }
  const float m = wave_max_dpp(mx);
  float lsum = 0.f;
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const float p = (lane + 64 * j < n) ? expf(sc[j] - m) : 0.f;
    lsum += p;
    psg[lane + 64 * j] = rbf(p);
  }
  m_out = m;
  l_out = wave_sum_dpp(lsum);
}

// --------------------------------------------------------------- vector gathers -----
// x / h / attention output: 1024 granules (one per thread) into an LDS vector, after one
// wave saw every producer's flag
TTS_DEV void gather_vec(PCtx& c, const uint64_t* gsrc, const int* flags, int nflags, bf16_t* dst, int l = 0,
                        int ev = -1) {
  if (c.wave == 0) wave_wait_flags(flags, nflags, (int)c.tag, c.a->err, c.lane);
  __builtin_amdgcn_s_barrier();
  if (ev >= 0) stamp(*c.a, c.b, l, ev);
  ((uint32_t*)dst)[c.tid] = gwait(gsrc + c.tid, c.tag, c.a->err);
  lds_barrier();
}

// RMSNorm of the LDS vector src -> dst (the launch path's canonical order: 16-B chunk sums,
// DPP wave sums per 512-value segment, segments in order; bf16(w * bf16(x * r)))
TTS_DEV void rmsnorm_lds(PCtx& c, const bf16_t* src, const bf16_t* w, bf16_t* dst) {
  u32x4_t g = {0u, 0u, 0u, 0u};
  if (c.tid < HID / 8) g = *(const u32x4_t*)(w + c.tid * 8);  // (in flight during the sums)
  if (c.wave < HID / 512) {
    const float s = wave_sum_dpp(chunk_sumsq(*(const u32x4_t*)(src + (c.wave * 64 + c.lane) * 8)));
    if (c.lane == 0) c.misc[c.wave] = s;
  }
  lds_barrier();
  float ss = 0.f;
  for (int sg = 0; sg < HID / 512; ++sg) ss += c.misc[sg];
  const float r = 1.0f / sqrtf(ss / (float)HID + c.a->eps);
  if (c.tid < HID / 8) {
    u32x4_t v = *(const u32x4_t*)(src + c.tid * 8);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float lo = rbf(bf_lo(g[q]) * rbf(bf_lo(v[q]) * r));
      const float hi = rbf(bf_hi(g[q]) * rbf(bf_hi(v[q]) * r));
      v[q] = pack_bf2(lo, hi);
    }
    *(u32x4_t*)(dst + c.tid * 8) = v;
  }
  lds_barrier();
}

// split-K combine of one 16-column unit over the 16 waves (K parts in order) -> wave 0
// lanes 0..15 hold the column sums
TTS_DEV float combine16(PCtx& c, f32x4_t acc) {
  if (c.lane < 16) c.red[c.wave * 16 + c.lane] = acc[0];
  lds_barrier();
  float s = acc[0];
  if (c.wave == 0) {
    for (int p = 1; p < PW; ++p) s += c.red[p * 16 + (c.lane & 15)];
  }
  return s;
}

// publish lanes 0..15's 16 bf16 columns [n0, n0 + 16) as 8 granules
TTS_DEV void publish16(PCtx& c, uint64_t* gdst, int n0, float v) {
  const uint32_t mine = (uint32_t)f2bf(v);
  const uint32_t other = (uint32_t)__shfl_xor((int)mine, 1, 64);
  if (c.lane < 16 && !(c.lane & 1)) gstore(gdst + (n0 + c.lane) / 2, (other << 16) | mine, c.tag);
}

// ----------------------------------------------------------------------- phases -----
template <class R>
TTS_DEV void phase_qkv(PCtx& c, R& ring, int l, int u) {
  const PersistArgs& a = *c.a;
  uint64_t* slab = a.gran + (size_t)l * G_SLAB;
  int* fl = a.flags + (size_t)l * F_SLAB;
  if (l == 0) {
    ((uint32_t*)c.v1)[c.tid] = ((const uint32_t*)a.x)[c.tid];
    lds_barrier();
  } else {
    gather_vec(c, slab + G_X, fl + F_X, 128, c.v1, l, 11);
  }
  rmsnorm_lds(c, c.v1, a.ln[l][0], c.v2);
  stamp(a, c.b, l, 1);
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int i = 0; i < 4; ++i) acc = tile_step(ring, c.v2, c.wave * 4 + i, c.lane, acc);
  stamp(a, c.b, l, 14);
  const float s = combine16(c, acc);
  if (c.wave == 0) {
    publish16(c, slab + G_QKV, u * 16, s);
    if (c.lane == 0) fstore(fl + F_QKV + u, (int)c.tag);
  }
  lds_barrier();  // (red reused)
}

// attention task t: kv head t % 8, chunks t / 8, t / 8 + 8, ... (as fattn_consumer)
TTS_DEV void phase_attn(PCtx& c, int l, int t) {
  constexpr int D = HDIM, KROW = ATT_KROW, CH = D / 8, H2 = D / 2, G = GQ;
  const PersistArgs& a = *c.a;
  uint64_t* slab = a.gran + (size_t)l * G_SLAB;
  int* fl = a.flags + (size_t)l * F_SLAB;
  const int kvh = t % NKV, c0 = t / NKV;
  const int slot = a.row_slot[0], pos = a.row_pos[0], ctx = pos + 1;
  if (c0 * SPLIT < ctx) {
    bf16_t* Ks = (bf16_t*)c.att;
    bf16_t* Vs = Ks + SPLIT * KROW;
    float* qs = (float*)(Vs + SPLIT * KROW);
    float* ps = qs + G * D;
    uint32_t* raw = (uint32_t*)(ps + G * SPLIT);
    const bf16_t* rawb = (const bf16_t*)raw;
    bf16_t* knew = (bf16_t*)(raw + G * D / 2 + D);
    const int tid = c.tid, lane = c.lane, wave = c.wave;
    const bool has_new = ((pos / SPLIT) - c0) % NSLOT_ATT == 0;
    const size_t cbase = ((size_t)slot * NKV + kvh) * a.max_seq * D;
    bf16_t* kcache = a.kv + (size_t)l * 2 * a.kv_layer;
    bf16_t* vcache = kcache + a.kv_layer;
    const bf16_t* kc = kcache + cbase;
    const bf16_t* vc = vcache + cbase;
    u32x4_t kr4, vr4;
    auto load_chunk = [&](int sp) {
      const int t0 = sp * SPLIT, t1 = min(t0 + SPLIT, ctx);
      const int q = min(tid, SPLIT * CH - 1), tl = q / CH, cc = q % CH;
      const int tt = (t0 + tl < t1) ? t0 + tl : t0;
      kr4 = *(const u32x4_t*)(kc + (size_t)tt * D + cc * 8);
      vr4 = *(const u32x4_t*)(vc + (size_t)tt * D + cc * 8);
    };
    auto stage_chunk = [&](int sp) {
      const int t0 = sp * SPLIT, t1 = min(t0 + SPLIT, ctx);
      const int q = tid, tl = q / CH, cc = q % CH, tt = t0 + tl;
      if (q < SPLIT * CH && tt < t1 && tt != pos) {
        *(u32x4_t*)(Ks + tl * KROW + cc * 8) = kr4;
        *(u32x4_t*)(Vs + tl * KROW + cc * 8) = vr4;
      }
    };
    load_chunk(c0);
    const int qi = min(tid, G * D - 1), qd = qi % D;
    const float qc = bf2f(a.rope_cos[(size_t)pos * D + qd]), qsn = bf2f(a.rope_sin[(size_t)pos * D + qd]);
    stage_chunk(c0);
    // q / k / v of this kv group: 16 q units, 4 k units, 4 v units
    if (wave == 0) {
      int ok_spins = 0;
      while (true) {
        int u = -1;
        if (lane < 16) u = kvh * 16 + lane;
        else if (lane < 20) u = NH * D / 16 + kvh * 4 + (lane - 16);
        else if (lane < 24) u = (NH + NKV) * D / 16 + kvh * 4 + (lane - 20);
        const bool ok = u < 0 || fload(fl + F_QKV + u) == (int)c.tag;
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        if (++ok_spins > MAX_SPINS || ((ok_spins & 63) == 0 && fload(a.err))) {
          if (lane == 0) raise_err(a.err);
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
    }
    __builtin_amdgcn_s_barrier();
    stamp(a, c.b, l, 12);
    const int nq = G * D / 2, ngr = has_new ? nq + D : nq;
    if (tid < ngr) {
      int col;
      if (tid < nq) col = kvh * G * D + 2 * tid;
      else if (tid < nq + D / 2) col = NH * D + kvh * D + 2 * (tid - nq);
      else col = NH * D + NKV * D + kvh * D + 2 * (tid - nq - D / 2);
      raw[tid] = gwait(slab + G_QKV + col / 2, c.tag, a.err);
    }
    lds_barrier();
    stamp(a, c.b, l, 13);
    if (tid < G * D) {
      const int g = tid / D;
      qs[tid] = rope_elem(rawb[tid], rawb[g * D + (qd < H2 ? qd + H2 : qd - H2)], qd < H2, qc, qsn);
    }
    if (has_new && tid < D) {
      const bf16_t kb = f2bf(rope_elem(rawb[G * D + tid], rawb[G * D + (tid < H2 ? tid + H2 : tid - H2)],
                                       tid < H2, qc, qsn));
      knew[tid] = kb;
      kcache[cbase + (size_t)pos * D + tid] = kb;
      vcache[cbase + (size_t)pos * D + tid] = rawb[G * D + D + tid];
    }
    for (int sp = c0; sp * SPLIT < ctx; sp += NSLOT_ATT) {
      const int t0 = sp * SPLIT, t1 = min(t0 + SPLIT, ctx), n = t1 - t0;
      if (sp != c0) {
        lds_barrier();
        stage_chunk(sp);
      }
      if (pos >= t0 && pos < t1 && tid < D) {
        Ks[(pos - t0) * KROW + tid] = knew[tid];
        Vs[(pos - t0) * KROW + tid] = rawb[G * D + D + tid];
      }
      lds_barrier();
      if (sp == c0) stamp(a, c.b, l, 16);
      if ((sp + NSLOT_ATT) * SPLIT < ctx) load_chunk(sp + NSLOT_ATT);
      if (wave < G) {
        float m, lsum;
        chunk_softmax_lean<D, SPLIT>(Ks, qs + wave * D, n, a.scale, lane, ps + wave * SPLIT, m, lsum);
        if (sp == c0) stamp(a, c.b, l, 17);
        float ov[D / 64];
        attn_chunk_pv<D, SPLIT>(Vs, ps + wave * SPLIT, n, lane, ov);
        const float o = ov[0];
        if (sp == c0) stamp(a, c.b, l, 18);
        const int hh = kvh * G + wave;
        gstore(slab + G_PO + ((size_t)hh * NSMAX + sp) * D + lane, __float_as_uint(o), c.tag);
        if (lane == 0) {
          gstore(slab + G_PML + ((size_t)hh * NSMAX + sp) * 2 + 0, __float_as_uint(m), c.tag);
          gstore(slab + G_PML + ((size_t)hh * NSMAX + sp) * 2 + 1, __float_as_uint(lsum), c.tag);
        }
      }
    }
  }
  lds_barrier();
  if (c.tid == 0) fstore(fl + F_PART + t, (int)c.tag);
}

// merge of kv head kvh's chunk partials (slot-0 workgroups): the o_proj prologue's
// register-staged merge (lm_gemm_kernel.h, early_o) per output dimension, its chunk groups
// (agroups 4, acpg = ceil(NS / 4) chunks each, summed in group order)
TTS_DEV void phase_merge(PCtx& c, int l, int kvh) {
  const PersistArgs& a = *c.a;
  uint64_t* slab = a.gran + (size_t)l * G_SLAB;
  int* fl = a.flags + (size_t)l * F_SLAB;
  if (c.wave == 0) {
    int spins = 0;
    while (true) {
      const bool ok = c.lane >= NSLOT_ATT || fload(fl + F_PART + c.lane * NKV + kvh) == (int)c.tag;
      if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
      if (++spins > MAX_SPINS || ((spins & 63) == 0 && fload(a.err))) {
        if (c.lane == 0) raise_err(a.err);
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  __builtin_amdgcn_s_barrier();
  // the kv group's chunk statistics (m, l) once into LDS, then each thread its dimension
  const int pos = a.row_pos[0];
  const int ns = (pos + SPLIT) / SPLIT;
  float* mls = c.misc + 16;  // [GQ][NSMAX][2]  (L_MISC covers it)
  if (c.tid < GQ * NSMAX * 2) {
    const int g = c.tid / (NSMAX * 2), s = (c.tid / 2) % NSMAX;
    mls[c.tid] = s < ns ? __uint_as_float(gwait(slab + G_PML + (size_t)(kvh * GQ + g) * NSMAX * 2 + (c.tid % (NSMAX * 2)),
                                                c.tag, a.err))
                        : 0.f;
  }
  lds_barrier();
  if (c.tid < GQ * HDIM) {
    const int g = c.tid / HDIM, d = c.tid % HDIM, hh = kvh * GQ + g;
    const int NS = a.NS, agroups = 4, acpg = (NS + agroups - 1) / agroups;
    constexpr int CPG = 2;
    float po[NSMAX];
    const float* ms = mls + g * NSMAX * 2;  // (m, l) pairs of the head's chunks
    const uint64_t* ppo = slab + G_PO + (size_t)hh * NSMAX * HDIM + d;
    uint64_t vo[NSMAX];
#pragma unroll
    for (int s = 0; s < NSMAX; ++s)  // one round of loads in flight (the flags were seen)
      if (s < ns) vo[s] = gload(ppo + s * HDIM);
#pragma unroll
    for (int s = 0; s < NSMAX; ++s)
      po[s] = s < ns ? __uint_as_float((uint32_t)(vo[s] >> 32) == c.tag ? (uint32_t)vo[s] : gwait(ppo + s * HDIM, c.tag, a.err))
                     : 0.f;
    float mx = -INFINITY;
#pragma unroll
    for (int s = 0; s < NSMAX; ++s) if (s < ns) mx = fmaxf(mx, ms[2 * s]);
    float lt = 0.f;
#pragma unroll
    for (int s = 0; s < NSMAX; ++s) if (s < ns) lt += ms[2 * s + 1] * expf(ms[2 * s] - mx);
    const float il = 1.0f / lt;
    float o = 0.f;
    for (int grp = 0; grp < agroups; ++grp) {
      float og = 0.f;
#pragma unroll
      for (int i = 0; i < CPG; ++i) {
        const int s = grp * acpg + i;
        if (i < acpg && s < ns) {
          float pv = 0.f;
#pragma unroll
          for (int q = 0; q < NSMAX; ++q) if (q == s) pv = po[q];
          og += pv * (expf(ms[2 * s] - mx) * il);
        }
      }
      o = grp == 0 ? og : o + og;
    }
    const uint32_t mine = (uint32_t)f2bf(o);
    const uint32_t other = (uint32_t)__shfl_xor((int)mine, 1, 64);
    if (!(d & 1)) gstore(slab + G_AO + (hh * HDIM + d) / 2, (other << 16) | mine, c.tag);
  }
  lds_barrier();
  if (c.tid == 0) fstore(fl + F_AO + kvh, (int)c.tag);
}

template <class R>
TTS_DEV void phase_o(PCtx& c, R& ring, int l, int u, bool have_x) {
  const PersistArgs& a = *c.a;
  uint64_t* slab = a.gran + (size_t)l * G_SLAB;
  int* fl = a.flags + (size_t)l * F_SLAB;
  gather_vec(c, slab + G_AO, fl + F_AO, NKV, c.v2);
  stamp(a, c.b, l, 4);
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int i = 0; i < 4; ++i) acc = tile_step(ring, c.v2, c.wave * 4 + i, c.lane, acc);
  const float s = combine16(c, acc);
  if (c.wave == 0) {
    const int n = u * 16 + (c.lane & 15);
    float xr;  // residual x_l: in LDS where this workgroup gathered it (qkv phase), else its granules
    if (have_x) {
      xr = bf2f(c.v1[n]);
    } else if (l == 0) {
      xr = bf2f(a.x[n]);
    } else {
      const uint32_t g = gwait(slab + G_X + n / 2, c.tag, a.err);
      xr = (n & 1) ? bf_hi(g) : bf_lo(g);
    }
    const float h = bf2f(f2bf(xr + rbf(s)));  // residual: x_l + o
    publish16(c, slab + G_H, u * 16, h);
    if (c.lane == 0) fstore(fl + F_H + u, (int)c.tag);
  }
  lds_barrier();
}

template <class R>
TTS_DEV void phase_gu(PCtx& c, R& ring, int l) {
  const PersistArgs& a = *c.a;
  uint64_t* slab = a.gran + (size_t)l * G_SLAB;
  int* fl = a.flags + (size_t)l * F_SLAB;
  gather_vec(c, slab + G_H, fl + F_H, 128, c.v1, l, 15);  // h (raw: the down residual)
  rmsnorm_lds(c, c.v1, a.ln[l][1], c.v2);
  stamp(a, c.b, l, 6);
  const int kp = c.wave & 3;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int i = 0; i < 16; ++i) acc = tile_step(ring, c.v2, kp * 16 + i, c.lane, acc);
  // partials [unit][g][kp][16]; the (g 0, kp 0) wave of each unit finishes
  if (c.lane < 16) c.red[c.wave * 16 + c.lane] = acc[0];
  lds_barrier();
  if ((c.wave & 7) == 0) {
    const int ug = c.wave >> 3;
    const float* r = c.red + ug * 8 * 16;
    float gt = acc[0];
    for (int p = 1; p < 4; ++p) gt += r[p * 16 + (c.lane & 15)];
    float up = r[4 * 16 + (c.lane & 15)];
    for (int p = 1; p < 4; ++p) up += r[(4 + p) * 16 + (c.lane & 15)];
    const float v = rbf(silu_f(rbf(gt))) * rbf(up);
    const int unit = 2 * c.b + ug;
    publish16(c, slab + G_ACT, unit * 16, v);
  }
  lds_barrier();
  if (c.tid == 0) fstore(fl + F_ACT + c.b, (int)c.tag);
  stamp(a, c.b, l, 7);
}

template <class R>
TTS_DEV void phase_down(PCtx& c, R& ring, int l) {
  const PersistArgs& a = *c.a;
  uint64_t* slab = a.gran + (size_t)l * G_SLAB;
  int* fl = a.flags + (size_t)l * F_SLAB;
  const int kp = c.wave;
  // this wave's K part: k-tiles ch * 64 + kp * 4 + j (ch, j < 4) = act of gate/up
  // workgroups b = kt (their units 2b, 2b+1 are the k-tile's 32 columns)
  {
    int spins = 0;
    while (true) {
      bool ok = true;
      if (c.lane < 16) ok = fload(fl + F_ACT + (c.lane >> 2) * 64 + kp * 4 + (c.lane & 3)) == (int)c.tag;
      if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
      if (++spins > MAX_SPINS || ((spins & 63) == 0 && fload(a.err))) {
        if (c.lane == 0) raise_err(a.err);
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
  {
    int gi[4];
    uint64_t v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = c.lane + 64 * q, m = p >> 4, e = p & 15;
      gi[q] = ((m >> 2) * 64 + kp * 4 + (m & 3)) * 16 + e;
      v[q] = gload(slab + G_ACT + gi[q]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
      ((uint32_t*)c.act)[gi[q]] =
          (uint32_t)(v[q] >> 32) == c.tag ? (uint32_t)v[q] : gwait(slab + G_ACT + gi[q], c.tag, a.err);
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_lgkm0());
  stamp(a, c.b, l, 8);
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int i = 0; i < 16; ++i) acc = tile_step(ring, c.act, (i >> 2) * 64 + kp * 4 + (i & 3), c.lane, acc);
  const float s = combine16(c, acc);
  if (c.wave == 0) {
    const int u = c.b;
    const int n = u * 16 + (c.lane & 15);
    const float xn = bf2f(f2bf(bf2f(c.v1[n]) + rbf(s)));  // residual: h (raw, v1) + down
    if (l + 1 < a.L) {
      uint64_t* nslab = a.gran + (size_t)(l + 1) * G_SLAB;
      publish16(c, nslab + G_X, u * 16, xn);
      if (c.lane == 0) fstore(a.flags + (size_t)(l + 1) * F_SLAB + F_X + u, (int)c.tag);
    } else if (c.lane < 16) {
      a.x[n] = f2bf(xn);
    }
  }
  lds_barrier();
}

template <int ROLE>
TTS_DEV void role_body(const PersistArgs& a, char* smem, int b, uint32_t tag) {
  constexpr int NSL = ring_slots(ROLE), D = NSL - 1;
  PCtx c;
  c.a = &a;
  c.smem = smem;
  c.b = b;
  c.tid = threadIdx.x;
  c.lane = threadIdx.x & 63;
  c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.tag = tag;
  char* p = smem;
  c.ring = p; p += PW * NSL * 1024;
  c.v1 = (bf16_t*)p; p += L_V;
  c.v2 = (bf16_t*)p; p += L_V;
  c.red = (float*)p; p += L_RED;
  c.misc = (float*)p; p += L_MISC;
  c.act = nullptr;
  c.att = nullptr;
  if (ROLE == ROLE_A) { c.act = (bf16_t*)p; p += L_ACT; }
  if (ROLE == ROLE_C) { c.att = p; p += L_ATT; }

  const int o_unit = b - 128;
  Ring<ROLE, D> ring;
  ring.a = &a;
  ring.base = c.ring + c.wave * NSL * 1024;
  ring.lane = c.lane;
  ring.b = b;
  ring.w = c.wave;
  ring.prime();

  for (int l = 0; l < a.L; ++l) {
    stamp(a, b, l, 0);
    if (ROLE != ROLE_C) {
      phase_qkv(c, ring, l, ROLE == ROLE_A ? b + 64 : b - 128);
      stamp(a, b, l, 2);
    }
    if (ROLE == ROLE_C) {
      phase_attn(c, l, b - 192);
      stamp(a, b, l, 3);
      if (b - 192 < NKV) phase_merge(c, l, b - 192);
      stamp(a, b, l, 10);
    }
    if (ROLE != ROLE_A) {
      phase_o(c, ring, l, o_unit, ROLE == ROLE_B);
      stamp(a, b, l, 5);
    }
    phase_gu(c, ring, l);
    if (ROLE == ROLE_A) {
      phase_down(c, ring, l);
      stamp(a, b, l, 9);
    }
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
}

__global__ __launch_bounds__(PNT, 1) void persist_step_kernel(PersistArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  const uint32_t tag = (uint32_t)*a.seq;
#ifndef PERSIST_ONLY_ROLE
  if (b < 128) role_body<ROLE_A>(a, smem, b, tag);
  else if (b < 192) role_body<ROLE_B>(a, smem, b, tag);
  else role_body<ROLE_C>(a, smem, b, tag);
#else
  role_body<PERSIST_ONLY_ROLE>(a, smem, b, tag);
#endif
  // every workgroup read the tag before workgroup 0 can finish (its last down phase needs
  // every workgroup's last gate/up): the next step's tag
  if (b == 0 && threadIdx.x == 0) *a.seq = (int)(tag + 1);
}

}  // namespace

size_t persist_gran_elems(int L) { return (size_t)L * G_SLAB; }
size_t persist_flag_elems(int L) { return (size_t)L * F_SLAB; }

bool persist_supported(int hidden, int heads, int kv_heads, int head_dim, int ffn, int L, int max_seq, int nsplit,
                       int split, int num_cu, int* ur) {
  if (!(hidden == HID && heads == NH && kv_heads == NKV && head_dim == HDIM && ffn == FFN)) return false;
  if (num_cu != NWG || L < 1 || L > 32 || split != SPLIT || nsplit > NSMAX || max_seq > NSMAX * SPLIT) return false;
  // layouts: one round of units per matrix, the shapes the launch path streams at one row
  const StreamPlan pq = stream_plan(QKVN, HID, 1, num_cu), po = stream_plan(HID, HID, 1, num_cu);
  const StreamPlan pg = stream_plan(2 * FFN, HID, 2, num_cu), pd = stream_plan(HID, FFN, 1, num_cu);
  auto ok = [](const StreamPlan& p, int ks, int ku, int kc, int units) {
    return p.ksplit == ks && p.ku == ku && p.kc == kc && p.ur() >= units;
  };
  if (!ok(pq, 16, 2, 1, QKVN / 16) || !ok(po, 16, 2, 1, HID / 16) || !ok(pg, 4, 2, 1, FFN / 16) ||
      !ok(pd, 16, 4, 4, HID / 16))
    return false;
  ur[0] = pq.ur(); ur[1] = po.ur(); ur[2] = pg.ur(); ur[3] = pd.ur();
  return true;
}

void persist_init() {
  (void)hipFuncSetAttribute((const void*)persist_step_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

void launch_persist_step(const PersistArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(persist_step_kernel, dim3(NWG), dim3(PNT), 160 * 1024, s, a);
}

}  // namespace tts
