// codec_gemm.hip — the codec's fp32 contractions over operands already split into their bf16
// planes (x = h + m + l, h = bf16(x), m = bf16(x - h), l = bf16(x - h - m): the fp32 value):
// A by its producer (RMSNorm, GroupNorm + swish, attention, a GEMM epilogue write the planes
// instead of fp32), B (weights) once at load.  Six bf16 products per fp32 multiply-add in the
// order of gemm_bx3_kernel (codec_kernels.hip), so both kernels give the same bits.
//
// What changes against gemm_bx3_kernel: nothing is computed between the loads and the LDS
// image any more (the split moved to the producer, once per element instead of once per
// N tile), so the staging is LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave instruction,
// no VGPRs) into two LDS stages: stage s + 1 lands while stage s is multiplied, and a K step
// costs one counted vmcnt wait and two barriers, no VALU.
//
// LDS image of a stage: A planes [3][TM rows][32 k], then B planes [3][TN rows][32 k], bf16, a
// 64-B row each; the four 16-B chunks of row r sit at chunk index c ^ ((r >> 2) & 3), so the
// MFMA fragment reads (rows r .. r + 15 of one chunk per lane group) touch 16 distinct 4-bank
// groups: conflict-free with no padding.  One DMA instruction fills 16 rows: lane L reads
// 16 B of row (L >> 2) — four lanes per 64-B row segment of the plane in HBM / L2.
//
// The fragment reads are inline-asm ds_read_b128: the compiler treats any LDS read after an
// LDS-DMA as a possible alias of the DMA destination and would drain the next stage's DMA
// (s_waitcnt vmcnt(0)) before it.  The stage protocol orders them instead: a stage is read
// only after its own DMA was counted in (vmcnt) and every wave passed the barrier, and it is
// refilled only after every wave passed the barrier that ends its reads.
#include <algorithm>
#include <cstdio>
#include <stdexcept>

#include "codec_kernels.h"
#include "hip_common.h"

namespace tts {

typedef __attribute__((address_space(3))) char lds_char_t;

#ifdef TTS_STAMPS
// diagnostic build only: per-wave shader-clock sums of the K loop's phases, over every launch
// (x3p_stamps_dump: [0] wait + barrier, [1] kk0 fragments landing, [2] MFMA phase, [3] epilogue,
// [4] whole wave, [5] waves)
__device__ unsigned long long g_x3p_cyc[8];
#define X3P_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define X3P_T(v) do {} while (0)
#endif

// one 16-B LDS read (inline asm: invisible to the compiler's LDS-DMA alias waits)
TTS_DEV u32x4_t lds_rd16(uint32_t addr) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

template <int TM, int TN, int WM, int WN, bool ILV, int NS = 2, bool PP = false>
__global__ __launch_bounds__(64 * WM * WN) void gemm_x3p_kernel(GemmF32Args g) {
  constexpr int NW = WM * WN, NT = 64 * NW;
  constexpr int MI = TM / WM / 32, NJ = TN / WN / 32;  // 32x32 accumulators per wave
  constexpr int QA = 3 * TM / 16, QB = 3 * TN / 16;     // DMA instructions per stage (16 rows each)
  constexpr int QW = (QA + QB) / NW;                     // per wave (host-checked: divides)
  static_assert((QA + QB) % NW == 0, "DMA instructions per stage must divide over the waves");
  constexpr int APL = TM * 64, BPL = TN * 64;            // bytes of one plane's stage image
  constexpr int STAGE = 3 * (APL + BPL);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  X3P_T(t_entry);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave / WN, wn = wave % WN;
#ifdef TTS_STAMPS
  unsigned long long c_wait = 0, c_land = 0, c_mfma = 0;
#endif
  // XCD-aware tile order: consecutive blocks land on the 8 XCDs in turn, so tile id
  // (b % 8) * (tiles / 8) + b / 8 gives each XCD a contiguous run of tiles, i.e. the N tiles
  // of the same A rows share that XCD's L2
  const int nbn = (g.N + TN - 1) / TN, nbm = (g.M + TM - 1) / TM, ntiles = nbn * nbm;
  int tile = blockIdx.x;
  if (ntiles % 8 == 0) tile = (blockIdx.x % 8) * (ntiles / 8) + blockIdx.x / 8;
  const int m0 = (tile / nbn) * TM, n0 = (tile % nbn) * TN;
  const int nsteps = g.K / 32;

  // ---- per-lane DMA sources: row (lane >> 2) of each 16-row block, chunk (lane & 3) ^ swizzle
  // PP: only the upper half of the waves (one per SIMD) issue the DMA, twice the pieces each,
  // between their first MFMA tiles; the lower half starts its MFMAs right after the barrier, so
  // the two waves of a SIMD run out of phase and one of them is multiplying while the other
  // issues or lands fragments
  constexpr int QD = PP ? 2 * QW : QW;        // pieces per issuing wave
  constexpr int NL = PP ? NW / 2 : NW;        // issuing waves
  const bool loader = !PP || wave >= NW - NL;
  const int lw = PP ? wave - (NW - NL) : wave;
  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ ((lane >> 4) & 3);
  const uint16_t* srcp[QD];
  uint32_t dstoff[QD];
#pragma unroll
  for (int j = 0; j < QD; ++j) {
    const int q = min(max(lw, 0) + j * NL, QA + QB - 1);
    if (q < QA) {
      const int p = q / (TM / 16), rb = q % (TM / 16);
      const int r = min(m0 + rb * 16 + drow, g.M - 1);
      srcp[j] = g.Ap + p * g.ap_plane + (long long)r * g.lda + dchunk * 8;
      dstoff[j] = p * APL + rb * 1024;
    } else {
      const int qb = q - QA, p = qb / (TN / 16), rb = qb % (TN / 16);
      const int r = min(n0 + rb * 16 + drow, g.N - 1);
      srcp[j] = g.Bp + p * (long long)g.N * g.K + (long long)r * g.K + dchunk * 8;
      dstoff[j] = 3 * APL + p * BPL + rb * 1024;
    }
  }
  lds_char_t* lbase = (lds_char_t*)smem;
  auto issue1 = [&](int j, int s, int buf) {
    __builtin_amdgcn_global_load_lds((gptr_t)(srcp[j] + s * 32), (lptr_t)(lbase + buf * STAGE + dstoff[j]), 16, 0, 0);
  };
  auto issue = [&](int s, int buf) {
    if (loader) {
#pragma unroll
      for (int j = 0; j < QD; ++j) issue1(j, s, buf);
    }
  };

  // ---- per-lane fragment offsets (row r, k chunk c = 2 kk + (lane >> 5))
  const uint32_t l0 = (uint32_t)(size_t)lbase;
  uint32_t aoff[2][MI], boff[2][NJ];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int c = 2 * kk + (lane >> 5);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int r = wm * (TM / WM) + i * 32 + (lane & 31);
      aoff[kk][i] = r * 64 + ((c ^ ((r >> 2) & 3)) << 4);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int r = wn * (TN / WN) + j * 32 + (lane & 31);
      boff[kk][j] = 3 * APL + r * 64 + ((c ^ ((r >> 2) & 3)) << 4);
    }
  }

  f32x16_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto bf = [](const u32x4_t& x) { return __builtin_bit_cast(bf16x8_t, x); };
  // the 3 (MI + NJ) fragments of k-slice kk of the stage at LDS byte address sb
  auto read_frags = [&](uint32_t sb, int kk, u32x4_t (&a)[3][MI], u32x4_t (&b)[3][NJ]) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int p = 0; p < 3; ++p) a[p][i] = lds_rd16(sb + aoff[kk][i] + p * APL);
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int p = 0; p < 3; ++p) b[p][j] = lds_rd16(sb + boff[kk][j] + p * BPL);
  };
  // the reads' results are used only after this wait: each fragment passes through an (empty)
  // volatile asm after it, which the compiler keeps in order behind the wait
  auto land_frags = [&](u32x4_t (&a)[3][MI], u32x4_t (&b)[3][NJ]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int i = 0; i < MI; ++i) asm volatile("" : "+v"(a[p][i]));
#pragma unroll
      for (int j = 0; j < NJ; ++j) asm volatile("" : "+v"(b[p][j]));
    }
  };
  // between(t) runs after the six MFMAs of accumulator tile t (ILV: the next stage's DMA pieces)
  auto mfmas = [&](const u32x4_t (&a)[3][MI], const u32x4_t (&b)[3][NJ], auto&& between) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        f32x16_t c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(a[1][i]), bf(b[1][j]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(a[2][i]), bf(b[0][j]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(a[0][i]), bf(b[2][j]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(a[1][i]), bf(b[0][j]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(a[0][i]), bf(b[1][j]), c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(a[0][i]), bf(b[0][j]), c, 0, 0, 0);
        between(i * NJ + j);
      }
  };
  // one stage: k-slice 1's fragment reads are issued before k-slice 0's MFMAs (the scheduling
  // barrier keeps them there), so their LDS latency hides under those MFMAs.  ILV: the DMA
  // pieces of stage s + 1 (into the other buffer, free since every wave passed this step's
  // barrier) go out in the gaps after the first IT MFMA tiles — early, so they land before
  // the next step's wait, and beside MFMAs, so no phase of the step issues DMA alone
  constexpr int IT = MI * NJ < 3 ? MI * NJ : 3;  // tiles whose gaps carry the DMA pieces
  auto compute = [&](int buf, int snext, int nbuf) {
    const uint32_t sb = l0 + buf * STAGE;
    auto between = [&](int kk, int t) {
      if constexpr (ILV) {
        if (kk == 0 && t < IT) {
          if (snext >= 0 && loader) {
#pragma unroll
            for (int j = t * QD / IT; j < (t + 1) * QD / IT; ++j) issue1(j, snext, nbuf);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    u32x4_t a0[3][MI], b0[3][NJ], a1[3][MI], b1[3][NJ];
    X3P_T(t1);
    read_frags(sb, 0, a0, b0);
    land_frags(a0, b0);
    X3P_T(t2);
#ifdef TTS_STAMPS
    c_land += t2 - t1;
#endif
    read_frags(sb, 1, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mfmas(a0, b0, [&](int t) { between(0, t); });
    __builtin_amdgcn_sched_barrier(0);
    land_frags(a1, b1);
    mfmas(a1, b1, [&](int t) { between(1, t); });
#ifdef TTS_STAMPS
    X3P_T(t3);
    c_mfma += t3 - t2;
#endif
  };

  if constexpr (ILV) {
    // NS - 1 stages in flight: stage s + NS - 1 is issued while stage s is multiplied, into the
    // buffer stage s - 1 used (every wave left it: this step's barrier); one barrier per step
    static_assert(NS >= 2 && NS <= 4, "two to four stage buffers");
    constexpr int AHEAD = (NS - 2) * QD;  // pieces of the younger stages allowed in flight
#pragma unroll
    for (int q = 0; q < NS - 1; ++q)
      if (q < nsteps) issue(q, q);
    int buf = 0;
    for (int s = 0; s < nsteps; ++s) {
      X3P_T(t0);
      if (s + NS - 2 < nsteps) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(AHEAD) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_barrier" ::: "memory");
#ifdef TTS_STAMPS
      X3P_T(t0b);
      c_wait += t0b - t0;
#endif
      const int nbuf = buf == 0 ? NS - 1 : buf - 1;
      compute(buf, s + NS - 1 < nsteps ? s + NS - 1 : -1, nbuf);
      buf = buf == NS - 1 ? 0 : buf + 1;
    }
  } else {
    // ---- two stages in flight; stage s is read after its DMA was counted in and every wave
    // passed the barrier, refilled (stage s + 2) after the barrier that ends its reads
    issue(0, 0);
    if (nsteps > 1) issue(1, 1);
    for (int s = 0; s < nsteps; ++s) {
      if (s + 1 < nsteps) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_barrier" ::: "memory");
      compute(s & 1, -1, 0);
      asm volatile("s_barrier" ::: "memory");
      if (s + 2 < nsteps) issue(s + 2, s & 1);
    }
  }

  X3P_T(t_epi);
  const bool has_bias = g.bias != nullptr, has_resid = g.resid != nullptr;
  // ---- epilogue through LDS: each wave parks its WTM x WTN fp32 tile in LDS (the K loop's
  // stages are free once every wave passed the barrier) and reads it back as 16-B row pieces, so
  // a store instruction writes whole contiguous rows (1 KiB of C per wave instruction, 4 bf16 per
  // lane and plane) instead of one column element per lane in two rows (the accumulator layout:
  // 256 store instructions per wave and tile set; measured 17 % of the kernel, stamps build).
  // Same arithmetic per element: acc + bias, act, resid + v, split
  constexpr int WTM = TM / WM, WTN = TN / WN;
  static_assert(NW * WTM * WTN * 4 <= NS * STAGE, "the output tiles must fit the stage buffers");
  const bool vec = ((g.N | g.ldc) & 3) == 0 && (((size_t)g.C | (size_t)g.resid) & 15) == 0 &&
                   (((size_t)g.Cp | (size_t)(g.cp_plane * 2)) & 7) == 0;
  if (vec) {
    asm volatile("s_barrier" ::: "memory");  // (every wave's fragment reads completed: land_frags)
    float* tile = (float*)smem + wave * (WTM * WTN);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          tile[(i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * WTN + j * 32 + (lane & 31)] = acc[i][j][r];
    constexpr int LPR = WTN / 4, RPI = 64 / LPR, IT = WTM / RPI;  // lanes per row, rows per instruction
    const int cq = lane % LPR, rr = lane / LPR;
    const int n = n0 + wn * WTN + 4 * cq;
    const int nc = min(n, g.N - 4);
    float bias[4] = {0.f, 0.f, 0.f, 0.f};
    if (has_bias) {
#pragma unroll
      for (int q = 0; q < 4; ++q) bias[q] = g.bias[nc + q];
    }
    const int mb = m0 + wm * WTM + rr;
    float4 rv[IT];
    if (has_resid) {
#pragma unroll
      for (int it = 0; it < IT; ++it) rv[it] = *(const float4*)(g.resid + (size_t)min(mb + it * RPI, g.M - 1) * g.ldc + nc);
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int m = mb + it * RPI;
      const float4 a4 = *(const float4*)(tile + (rr + it * RPI) * WTN + 4 * cq);
      float v[4] = {a4.x, a4.y, a4.z, a4.w};
      const float rq[4] = {rv[it].x, rv[it].y, rv[it].z, rv[it].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[q] = v[q] + bias[q];
        if (g.act == 1) v[q] = v[q] / (1.0f + expf(-v[q]));
        if (has_resid) v[q] = rq[q] + v[q];
      }
      if (m < g.M && n < g.N) {
        const size_t o = (size_t)m * g.ldc + n;
        if (g.C) *(float4*)(g.C + o) = make_float4(v[0], v[1], v[2], v[3]);
        if (g.Cp) {  // the consumer GEMM's planes (the split every producer uses)
          uint32_t hw[2], mw[2], lw[2];
#pragma unroll
          for (int q = 0; q < 4; q += 2) {
            float x0 = v[q], x1 = v[q + 1];
            asm("" : "+v"(x0), "+v"(x1));  // (no contraction into v - h: see store_planes)
            const float h0 = rbf(x0), r0 = x0 - h0, m0v = rbf(r0);
            const float h1 = rbf(x1), r1 = x1 - h1, m1v = rbf(r1);
            hw[q >> 1] = (uint32_t)f2bf(h0) | ((uint32_t)f2bf(h1) << 16);
            mw[q >> 1] = (uint32_t)f2bf(m0v) | ((uint32_t)f2bf(m1v) << 16);
            lw[q >> 1] = (uint32_t)f2bf(r0 - m0v) | ((uint32_t)f2bf(r1 - m1v) << 16);
          }
          *(uint2*)(g.Cp + o) = make_uint2(hw[0], hw[1]);
          *(uint2*)(g.Cp + g.cp_plane + o) = make_uint2(mw[0], mw[1]);
          *(uint2*)(g.Cp + 2 * g.cp_plane + o) = make_uint2(lw[0], lw[1]);
        }
      }
    }
  } else {
  // ---- fallback (unaligned or odd widths): lane owns column (lane & 31); rows (r&3) +
  // 8(r>>2) + 4(lane>>5), as gemm_bx3_kernel; the residual values of an accumulator's 16 rows
  // are loaded together before any of them is used
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wn * (TN / WN) + j * 32 + (lane & 31);
      const int nc = min(n, g.N - 1);
      const float bias = has_bias ? g.bias[nc] : 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int mb = m0 + wm * (TM / WM) + i * 32 + 4 * (lane >> 5);
        float rv[16];
        if (has_resid) {
#pragma unroll
          for (int r = 0; r < 16; ++r) rv[r] = g.resid[(size_t)min(mb + (r & 3) + 8 * (r >> 2), g.M - 1) * g.ldc + nc];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mb + (r & 3) + 8 * (r >> 2);
          float v = acc[i][j][r] + bias;
          if (g.act == 1) v = v / (1.0f + expf(-v));
          if (has_resid) v = rv[r] + v;
          if (m < g.M && n < g.N) {
            const size_t o = (size_t)m * g.ldc + n;
            if (g.C) g.C[o] = v;
            if (g.Cp) {  // the consumer GEMM's planes (the split every producer uses)
              asm("" : "+v"(v));  // (no contraction into v - h: see store_planes)
              const float h = rbf(v), rm = v - h, mm = rbf(rm);
              g.Cp[o] = f2bf(h);
              g.Cp[g.cp_plane + o] = f2bf(mm);
              g.Cp[2 * g.cp_plane + o] = f2bf(rm - mm);
            }
          }
        }
      }
    }
  }
#ifdef TTS_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  X3P_T(t_end);
  if (lane == 0) {
    atomicAdd(&g_x3p_cyc[0], c_wait);
    atomicAdd(&g_x3p_cyc[1], c_land);
    atomicAdd(&g_x3p_cyc[2], c_mfma);
    atomicAdd(&g_x3p_cyc[3], t_end - t_epi);
    atomicAdd(&g_x3p_cyc[4], t_end - t_entry);
    atomicAdd(&g_x3p_cyc[5], 1ull);
  }
#endif
}

template <int TM, int TN, int WM, int WN, int NS = 2>
static void launch_x3p(const GemmF32Args& g, hipStream_t s) {
  constexpr size_t lds = NS * 3 * (size_t)(TM + TN) * 64;
  static_assert(lds <= 160 * 1024, "LDS");
  const int tiles = ((g.M + TM - 1) / TM) * ((g.N + TN - 1) / TN);
  // the one-stage-ahead schedule with the DMA between the MFMAs on the 8- and 4-wave 64x64-per-
  // wave tiles (a step is long enough to cover the DMA's latency); the two-stage schedule on
  // the small tiles, whose steps are not (one 650-code utterance 4.8 -> 5.3 ms with the first,
  // profiles/r5h_ab_codec_ilv.txt).  TTS_CODEC_X3P_ILV=0 / 1 forces one (A/B)
  static const int ilv_env = getenv("TTS_CODEC_X3P_ILV") ? atoi(getenv("TTS_CODEC_X3P_ILV")) : -1;
  const bool ilv = NS >= 3 || (ilv_env >= 0 ? ilv_env != 0 : (TM / WM == 64 && TN / WN == 64));
  // TTS_CODEC_X3P_PP=1: the out-of-phase DMA split (PP, above) on the 8-wave tile (experiment)
  static const bool pp = getenv("TTS_CODEC_X3P_PP") && atoi(getenv("TTS_CODEC_X3P_PP"));
  if (ilv && pp && NS == 2 && WM * WN == 8)
    hipLaunchKernelGGL((gemm_x3p_kernel<TM, TN, WM, WN, true, NS, WM * WN == 8>), dim3(tiles), dim3(64 * WM * WN), lds, s, g);
  else if (ilv) hipLaunchKernelGGL((gemm_x3p_kernel<TM, TN, WM, WN, true, NS>), dim3(tiles), dim3(64 * WM * WN), lds, s, g);
  else hipLaunchKernelGGL((gemm_x3p_kernel<TM, TN, WM, WN, false>), dim3(tiles), dim3(64 * WM * WN), lds, s, g);
}

static bool small4() {
  static const bool v = getenv("TTS_CODEC_X3P_SMALL4") && atoi(getenv("TTS_CODEC_X3P_SMALL4"));
  return v;
}

bool gemm_x3p_supported(const GemmF32Args& g) {
  // 32-deep K steps; 16-B aligned rows of both operands' planes (DMA pieces)
  return g.Ap && g.Bp && g.K % 32 == 0 && g.lda % 8 == 0 && ((size_t)g.Ap & 15) == 0 && g.M >= 1 && g.N >= 1;
}

void launch_gemm_x3p(const GemmF32Args& g, hipStream_t s) {
  if (!gemm_x3p_supported(g)) throw std::runtime_error("gemm_x3p: A and B planes, K % 32 == 0, 16-B aligned rows");
  // tiles: 256x128 (8 waves of 64x64, one workgroup per CU) where that makes >= 2 rounds of
  // the CUs (the ragged batch's big GEMMs); else 128x128, 128x64, 64x64 (4 waves) or 32x32 (one
  // wave) down to what fills the chip (every tile sweeps an output's K in the same order: the
  // same bits; a lone utterance's tile choices swept in profiles/r5w_ab_codec1_tile.txt, and
  // 64x64 from half a round, r5z2_ab_codec1_heur.txt, measured the same).  TTS_CODEC_X3P_TILE
  // forces one (0..5).
  static const int forced = getenv("TTS_CODEC_X3P_TILE") ? atoi(getenv("TTS_CODEC_X3P_TILE")) : -1;
  auto tiles = [&](int tm, int tn) { return ((g.M + tm - 1) / tm) * ((g.N + tn - 1) / tn); };
  int c = forced;
  if (c < 0)
    c = tiles(256, 128) >= 512 ? 0 : tiles(128, 128) >= 256 ? 1 : tiles(128, 64) >= 256 ? 2 : tiles(64, 64) >= 256 ? 3 : 4;
  switch (c) {
    case 0: launch_x3p<256, 128, 4, 2>(g, s); break;
    case 1: launch_x3p<128, 128, 2, 2>(g, s); break;
    case 2: launch_x3p<128, 64, 2, 2>(g, s); break;
    case 3: launch_x3p<64, 64, 2, 2>(g, s); break;
    case 5: launch_x3p<128, 128, 2, 4, 3>(g, s); break;  // (8 waves of 64x32, three stages: experiment)
    default:  // one wave: a lone utterance's small GEMMs (TTS_CODEC_X3P_SMALL4=1: four stages, the DMA
      // three steps ahead — experiment)
      if (small4()) launch_x3p<32, 32, 1, 1, 4>(g, s);
      else launch_x3p<32, 32, 1, 1>(g, s);
      break;
  }
}

void x3p_stamps_dump(FILE* f) {
#ifdef TTS_STAMPS
  unsigned long long h[8] = {};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_x3p_cyc), sizeof(h)) != hipSuccess) return;
  const double tot = (double)(h[4] ? h[4] : 1);
  fprintf(f, "x3p phases over %llu waves: wait+barrier %.3f  kk0 landing %.3f  MFMA phase %.3f  epilogue %.3f  "
             "(of %.0f cycles per wave)\n", h[5], h[0] / tot, h[1] / tot, h[2] / tot, h[3] / tot, tot / (h[5] ? h[5] : 1));
  const unsigned long long z[8] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_x3p_cyc), z, sizeof(z));
#else
  (void)f;
#endif
}

}  // namespace tts
