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
#include <stdexcept>

#include "codec_kernels.h"
#include "hip_common.h"

namespace tts {

typedef __attribute__((address_space(3))) char lds_char_t;

// one 16-B LDS read (inline asm: invisible to the compiler's LDS-DMA alias waits)
TTS_DEV u32x4_t lds_rd16(uint32_t addr) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

template <int TM, int TN, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void gemm_x3p_kernel(GemmF32Args g) {
  constexpr int NW = WM * WN, NT = 64 * NW;
  constexpr int MI = TM / WM / 32, NJ = TN / WN / 32;  // 32x32 accumulators per wave
  constexpr int QA = 3 * TM / 16, QB = 3 * TN / 16;     // DMA instructions per stage (16 rows each)
  constexpr int QW = (QA + QB) / NW;                     // per wave (host-checked: divides)
  static_assert((QA + QB) % NW == 0, "DMA instructions per stage must divide over the waves");
  constexpr int APL = TM * 64, BPL = TN * 64;            // bytes of one plane's stage image
  constexpr int STAGE = 3 * (APL + BPL);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware tile order: consecutive blocks land on the 8 XCDs in turn, so tile id
  // (b % 8) * (tiles / 8) + b / 8 gives each XCD a contiguous run of tiles, i.e. the N tiles
  // of the same A rows share that XCD's L2
  const int nbn = (g.N + TN - 1) / TN, nbm = (g.M + TM - 1) / TM, ntiles = nbn * nbm;
  int tile = blockIdx.x;
  if (ntiles % 8 == 0) tile = (blockIdx.x % 8) * (ntiles / 8) + blockIdx.x / 8;
  const int m0 = (tile / nbn) * TM, n0 = (tile % nbn) * TN;
  const int nsteps = g.K / 32;

  // ---- per-lane DMA sources: row (lane >> 2) of each 16-row block, chunk (lane & 3) ^ swizzle
  const int drow = lane >> 2;
  const int dchunk = (lane & 3) ^ ((lane >> 4) & 3);
  const uint16_t* srcp[QW];
  uint32_t dstoff[QW];
#pragma unroll
  for (int j = 0; j < QW; ++j) {
    const int q = wave + j * NW;
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
  auto issue = [&](int s, int buf) {
    const int k0 = s * 32;
#pragma unroll
    for (int j = 0; j < QW; ++j)
      __builtin_amdgcn_global_load_lds((gptr_t)(srcp[j] + k0), (lptr_t)(lbase + buf * STAGE + dstoff[j]), 16, 0, 0);
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
  auto mfmas = [&](const u32x4_t (&a)[3][MI], const u32x4_t (&b)[3][NJ]) {
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
      }
  };
  // one stage: k-slice 1's fragment reads are issued before k-slice 0's MFMAs (the scheduling
  // barrier keeps them there), so their LDS latency hides under those MFMAs
  auto compute = [&](int buf) {
    const uint32_t sb = l0 + buf * STAGE;
    u32x4_t a0[3][MI], b0[3][NJ], a1[3][MI], b1[3][NJ];
    read_frags(sb, 0, a0, b0);
    land_frags(a0, b0);
    read_frags(sb, 1, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mfmas(a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    land_frags(a1, b1);
    mfmas(a1, b1);
  };

  // ---- two stages in flight; stage s is read after its DMA was counted in and every wave
  // passed the barrier, refilled (stage s + 2) after the barrier that ends its reads
  issue(0, 0);
  if (nsteps > 1) issue(1, 1);
  for (int s = 0; s < nsteps; ++s) {
    if (s + 1 < nsteps) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    compute(s & 1);
    asm volatile("s_barrier" ::: "memory");
    if (s + 2 < nsteps) issue(s + 2, s & 1);
  }

  // ---- epilogue (as gemm_bx3_kernel): lane owns column (lane & 31); rows (r&3) + 8(r>>2) +
  // 4(lane>>5).  The residual values of an accumulator's 16 rows are loaded together
  // (clamped rows, unconditional) before any of them is used: one L2 round trip, not 16
  const bool has_bias = g.bias != nullptr, has_resid = g.resid != nullptr;
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

template <int TM, int TN, int WM, int WN>
static void launch_x3p(const GemmF32Args& g, hipStream_t s) {
  constexpr size_t lds = 2 * 3 * (size_t)(TM + TN) * 64;
  const int tiles = ((g.M + TM - 1) / TM) * ((g.N + TN - 1) / TN);
  hipLaunchKernelGGL((gemm_x3p_kernel<TM, TN, WM, WN>), dim3(tiles), dim3(64 * WM * WN), lds, s, g);
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
  // same bits).  TTS_CODEC_X3P_TILE forces one (0..4) for experiments.
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
    default: launch_x3p<32, 32, 1, 1>(g, s); break;  // one wave: a lone utterance's small GEMMs
  }
}

}  // namespace tts
