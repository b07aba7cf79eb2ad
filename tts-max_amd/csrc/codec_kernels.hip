// codec_kernels.hip — fp32 kernels of the xcodec2-compatible codec decoder.
//
// Reference: tts/core/codec/decoder.py:69-89 (Decoder.forward) and decoder_modules.py
// (ISTFT 19-93, ISTFTHead 96-148, ResnetBlock 162-223, RMSNorm 226-236, MLP 239-251,
// Attention 254-290, TransformerBlock 293-314, VocosBackbone 317-400), upsampler.py 9-69.
// The reference runs the codec in fp32; so does this path: every contraction is a
// v_mfma_f32_32x32x2_f32 GEMM (exact fp32 products, fp32 accumulation).
//
// MI355X layout: activations are time-major [T][C] (row = one frame, channels contiguous),
// so a Conv1d(k) over a zero-padded buffer is a plain GEMM whose A operand is a sliding
// window: row t starts at x + (t - k/2)*C and spans k*C contiguous floats (lda = C < K).
// No im2col buffer is ever written.
#include <algorithm>
#include <stdexcept>

#include "codec_kernels.h"
#include "hip_common.h"

namespace tts {

// one fp32 value as its three bf16 planes (element o of plane p at q + p * plane + o): the
// split gemm_bx3_kernel applies while staging, written by the producer for gemm_x3p
TTS_DEV void store_planes(uint16_t* __restrict__ q, long long plane, size_t o, float v) {
  // (v as the fp32 value a store would hold: the compiler must not contract the product that
  // made v into v - h, or the planes would split a value the fp32 path never sees)
  asm("" : "+v"(v));
  const float h = rbf(v), r = v - h, m = rbf(r);
  q[o] = f2bf(h);
  q[plane + o] = f2bf(m);
  q[2 * plane + o] = f2bf(r - m);
}


// ------------------------------------------------------------------ fp32 MFMA GEMM ----
// Tile TM x TN x 16, four waves in a 2x2 grid, each wave (TM/2) x (TN/2) built from
// 32x32 v_mfma_f32_32x32x2_f32 tiles.  Operands are staged k-major in LDS (row stride
// TM+2 floats: the transposed stores of one wave-instruction hit 32 distinct banks) so an
// MFMA operand read is 32 consecutive floats.  The next K tile is loaded into registers
// while the current one is consumed.  64x64 tiles are used when 128x128 would leave CUs
// idle (the codec's T ~ 500-2000 rows).
template <int TM, int TN, int GBK>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmF32Args g) {
  constexpr int LSA = TM + 2, LSB = TN + 2;
  constexpr int AV = TM * GBK / 256 / 4;  // float4 per thread for the A tile (1 or 2)
  constexpr int BV = TN * GBK / 256 / 4;
  constexpr int MI = TM / 64, NJ = TN / 64;  // 32x32 MFMA tiles per wave
  __shared__ float As[GBK * LSA];
  __shared__ float Bs[GBK * LSB];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nbn = (g.N + TN - 1) / TN;
  const int m0 = (blockIdx.x / nbn) * TM, n0 = (blockIdx.x % nbn) * TN;
  const int kbeg = blockIdx.y * g.kchunk;  // split-K range (kchunk = K when not split)
  const int kend = min(g.K, kbeg + g.kchunk);
  // staging map: thread -> (row, 4*AV consecutive k)
  const int arow = t / (GBK / (4 * AV)), ak = (t % (GBK / (4 * AV))) * 4 * AV;
  const int brow = t / (GBK / (4 * BV)), bk = (t % (GBK / (4 * BV))) * 4 * BV;
  const int ar = m0 + arow, br = n0 + brow;
  const bool aok = ar < g.M, bok = br < g.N;
  // out-of-range rows read a clamped (valid) row and are zeroed after the load: a load
  // inside a branch makes hipcc wait on it before the next one is issued
  const float* ap = g.A + (size_t)(aok ? ar : g.M - 1) * g.lda + kbeg + ak;
  const float* bp = g.B + (size_t)(bok ? br : g.N - 1) * g.K + kbeg + bk;
  f32x16_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 ra[AV], rb[BV];
#pragma unroll
  for (int v = 0; v < AV; ++v) {
    const float4 l = *(const float4*)(ap + 4 * v);
    ra[v] = aok ? l : z4;
  }
#pragma unroll
  for (int v = 0; v < BV; ++v) {
    const float4 l = *(const float4*)(bp + 4 * v);
    rb[v] = bok ? l : z4;
  }
  for (int k0 = kbeg; k0 < kend; k0 += GBK) {
    __syncthreads();
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      As[(ak + 4 * v + 0) * LSA + arow] = ra[v].x;
      As[(ak + 4 * v + 1) * LSA + arow] = ra[v].y;
      As[(ak + 4 * v + 2) * LSA + arow] = ra[v].z;
      As[(ak + 4 * v + 3) * LSA + arow] = ra[v].w;
    }
#pragma unroll
    for (int v = 0; v < BV; ++v) {
      Bs[(bk + 4 * v + 0) * LSB + brow] = rb[v].x;
      Bs[(bk + 4 * v + 1) * LSB + brow] = rb[v].y;
      Bs[(bk + 4 * v + 2) * LSB + brow] = rb[v].z;
      Bs[(bk + 4 * v + 3) * LSB + brow] = rb[v].w;
    }
    __syncthreads();
    if (k0 + GBK < kend) {  // prefetch next K tile while the MFMAs run
      const int kn = k0 + GBK - kbeg;
#pragma unroll
      for (int v = 0; v < AV; ++v) {
        const float4 l = *(const float4*)(ap + kn + 4 * v);
        ra[v] = aok ? l : z4;
      }
#pragma unroll
      for (int v = 0; v < BV; ++v) {
        const float4 l = *(const float4*)(bp + kn + 4 * v);
        rb[v] = bok ? l : z4;
      }
    }
#pragma unroll
    for (int kk = 0; kk < GBK / 2; ++kk) {
      const int kr = 2 * kk + (lane >> 5);
      float a[MI], b[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = As[kr * LSA + wm * (TM / 2) + i * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < NJ; ++j) b[j] = Bs[kr * LSB + wn * (TN / 2) + j * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  // epilogue: lane owns column (lane & 31); rows (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = n0 + wn * (TN / 2) + j * 32 + (lane & 31);
    if (n >= g.N) continue;
    const float bias = g.bias ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * (TM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= g.M) continue;
        if (g.ksplit > 1) {  // raw partial; bias / act / residual in the reduce
          g.part[((size_t)blockIdx.y * g.M + m) * g.N + n] = acc[i][j][r];
          continue;
        }
        float v = acc[i][j][r] + bias;
        if (g.act == 1) v = v / (1.0f + expf(-v));
        if (g.resid) v = g.resid[(size_t)m * g.ldc + n] + v;
        if (g.C) g.C[(size_t)m * g.ldc + n] = v;
        if (g.Cp) store_planes(g.Cp, g.cp_plane, (size_t)m * g.ldc + n, v);
      }
  }
}

__global__ void gemm_f32_reduce_kernel(const float* __restrict__ part, int S, int M, int N,
                                       const float* __restrict__ bias, int act, const float* resid,
                                       float* C, int ldc) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)M * N) return;
  const int m = (int)(i / N), n = (int)(i % N);
  float v = 0.f;
  for (int s = 0; s < S; ++s) v += part[((size_t)s * M + m) * N + n];
  if (bias) v += bias[n];
  if (act == 1) v = v / (1.0f + expf(-v));
  if (resid) v = resid[(size_t)m * ldc + n] + v;
  C[(size_t)m * ldc + n] = v;
}

// K step per barrier pair: 64 (64x64 tiles) / 32 (128x128) where K allows — enough MFMA
// work per step to cover the next step's L2 latency; 16 otherwise
template <int TM, int TN>
static void launch_tile(const GemmF32Args& g, dim3 grid, hipStream_t s) {
  constexpr int BIG = TM == 128 ? 32 : 64;
  if (g.kchunk % BIG == 0 && g.K % BIG == 0)
    hipLaunchKernelGGL((gemm_f32_kernel<TM, TN, BIG>), grid, dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<TM, TN, 16>), grid, dim3(256), 0, s, g);
}

// Tiles: 128x128 (4 waves x 2x2 MFMA accumulators, K step 32) when that grid fills the
// chip, else 64x64 split over K up to ~768 workgroups (measured best at T = 650: 128x128
// tiles split to the same count were 25 % slower).
template <int TM, int TN>
static void launch_split(GemmF32Args g, int target, hipStream_t s) {
  const int grid = ((g.M + TM - 1) / TM) * ((g.N + TN - 1) / TN);
  int S = 1;
  if (g.part != nullptr && grid < target * 3 / 4 && g.K >= 512) {
    S = std::min(16, std::max(1, (target + grid - 1) / grid));
    S = std::min(S, g.K / 256);
    while (S > 1 && (size_t)S * g.M * g.N > g.part_elems) --S;
  }
  if (S <= 1) {
    g.ksplit = 1; g.kchunk = g.K;
    launch_tile<TM, TN>(g, dim3(grid), s);
    return;
  }
  const int step = (g.K % 64 == 0) ? 64 : 16;
  g.kchunk = ((g.K + S - 1) / S + step - 1) / step * step;
  S = (g.K + g.kchunk - 1) / g.kchunk;
  g.ksplit = S;
  launch_tile<TM, TN>(g, dim3(grid, S), s);
  const long long n = (long long)g.M * g.N;
  hipLaunchKernelGGL(gemm_f32_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g.part, S,
                     g.M, g.N, g.bias, g.act, g.resid, g.C, g.ldc);
}

// ------------------------------------------------- fp32 GEMM as three bf16 MFMA products -----
// The codec is fp32 end to end (the reference never casts).  fp32 MFMA (32x32x2) peaks at a
// sixteenth of the bf16 rate on CDNA4, so every fp32 operand is split once, in the LDS staging,
// into x = h + m + l with h = bf16(x), m = bf16(x - h), l = bf16(x - h - m) (24 significant
// bits: the fp32 value), and a.b = ah.bh + (ah.bm + am.bh) + (ah.bl + al.bh + am.bm) with fp32
// accumulation (v_mfma_f32_32x32x16_bf16, smallest terms first); the dropped terms are
// <= 2^-24 relative, i.e. fp32 products.  Same tiles, staging order and epilogue as
// gemm_f32_kernel.
// Tile TM x TN over WM x WN waves, each wave (TM/WM) x (TN/WN) = MI x NJ accumulators of 32x32.
// 64x64 and 128x128: 2 x 2 waves (256 threads); 256x128 / 256x256: 4 x 2 / 4 x 4 waves, each
// 64x64 — half (a quarter) the operand bytes per MAC of the 128x128 tile, one workgroup per CU.
template <int TM, int TN, int WM, int WN, bool BPRE, bool APRE = false>
__global__ __launch_bounds__(64 * WM * WN) void gemm_bx3_kernel(GemmF32Args g) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BK = 32, LS = BK + 8;           // bf16 row stride 80 B
  constexpr int MI = TM / WM / 32, NJ = TN / WN / 32;  // 32x32 accumulators per wave
  constexpr int TPA = NT / TM, KPA = BK / TPA; // A staging: threads per row, floats per thread
  constexpr int TPB = NT / TN, KPB = BK / TPB;
  static_assert(KPA >= 8 && KPA % 8 == 0 && KPB >= 8 && KPB % 8 == 0, "staging: whole 8-element chunks per thread");
  __shared__ __attribute__((aligned(16))) bf16_t Ah[TM * LS], Am[TM * LS], Al[TM * LS];
  __shared__ __attribute__((aligned(16))) bf16_t Bh[TN * LS], Bm[TN * LS], Bl[TN * LS];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int nbn = (g.N + TN - 1) / TN;
  const int m0 = (blockIdx.x / nbn) * TM, n0 = (blockIdx.x % nbn) * TN;
  const int kbeg = blockIdx.y * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const int arow = t / TPA, ak = (t % TPA) * KPA;
  const int brow = t / TPB, bk = (t % TPB) * KPB;
  const int ar = m0 + arow, br = n0 + brow;
  const bool aok = ar < g.M, bok = br < g.N;
  const float* ap = g.A + (size_t)(aok ? ar : g.M - 1) * g.lda + kbeg + ak;
  // APRE: A already split into its planes (one pass per GEMM input, shared by every N tile)
  const bf16_t* aq = APRE ? (const bf16_t*)g.Ap + (size_t)(aok ? ar : g.M - 1) * g.lda + kbeg + ak : nullptr;
  const float* bp = g.B + (size_t)(bok ? br : g.N - 1) * g.K + kbeg + bk;
  // BPRE: B already split into its h / m / l planes (weights, split once at load)
  const bf16_t* bq = BPRE ? (const bf16_t*)g.Bp + (size_t)(bok ? br : g.N - 1) * g.K + kbeg + bk : nullptr;
  const size_t bplane = (size_t)g.N * g.K;
  const u32x4_t zq = {0u, 0u, 0u, 0u};
  f32x16_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  // two register sets: the global loads of step s+2 are in flight while step s computes
  // (unconditional, step index clamped: exact vmcnt waits)
  const int nsteps = (kend - kbeg) / BK;
  constexpr int RB = BPRE ? 1 : KPB / 4, RQ = BPRE ? KPB / 8 : 1;
  constexpr int RA = APRE ? 1 : KPA / 4, RAQ = APRE ? KPA / 8 : 1;
  float4 ra[2][RA], rb[2][RB];
  u32x4_t rq[2][3][RQ], raq[2][3][RAQ];
  auto load = [&](int st, float4 (&xa)[RA], float4 (&xb)[RB], u32x4_t (&xq)[3][RQ], u32x4_t (&xaq)[3][RAQ]) {
    const int kn = min(st, nsteps - 1) * BK;
    if constexpr (APRE) {
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
#pragma unroll
        for (int v = 0; v < RAQ; ++v) {
          const u32x4_t l = *(const u32x4_t*)(aq + pl * g.ap_plane + kn + 8 * v);
          xaq[pl][v] = aok ? l : zq;
        }
    } else {
#pragma unroll
      for (int v = 0; v < KPA / 4; ++v) {
        const float4 l = *(const float4*)(ap + kn + 4 * v);
        xa[v] = aok ? l : z4;
      }
    }
    if constexpr (BPRE) {
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
#pragma unroll
        for (int v = 0; v < RQ; ++v) {
          const u32x4_t l = *(const u32x4_t*)(bq + pl * bplane + kn + 8 * v);
          xq[pl][v] = bok ? l : zq;
        }
    } else {
#pragma unroll
      for (int v = 0; v < RB; ++v) {
        const float4 l = *(const float4*)(bp + kn + 4 * v);
        xb[v] = bok ? l : z4;
      }
    }
  };
  // 8 fp32 -> 8 bf16 each of h, m, l (exact residuals: x - h and x - h - m are fp32-exact),
  // one 16-B store per plane
  auto split8 = [](const float4& x0, const float4& x1, bf16_t* hp, bf16_t* mp, bf16_t* lp) {
    const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    u32x4_t h, m, l;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float h0 = rbf(v[2 * q]), h1 = rbf(v[2 * q + 1]);
      const float r0 = v[2 * q] - h0, r1 = v[2 * q + 1] - h1;
      const float m0 = rbf(r0), m1 = rbf(r1);
      h[q] = pack_bf2(h0, h1);
      m[q] = pack_bf2(m0, m1);
      l[q] = pack_bf2(r0 - m0, r1 - m1);
    }
    *(u32x4_t*)hp = h;
    *(u32x4_t*)mp = m;
    *(u32x4_t*)lp = l;
  };
  auto stage = [&](const float4 (&xa)[RA], const float4 (&xb)[RB], const u32x4_t (&xq)[3][RQ],
                   const u32x4_t (&xaq)[3][RAQ]) {
    if constexpr (APRE) {
#pragma unroll
      for (int v = 0; v < RAQ; ++v) {
        *(u32x4_t*)(Ah + arow * LS + ak + 8 * v) = xaq[0][v];
        *(u32x4_t*)(Am + arow * LS + ak + 8 * v) = xaq[1][v];
        *(u32x4_t*)(Al + arow * LS + ak + 8 * v) = xaq[2][v];
      }
    } else {
#pragma unroll
      for (int v = 0; v < KPA / 8; ++v)
        split8(xa[2 * v], xa[2 * v + 1], Ah + arow * LS + ak + 8 * v, Am + arow * LS + ak + 8 * v,
               Al + arow * LS + ak + 8 * v);
    }
    if constexpr (BPRE) {
#pragma unroll
      for (int v = 0; v < RQ; ++v) {
        *(u32x4_t*)(Bh + brow * LS + bk + 8 * v) = xq[0][v];
        *(u32x4_t*)(Bm + brow * LS + bk + 8 * v) = xq[1][v];
        *(u32x4_t*)(Bl + brow * LS + bk + 8 * v) = xq[2][v];
      }
    } else {
#pragma unroll
      for (int v = 0; v < KPB / 8; ++v)
        split8(xb[2 * v], xb[2 * v + 1], Bh + brow * LS + bk + 8 * v, Bm + brow * LS + bk + 8 * v,
               Bl + brow * LS + bk + 8 * v);
    }
  };
  auto compute = [&]() {
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const int ko = kk * 16 + 8 * (lane >> 5);
      bf16x8_t ah[MI], am[MI], al[MI], bh[NJ], bm[NJ], bl[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int r = wm * (TM / WM) + i * 32 + (lane & 31);
        ah[i] = *(const bf16x8_t*)(Ah + r * LS + ko);
        am[i] = *(const bf16x8_t*)(Am + r * LS + ko);
        al[i] = *(const bf16x8_t*)(Al + r * LS + ko);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = wn * (TN / WN) + j * 32 + (lane & 31);
        bh[j] = *(const bf16x8_t*)(Bh + r * LS + ko);
        bm[j] = *(const bf16x8_t*)(Bm + r * LS + ko);
        bl[j] = *(const bf16x8_t*)(Bl + r * LS + ko);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          f32x16_t c = acc[i][j];
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bm[j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bh[j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bm[j], c, 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], c, 0, 0, 0);
        }
    }
  };
  load(0, ra[0], rb[0], rq[0], raq[0]);
  load(1, ra[1], rb[1], rq[1], raq[1]);
  for (int st = 0; st < nsteps; st += 2) {
    __syncthreads();
    stage(ra[0], rb[0], rq[0], raq[0]);
    __syncthreads();
    load(st + 2, ra[0], rb[0], rq[0], raq[0]);
    compute();
    __syncthreads();
    stage(ra[1], rb[1], rq[1], raq[1]);  // (an odd last step stages a clamped duplicate, not computed)
    __syncthreads();
    load(st + 3, ra[1], rb[1], rq[1], raq[1]);
    if (st + 1 < nsteps) compute();
  }
  // epilogue (as gemm_f32_kernel): lane owns column (lane & 31); rows (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = n0 + wn * (TN / WN) + j * 32 + (lane & 31);
    if (n >= g.N) continue;
    const float bias = g.bias ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * (TM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= g.M) continue;
        if (g.ksplit > 1) {
          g.part[((size_t)blockIdx.y * g.M + m) * g.N + n] = acc[i][j][r];
          continue;
        }
        float v = acc[i][j][r] + bias;
        if (g.act == 1) v = v / (1.0f + expf(-v));
        if (g.resid) v = g.resid[(size_t)m * g.ldc + n] + v;
        if (g.C) g.C[(size_t)m * g.ldc + n] = v;
        if (g.Cp) store_planes(g.Cp, g.cp_plane, (size_t)m * g.ldc + n, v);
      }
  }
}

// The codec never splits K over workgroups: every output element is one in-order sweep of K
// whatever the tile shape, so a row's bits do not depend on how many rows share the launch
// (an utterance decodes to the same samples alone or in any batch).  A ragged batch gives
// the GEMMs their rows; a lone short utterance leaves CUs idle instead.
void launch_gemm_f32(const GemmF32Args& g_in, hipStream_t s) {
  GemmF32Args g = g_in;
  g.part = nullptr;
  g.ksplit = 1;
  g.kchunk = g.K;
  // TTS_CODEC_BX3=0: plain fp32 MFMA for every contraction
  static const bool bx3 = !(getenv("TTS_CODEC_BX3") && !atoi(getenv("TTS_CODEC_BX3")));
  const int big = ((g.M + 127) / 128) * ((g.N + 127) / 128);
  if (bx3 && g.K % 32 == 0 && g.lda % 4 == 0) {
    const dim3 g128(big), g64(((g.M + 63) / 64) * ((g.N + 63) / 64));
    // TTS_CODEC_TILE: 0 = 128x128; 1 (default) = 256x128, 2 = 128x256 (8 waves of 64x64, one
    // workgroup per CU: fewer operand bytes per MAC, and with 256 columns each A element is
    // split for twice the outputs) where those tiles still make >= 2 rounds of the CUs (the
    // ragged batch's big GEMMs).  (256x256 on 16 waves spills: 4 waves per SIMD leave 128 VGPRs)
    static const int big_tiles = getenv("TTS_CODEC_TILE") ? atoi(getenv("TTS_CODEC_TILE")) : 1;
    const int t21 = ((g.M + 255) / 256) * ((g.N + 127) / 128);
    const int t12 = ((g.M + 127) / 128) * ((g.N + 255) / 256);
    if (g.Bp && g.Ap && big_tiles == 1 && t21 >= 2 * 256)
      hipLaunchKernelGGL((gemm_bx3_kernel<256, 128, 4, 2, true, true>), dim3(t21), dim3(512), 0, s, g);
    else if (g.Bp && g.Ap && big >= 256)
      hipLaunchKernelGGL((gemm_bx3_kernel<128, 128, 2, 2, true, true>), g128, dim3(256), 0, s, g);
    else if (g.Bp && big_tiles == 1 && t21 >= 2 * 256)
      hipLaunchKernelGGL((gemm_bx3_kernel<256, 128, 4, 2, true>), dim3(t21), dim3(512), 0, s, g);
    else if (g.Bp && big_tiles == 2 && t12 >= 2 * 256)
      hipLaunchKernelGGL((gemm_bx3_kernel<128, 256, 2, 4, true>), dim3(t12), dim3(512), 0, s, g);
    else if (g.Bp && big >= 256) hipLaunchKernelGGL((gemm_bx3_kernel<128, 128, 2, 2, true>), g128, dim3(256), 0, s, g);
    else if (g.Bp) hipLaunchKernelGGL((gemm_bx3_kernel<64, 64, 2, 2, true>), g64, dim3(256), 0, s, g);
    else if (big >= 256) hipLaunchKernelGGL((gemm_bx3_kernel<128, 128, 2, 2, false>), g128, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((gemm_bx3_kernel<64, 64, 2, 2, false>), g64, dim3(256), 0, s, g);
    return;
  }
  if (big >= 256) launch_split<128, 128>(g, 0, s);
  else launch_split<64, 64>(g, 0, s);
}

// B operand split once (weights at load): planes [3][n] = h, m, l with the kernel's rounding
__global__ void split_planes_kernel(const float* __restrict__ x, bf16_t* __restrict__ p, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float v = x[i], h = rbf(v), r = v - h, m = rbf(r);
    p[i] = f2bf(h);
    p[n + i] = f2bf(m);
    p[2 * n + i] = f2bf(r - m);
  }
}

void launch_split_planes(const float* x, uint16_t* planes, long long n, hipStream_t s) {
  const int grid = (int)std::min<long long>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(split_planes_kernel, dim3(grid), dim3(256), 0, s, x, planes, n);
}

// ------------------------------------------------------------------ small kernels -----
// ResidualFSQ(levels=[4]*8, num_quantizers=1).get_output_from_indices
// (vector_quantize_pytorch 1.17.8): digit_j = (i // 4^j) % 4, code_j = (digit_j - 2) / 2,
// scale 1 for quantizer 0, then project_out Linear(8 -> vq_dim).
__global__ void fsq_project_kernel(const int* __restrict__ codes, const int* __restrict__ code_row,
                                   const float* __restrict__ w, const float* __restrict__ b,
                                   float* __restrict__ out, int vq) {
  const int i = blockIdx.x;
  const int c = codes[i];
  const size_t t = (size_t)code_row[i];
  float z[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (float)(((c >> (2 * j)) & 3) - 2) * 0.5f;
  for (int o = threadIdx.x; o < vq; o += blockDim.x) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += z[j] * w[o * 8 + j];
    out[(size_t)t * vq + o] = acc + b[o];
  }
}

void launch_fsq_project(const int* codes, const int* code_row, int n, const float* w, const float* b,
                        float* out, int vq_dim, hipStream_t s) {
  hipLaunchKernelGGL(fsq_project_kernel, dim3(n), dim3(256), 0, s, codes, code_row, w, b, out, vq_dim);
}

// The zero rows around the utterances of a ragged buffer (the padding a Conv1d window
// reads): kPad rows before the first and after every utterance.
__global__ void zero_gaps_kernel(float* __restrict__ x, int C, const CodecSeg* __restrict__ seg,
                                 uint16_t* __restrict__ xp, long long plane) {
  const int g = blockIdx.x;
  const size_t r0 = g == 0 ? 0 : (size_t)(seg[g - 1].row + seg[g - 1].T);
  for (int i = threadIdx.x; i < kCodecPad * C; i += blockDim.x) {
    if (xp) {  // (the buffer's planes: all three are +0)
      xp[r0 * C + i] = 0;
      xp[plane + r0 * C + i] = 0;
      xp[2 * plane + r0 * C + i] = 0;
    } else {
      x[r0 * C + i] = 0.f;
    }
  }
}

void launch_zero_gaps(float* x, int C, const CodecSeg* seg, int B, hipStream_t s, uint16_t* xp, long long plane) {
  hipLaunchKernelGGL(zero_gaps_kernel, dim3(B + 1), dim3(256), 0, s, x, C, seg, xp, plane);
}

// GroupNorm statistics (torch.nn.GroupNorm, biased variance), two passes in fp32.
__global__ void groupnorm_stats_kernel(const float* __restrict__ x_all, const CodecSeg* __restrict__ seg,
                                       int C, int cg, float eps, float* __restrict__ stats_all) {
  __shared__ float red[16];
  const int grp = blockIdx.x;
  // one utterance per grid row: its own statistics over its own frames
  const int T = seg[blockIdx.y].T;
  const float* x = x_all + (size_t)seg[blockIdx.y].row * C;
  float* stats = stats_all + (size_t)blockIdx.y * gridDim.x * 2;
  const long long n = (long long)T * cg;
  // thread -> (column c of the group, rows t0, t0 + rs, ...): no per-element integer
  // division, independent loads (the launcher guarantees blockDim % cg == 0)
  const int c = threadIdx.x % cg, t0 = threadIdx.x / cg, rs = blockDim.x / cg;
  const float* xc = x + grp * cg + c;
  float sum = 0.f;
#pragma unroll 4
  for (int t = t0; t < T; t += rs) sum += xc[(size_t)t * C];
  const float mean = block_sum(sum, red) / (float)n;
  float sq = 0.f;
#pragma unroll 4
  for (int t = t0; t < T; t += rs) {
    const float d = xc[(size_t)t * C] - mean;
    sq += d * d;
  }
  const float var = block_sum(sq, red) / (float)n;
  if (threadIdx.x == 0) {
    stats[2 * grp] = mean;
    stats[2 * grp + 1] = 1.0f / sqrtf(var + eps);
  }
}

void launch_groupnorm_stats(const float* x, const CodecSeg* seg, int B, int C, int groups, float eps,
                            float* stats, hipStream_t s) {
  const int cg = C / groups;
  if (cg > 1024 || 1024 % cg != 0) throw std::runtime_error("groupnorm: channels per group must divide 1024");
  hipLaunchKernelGGL(groupnorm_stats_kernel, dim3(groups, B), dim3(1024), 0, s, x, seg, C, cg, eps, stats);
}

// y = swish(GN(x)) over each utterance's frames (grid row = utterance); the kPad rows
// after each utterance (and before the first) are written as zeros: y is a Conv1d input
__global__ void groupnorm_swish_kernel(const float* __restrict__ x_all, const CodecSeg* __restrict__ seg,
                                       int C, int cg, int groups, const float* __restrict__ stats_all,
                                       const float* __restrict__ gamma,
                                       const float* __restrict__ beta, float* __restrict__ y_all,
                                       uint16_t* __restrict__ yp, long long plane) {
  const int b = blockIdx.y;
  const size_t row = (size_t)seg[b].row;
  const long long n = (long long)seg[b].T * C;
  const float* x = x_all + row * C;
  const float* stats = stats_all + (size_t)b * groups * 2;
  // (yp: the conv GEMM's planes instead of fp32 y; same element offsets)
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C), grp = c / cg;
    const float v = (x[i] - stats[2 * grp]) * stats[2 * grp + 1] * gamma[c] + beta[c];
    const float o = v / (1.0f + expf(-v));
    if (yp) store_planes(yp, plane, row * C + i, o);
    else y_all[row * C + i] = o;
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (long long)kCodecPad * C;
       i += (long long)gridDim.x * blockDim.x) {
    if (yp) {
      store_planes(yp, plane, row * C + n + i, 0.f);
      if (b == 0) store_planes(yp, plane, i, 0.f);
    } else {
      y_all[row * C + n + i] = 0.f;
      if (b == 0) y_all[i] = 0.f;
    }
  }
}

void launch_groupnorm_swish(const float* x, const CodecSeg* seg, int B, int max_T, int C, int groups,
                            const float* stats, const float* gamma, const float* beta, float* y, hipStream_t s,
                            uint16_t* yp, long long plane) {
  const long long n = (long long)max_T * C;
  int grid = (int)std::min<long long>((n + 255) / 256, std::max(1, 8192 / B));
  hipLaunchKernelGGL(groupnorm_swish_kernel, dim3(grid, B), dim3(256), 0, s, x, seg, C, C / groups, groups,
                     stats, gamma, beta, y, yp, plane);
}

__global__ void rmsnorm_f32_kernel(const float* __restrict__ x, int C, const float* __restrict__ w,
                                   float eps, float* __restrict__ y, uint16_t* __restrict__ yp, long long plane) {
  __shared__ float red[16];
  const float* xr = x + (size_t)blockIdx.x * C;
  float ss = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) ss += xr[c] * xr[c];
  const float r = 1.0f / sqrtf(block_sum(ss, red) / (float)C + eps);
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float v = xr[c] * r * w[c];
    if (yp) store_planes(yp, plane, (size_t)blockIdx.x * C + c, v);  // (the GEMM's planes)
    else y[(size_t)blockIdx.x * C + c] = v;
  }
}

void launch_rmsnorm_f32(const float* x, int T, int C, const float* w, float eps, float* y,
                        hipStream_t s, uint16_t* yp, long long plane) {
  hipLaunchKernelGGL(rmsnorm_f32_kernel, dim3(T), dim3(256), 0, s, x, C, w, eps, y, yp, plane);
}

// (x and y may alias: callers normalise in place; each thread rewrites only elements it read)
__global__ void layernorm_f32_kernel(const float* x, int C, const float* __restrict__ w,
                                     const float* __restrict__ b, float eps, float* y) {
  __shared__ float red[16];
  const float* xr = x + (size_t)blockIdx.x * C;
  float s1 = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) s1 += xr[c];
  const float mean = block_sum(s1, red) / (float)C;
  float s2 = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) { const float d = xr[c] - mean; s2 += d * d; }
  const float rstd = 1.0f / sqrtf(block_sum(s2, red) / (float)C + eps);
  for (int c = threadIdx.x; c < C; c += blockDim.x)
    y[(size_t)blockIdx.x * C + c] = (xr[c] - mean) * rstd * w[c] + b[c];
}

void launch_layernorm_f32(const float* x, int T, int C, const float* w, const float* b, float eps,
                          float* y, hipStream_t s) {
  hipLaunchKernelGGL(layernorm_f32_kernel, dim3(T), dim3(256), 0, s, x, C, w, b, eps, y);
}


// ------------------------------------------------------------- codec attention --------
// Non-causal SDPA (decoder_modules.py:283-285) for head_dim 64 in fp32, as flash attention on
// the bf16x3 MFMA form of the GEMM (every fp32 operand x = h + m + l, six bf16 products,
// fp32 accumulation: fp32 products).  One workgroup = (utterance, 64-query block, head), four
// waves of 16 queries each; keys in chunks of 64 with online softmax.  Per chunk the
// workgroup stages K [key][d] and V^T [d][key] split into their three bf16 planes in LDS;
// each wave computes its S = Q K^T (16 x 64) on v_mfma_f32_16x16x32_bf16, does the softmax
// on the accumulators (a query row lives in one 16-lane DPP row), passes P through a private
// LDS tile to re-read it as the A operand, and accumulates O += P V.
constexpr int AB = 64;        // queries per workgroup / keys per chunk
constexpr int AD = 64;        // head dim
constexpr int APL = AB + 8;   // bf16 row stride of the K / V^T planes (144 B; 160 B, conflict-free in
                              // ds_read_b128's lane groups, took the conflicts from 43 % to 32 % of
                              // the LDS cycles and changed nothing else: profiles/r5l_*)
constexpr int APS = AB + 4;   // fp32 row stride of a wave's P tile
constexpr size_t attn_lds(int nw) { return 2 * 3 * 64 * APL * 2 + (size_t)nw * 16 * APS * 4; }

// 8 fp32 -> (h, m, l) bf16x8 planes with h + m + l == x (as split8 in gemm_bx3_kernel)
TTS_DEV void split3(const float (&v)[8], u32x4_t& h, u32x4_t& m, u32x4_t& l) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float h0 = rbf(v[2 * q]), h1 = rbf(v[2 * q + 1]);
    const float r0 = v[2 * q] - h0, r1 = v[2 * q + 1] - h1;
    const float m0 = rbf(r0), m1 = rbf(r1);
    h[q] = pack_bf2(h0, h1);
    m[q] = pack_bf2(m0, m1);
    l[q] = pack_bf2(r0 - m0, r1 - m1);
  }
}

// c += a . b over the three planes, smallest products first (as gemm_bx3_kernel)
TTS_DEV f32x4_t mfma_x3(const u32x4_t (&a)[3], const u32x4_t (&b)[3], f32x4_t c) {
  auto bf = [](const u32x4_t& x) { return __builtin_bit_cast(bf16x8_t, x); };
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf(a[1]), bf(b[1]), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf(a[2]), bf(b[0]), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf(a[0]), bf(b[2]), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf(a[1]), bf(b[0]), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf(a[0]), bf(b[1]), c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf(a[0]), bf(b[0]), c, 0, 0, 0);
}

// torchtune RotaryPositionalEmbeddings(dim=64, base=10000) as the reference applies it to
// [b, h, t, d] tensors: the rotated "sequence" index is the HEAD index (decoder_modules.py
// 276-281; same quirk documented in transformers models/xcodec2), pairs interleaved: the
// pair (d, d+1) of head h turns by h * 10000^(-d/64).  Applied in the attention kernel's
// staging to 8 consecutive dims d0 .. d0+7 of q (and, with the same formula, of k).
// (cos, sin) of every (head, pair) come from a table made once at load (codec_rope_table)
TTS_DEV void rope8(float (&v)[8], const float2* __restrict__ cs, int d0) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float2 t = cs[(d0 >> 1) + j];
    const float c = t.x, sn = t.y;
    const float x0 = v[2 * j], x1 = v[2 * j + 1];
    v[2 * j] = x0 * c - x1 * sn;
    v[2 * j + 1] = x1 * c + x0 * sn;
  }
}

// max / sum over the 16 lanes of a DPP row (every lane ends with the same bits)
TTS_DEV float row16_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(-INFINITY, v));
  v = fmaxf(v, dpp_mov<0x4E>(-INFINITY, v));
  v = fmaxf(v, dpp_mov<0x141>(-INFINITY, v));
  return fmaxf(v, dpp_mov<0x140>(-INFINITY, v));
}
TTS_DEV float row16_sum(float v) {
  v += dpp_mov<0xB1>(0.f, v);
  v += dpp_mov<0x4E>(0.f, v);
  v += dpp_mov<0x141>(0.f, v);
  return v + dpp_mov<0x140>(0.f, v);
}

// NW waves = 16 NW queries per workgroup (the K / V^T staging of a chunk is shared by them)
template <int NW>
__global__ __launch_bounds__(64 * NW) void codec_attn_kernel(const float* __restrict__ qkv_all,
                                                         const CodecSeg* __restrict__ seg,
                                                         const int2* __restrict__ qblk, int heads,
                                                         const float2* __restrict__ rope_cs,
                                                         float* __restrict__ out_all, int expf_mode,
                                                         uint16_t* __restrict__ outp, long long plane) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* Ks = (bf16_t*)smem;                 // [3][64 keys][APL]
  bf16_t* Vt = Ks + 3 * 64 * APL;             // [3][64 d][APL]
  float* Ps = (float*)(Vt + 3 * 64 * APL);    // [NW waves][16][APS]
  // block-diagonal over a ragged batch: (utterance, query block, head), keys of that
  // utterance only
  const int2 qb = qblk[blockIdx.x];
  const int h = blockIdx.y, q0 = qb.y;
  const int T = seg[qb.x].T;
  const int W = heads * AD, ld = 3 * W;
  const float* qkv = qkv_all + (size_t)seg[qb.x].row * ld;
  float* out = out_all + (size_t)seg[qb.x].row * W;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, g = lane >> 4, c16 = lane & 15;
  float* Pw = Ps + wave * 16 * APS;
  // expf_mode 0: softmax in base 2 (scores scaled by 1/sqrt(64) * log2(e) once, p = 2^(s - m) on
  // v_exp_f32); 1 (default): libm expf on s / 8
  const bool use_expf = expf_mode != 0;
  const float scale = use_expf ? 0.125f : 0.125f * 1.44269504088896341f;

  // Q fragments (A operand, row = query c16 of the wave, d = 32 kk + 8 g + j), split once
  u32x4_t qa[2][3];
  {
    const int q = q0 + wave * 16 + c16;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (q < T) {
        const float4* p = (const float4*)(qkv + (size_t)q * ld + h * AD + kk * 32 + 8 * g);
        const float4 a = p[0], b = p[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      }
      rope8(v, rope_cs + h * (AD / 2), kk * 32 + 8 * g);  // (the rotation of q, fused here)
      split3(v, qa[kk][0], qa[kk][1], qa[kk][2]);
    }
  }
  float mrow[4], lrow[4];
  f32x4_t o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    mrow[r] = -INFINITY;
    lrow[r] = 0.f;
  }
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // this thread's share of a chunk: K units (key, 8 d) u = t, t + 64 NW, ...; one V^T unit
  // of (8 keys, VD dims)
  constexpr int NT = 64 * NW, KIT = 512 / NT, VD = 512 / NT;
  const int dp = t % (64 / VD), kg = t / (64 / VD);
  float kreg[KIT][8], v0[8], v1[8];
  auto load = [&](int k0) {  // global -> registers (zeros past the utterance's last key)
#pragma unroll
    for (int it = 0; it < KIT; ++it) {
      const int u = t + NT * it, key = u >> 3, d8 = (u & 7) * 8;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (k0 + key < T) {
        const float4* p = (const float4*)(qkv + (size_t)(k0 + key) * ld + W + h * AD + d8);
        a = p[0];
        b = p[1];
      }
      kreg[it][0] = a.x; kreg[it][1] = a.y; kreg[it][2] = a.z; kreg[it][3] = a.w;
      kreg[it][4] = b.x; kreg[it][5] = b.y; kreg[it][6] = b.z; kreg[it][7] = b.w;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool in = k0 + 8 * kg + i < T;
      const float* vp = qkv + (size_t)(k0 + 8 * kg + i) * ld + 2 * W + h * AD + VD * dp;
      if constexpr (VD == 2) {
        float2 x = make_float2(0.f, 0.f);
        if (in) x = *(const float2*)vp;
        v0[i] = x.x;
        v1[i] = x.y;
      } else {
        v0[i] = in ? *vp : 0.f;
      }
    }
  };
  // the rotation of k (fused): this thread's K units always hold dims (t & 7) * 8 .. +7
  float kc_[4], ks_[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float2 cs = rope_cs[h * (AD / 2) + ((t & 7) * 8 >> 1) + j];
    kc_[j] = cs.x;
    ks_[j] = cs.y;
  }
  load(0);
  for (int k0 = 0; k0 < T; k0 += AB) {
    __syncthreads();  // the previous chunk's K / V^T reads are done
#pragma unroll
    for (int it = 0; it < KIT; ++it) {
      const int u = t + NT * it, key = u >> 3, d8 = (u & 7) * 8;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x0 = kreg[it][2 * j], x1 = kreg[it][2 * j + 1];
        kreg[it][2 * j] = x0 * kc_[j] - x1 * ks_[j];
        kreg[it][2 * j + 1] = x1 * kc_[j] + x0 * ks_[j];
      }
      u32x4_t ph, pm, pl;
      split3(kreg[it], ph, pm, pl);
      *(u32x4_t*)(Ks + (0 * 64 + key) * APL + d8) = ph;
      *(u32x4_t*)(Ks + (1 * 64 + key) * APL + d8) = pm;
      *(u32x4_t*)(Ks + (2 * 64 + key) * APL + d8) = pl;
    }
    {
      u32x4_t ph, pm, pl;
      split3(v0, ph, pm, pl);
      *(u32x4_t*)(Vt + (0 * 64 + VD * dp) * APL + 8 * kg) = ph;
      *(u32x4_t*)(Vt + (1 * 64 + VD * dp) * APL + 8 * kg) = pm;
      *(u32x4_t*)(Vt + (2 * 64 + VD * dp) * APL + 8 * kg) = pl;
      if constexpr (VD == 2) {
        split3(v1, ph, pm, pl);
        *(u32x4_t*)(Vt + (0 * 64 + 2 * dp + 1) * APL + 8 * kg) = ph;
        *(u32x4_t*)(Vt + (1 * 64 + 2 * dp + 1) * APL + 8 * kg) = pm;
        *(u32x4_t*)(Vt + (2 * 64 + 2 * dp + 1) * APL + 8 * kg) = pl;
      }
    }
    __syncthreads();
    if (k0 + AB < T) load(k0 + AB);  // next chunk in flight during this chunk's math
    // S tile kt (keys 16 kt + c16 of lane's column; rows 4 g + r)
    f32x4_t sc[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      sc[kt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        u32x4_t kb[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          kb[pl] = *(const u32x4_t*)(Ks + (pl * 64 + 16 * kt + c16) * APL + kk * 32 + 8 * g);
        sc[kt] = mfma_x3(qa[kk], kb, sc[kt]);
      }
    }
    // online softmax per query row (rows 4 g + r: one DPP row of 16 lanes)
    float alpha[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const float sv = (k0 + 16 * kt + c16 < T) ? sc[kt][r] * scale : -INFINITY;
        sc[kt][r] = sv;
        mx = fmaxf(mx, sv);
      }
      mx = row16_max(mx);
      const float mnew = fmaxf(mrow[r], mx);
      float ps = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const float p = use_expf ? expf(sc[kt][r] - mnew) : __builtin_amdgcn_exp2f(sc[kt][r] - mnew);
        Pw[(4 * g + r) * APS + 16 * kt + c16] = p;
        ps += p;
      }
      ps = row16_sum(ps);
      alpha[r] = use_expf ? expf(mrow[r] - mnew) : __builtin_amdgcn_exp2f(mrow[r] - mnew);
      lrow[r] = lrow[r] * alpha[r] + ps;
      mrow[r] = mnew;
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[dt][r] *= alpha[r];
    // O += P V: A = P (row = query c16, keys 32 kk + 8 g + j) from the wave's own tile
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x4_t pa[3];
      {
        const float4* p = (const float4*)(Pw + c16 * APS + kk * 32 + 8 * g);
        const float4 a = p[0], b = p[1];
        const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        split3(v, pa[0], pa[1], pa[2]);
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        u32x4_t vb[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          vb[pl] = *(const u32x4_t*)(Vt + (pl * 64 + 16 * dt + c16) * APL + kk * 32 + 8 * g);
        o[dt] = mfma_x3(pa, vb, o[dt]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = q0 + wave * 16 + 4 * g + r;
    if (q >= T) continue;
    const float inv = 1.0f / lrow[r];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const size_t oi = (size_t)q * W + h * AD + 16 * dt + c16;
      if (outp) store_planes(outp, plane, (size_t)seg[qb.x].row * W + oi, o[dt][r] * inv);  // (c_proj's planes)
      else out[oi] = o[dt][r] * inv;
    }
  }
}

// queries per workgroup: 64 (4 waves; the 8-wave form was dropped in round 5)
static int attn_waves() { return 4; }
int codec_attn_qrows() { return 16 * attn_waves(); }
int codec_attn_qblocks(int T) { return (T + codec_attn_qrows() - 1) / codec_attn_qrows(); }

void launch_codec_attention(const float* qkv, const CodecSeg* seg, const int2* qblk, int nqblk, int heads,
                            int hd, const float* rope_cs, float* out, hipStream_t s, uint16_t* outp, long long plane) {
  if (hd != AD) throw std::runtime_error("codec attention: head_dim 64 expected");
  dim3 grid(nqblk, heads);
  // libm expf by default: the base-2 v_exp_f32 form measured neutral here (32 x 650 codes 62.0 ms
  // either way, profiles/r4e_ab_codec_expf.txt: the softmax is not what bounds this kernel), so
  // the reference's exp stays.  TTS_CODEC_EXPF=0: v_exp_f32
  static const int expf_mode = getenv("TTS_CODEC_EXPF") ? atoi(getenv("TTS_CODEC_EXPF")) : 1;
  hipLaunchKernelGGL(codec_attn_kernel<4>, grid, dim3(256), attn_lds(4), s, qkv, seg, qblk, heads,
                     (const float2*)rope_cs, out, expf_mode, outp, plane);
}

// (cos, sin) of the torchtune rotation for every (head h, pair p): angle h * 10000^(-2p/64),
// fp32 as the reference's cache (decoder_modules.py:276-281: position = head index)
__global__ void codec_rope_table_kernel(float2* cs, int heads) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= heads * (AD / 2)) return;
  const int h = i / (AD / 2), pi = i % (AD / 2);
  const float theta = 1.0f / powf(10000.0f, (float)(2 * pi) / (float)AD);
  const float ang = (float)h * theta;
  cs[i] = make_float2(cosf(ang), sinf(ang));
}

void launch_codec_rope_table(float* cs, int heads, hipStream_t s) {
  hipLaunchKernelGGL(codec_rope_table_kernel, dim3((heads * (AD / 2) + 255) / 256), dim3(256), 0, s, (float2*)cs,
                     heads);
}

// ConvTranspose1d(stride u, padding pad) from Z[t][j*Cout + co] = sum_ci x[t][ci] W[ci][co][j]:
// output t' receives tap j from input t with t*u - pad + j = t'.
__global__ void convt_gather_kernel(const float* __restrict__ Z_all, const CodecSeg* __restrict__ seg_in,
                                    const CodecSeg* __restrict__ seg_out, int Cout, int k, int u, int pad,
                                    const float* __restrict__ bias, float* __restrict__ y_all) {
  const int b = blockIdx.y;
  const int T = seg_in[b].T, To = seg_out[b].T;
  const float* Z = Z_all + (size_t)seg_in[b].row * k * Cout;
  float* y = y_all + (size_t)seg_out[b].row * Cout;
  const long long n = (long long)To * Cout;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int tp = (int)(i / Cout), co = (int)(i % Cout);
    float acc = bias[co];
    for (int j = 0; j < k; ++j) {
      const int num = tp + pad - j;
      if (num < 0 || num % u) continue;
      const int ti = num / u;
      if (ti >= T) continue;
      acc += Z[(size_t)ti * k * Cout + j * Cout + co];
    }
    y[i] = acc;
  }
}

void launch_convt_gather(const float* Z, const CodecSeg* seg_in, const CodecSeg* seg_out, int B, int max_To, int Cout,
                         int k, int u, int pad, const float* bias, float* y, hipStream_t s) {
  const long long n = (long long)max_To * Cout;
  int grid = (int)std::min<long long>((n + 255) / 256, std::max(1, 8192 / B));
  hipLaunchKernelGGL(convt_gather_kernel, dim3(grid, B), dim3(256), 0, s, Z, seg_in, seg_out, Cout, k, u, pad,
                     bias, y);
}

// ISTFTHead (decoder_modules.py:134-147): mag = clip(exp(x[:nb]), max=1e2), p = x[nb:2nb],
// spec = [mag*cos(p) | mag*sin(p) | 0-pad]
__global__ void istft_spec_kernel(const float* __restrict__ head, int nb, int ld,
                                  float* __restrict__ spec) {
  const int f = blockIdx.x;
  const float* hr = head + (size_t)f * ld;
  float* sr = spec + (size_t)f * ld;
  for (int k = threadIdx.x; k < ld; k += blockDim.x) {
    if (k < nb) {
      const float mag = fminf(expf(hr[k]), 1e2f);
      const float p = hr[nb + k];
      sr[k] = mag * cosf(p);
      sr[nb + k] = mag * sinf(p);
    } else if (k >= 2 * nb) {
      sr[k] = 0.f;
    }
  }
}

void launch_istft_spec(const float* head, int F, int nb, int ld, float* spec, hipStream_t s) {
  hipLaunchKernelGGL(istft_spec_kernel, dim3(F), dim3(256), 0, s, head, nb, ld, spec);
}

// ISTFT 'same' overlap-add (decoder_modules.py:64-93): frames are already irfft'ed and
// windowed; y[i] = sum_f frames[f][i+pad-f*hop] / sum_f window^2[i+pad-f*hop].
__global__ void ola_kernel(const float* __restrict__ frames_all, const CodecSeg* __restrict__ seg,
                           const long long* __restrict__ wav_off, int nfft, int hop,
                           const float* __restrict__ win, float* __restrict__ y_all) {
  const int b = blockIdx.y;
  const int F = seg[b].T;
  const float* frames = frames_all + (size_t)seg[b].row * nfft;
  float* y = y_all + wav_off[b];
  const int pad = (nfft - hop) / 2;
  const long long L = (long long)F * hop;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < L;
       i += (long long)gridDim.x * blockDim.x) {
    const long long g = i + pad;
    long long f_hi = g / hop;
    if (f_hi > F - 1) f_hi = F - 1;
    long long f_lo = (g - nfft + hop) / hop;  // smallest f with g - f*hop < nfft
    if (g - nfft + hop < 0) f_lo = 0;
    if (f_lo < 0) f_lo = 0;
    float acc = 0.f, env = 0.f;
    for (long long f = f_lo; f <= f_hi; ++f) {
      const int n = (int)(g - f * hop);
      if (n < 0 || n >= nfft) continue;
      acc += frames[(size_t)f * nfft + n];
      env += win[n] * win[n];
    }
    y[i] = acc / env;
  }
}

void launch_ola(const float* frames, const CodecSeg* seg, const long long* wav_off, int B, int max_F, int nfft,
                int hop, const float* window, float* y, hipStream_t s) {
  const long long L = (long long)max_F * hop;
  int grid = (int)std::min<long long>((L + 255) / 256, std::max(1, 8192 / B));
  hipLaunchKernelGGL(ola_kernel, dim3(grid, B), dim3(256), 0, s, frames, seg, wav_off, nfft, hop, window, y);
}

__global__ void zero_kernel(float* p, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    p[i] = 0.f;
}

void launch_zero(float* p, long long n, hipStream_t s) {
  if (n <= 0) return;
  int grid = (int)std::min<long long>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(zero_kernel, dim3(grid), dim3(256), 0, s, p, n);
}

}  // namespace tts
