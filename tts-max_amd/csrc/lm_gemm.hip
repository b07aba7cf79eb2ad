// lm_gemm.hip — weight-streaming bf16 GEMM for the SpeechLM (decode GEMV, batched decode,
// chunked prefill) with fused prologue (RMSNorm) and epilogues (store / residual add /
// SwiGLU / lm_head+repetition-penalty+EOS-mask+argmax).
//
// Reference semantics (transformers LlamaForCausalLM, pinned 4.53.2 by uv.lock:4610):
//   nn.Linear in bf16 = fp32-accumulated dot product rounded once to bf16.
//   LlamaRMSNorm (modeling_llama.py:62-67): fp32 mean(x^2), rsqrt(var+eps), cast to bf16,
//     then weight * x in bf16.
//   LlamaMLP (modeling_llama.py:163-176): down(silu(gate(x)) * up(x)), each op rounded to bf16.
//   Decoder residual (modeling_llama.py:~310-322): residual + h rounded to bf16.
//   lm_head + GenerationMixin._sample (generation/utils.py:2894-2925): logits in bf16,
//     .float(), RepetitionPenaltyLogitsProcessor (logits_process.py:306-413),
//     MinNewTokensLengthLogitsProcessor (:164-236), argmax (first max on ties).
//
// MI355X design: weights are re-laid out at load time into 1 KiB MFMA B-fragment tiles so
// that every wave-instruction streams 1 KiB of contiguous HBM and feeds
// v_mfma_f32_16x16x32_bf16 with no shuffles.  Tile (nt, kt) holds
//   tile[lane*8 + j] = W[nt*16 + (lane & 15)][kt*32 + 8*(lane >> 4) + j]
// and tiles of one n-tile are consecutive along K.  Activations (M <= 64 rows) are the
// A operand; at M = 1 fifteen of the sixteen A rows are zero, which costs nothing because
// the kernel is HBM-bound on the weight stream.
#include "hip_common.h"
#include "lm_kernels.h"

namespace tts {

// ---------------------------------------------------------------- weight re-layout ----
__global__ void retile_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ t, int N,
                              int K, int nt_mult, int nt_off) {
  const int KT = K / 32;
  const long long nchunks = (long long)(N / 16) * KT * 64;
  for (long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x; c < nchunks;
       c += (long long)gridDim.x * blockDim.x) {
    const int lane = (int)(c & 63);
    const long long tile = c >> 6;
    const int kt = (int)(tile % KT);
    const int nt = (int)(tile / KT);
    const int n = nt * 16 + (lane & 15);
    const int k = kt * 32 + 8 * (lane >> 4);
    const u32x4_t v = *(const u32x4_t*)(w + (size_t)n * K + k);
    const long long dtile = (long long)(nt * nt_mult + nt_off) * KT + kt;
    *(u32x4_t*)(t + (size_t)(dtile * 64 + lane) * 8) = v;
  }
}

void launch_retile(const bf16_t* w, bf16_t* t, int N, int K, hipStream_t s, int nt_mult,
                   int nt_off) {
  long long nchunks = (long long)(N / 16) * (K / 32) * 64;
  int grid = (int)((nchunks + 255) / 256);
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(retile_kernel, dim3(grid), dim3(256), 0, s, w, t, N, K, nt_mult, nt_off);
}

// ---------------------------------------------------------------- the GEMM kernel -----
// One workgroup = WAVES waves; KSPLIT consecutive waves split the K range of one unit
// (a unit = NG n-tiles of 16 output columns), WAVES/KSPLIT units run side by side, and
// the workgroup walks units grid-stride.  Each wave streams its weight tiles in stages
// of KU tiles (KU KiB), double-buffered, and the stream never stops: the first stage is
// issued before the A-operand prologue (RMSNorm / attention combine), and the last stage
// of a unit prefetches the first stage of the wave's next unit.
TTS_DEV bf16x8_t as_bf16x8(u32x4_t v) { return __builtin_bit_cast(bf16x8_t, v); }

// Better (value, index): larger value wins, lower index on ties (torch.argmax semantics).
TTS_DEV void argmax_merge(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}

constexpr int A_GLOBAL = 0, A_LDS = 1, A_ATTN = 2;

// MT_MAX: compile-time bound on 16-row m-tiles (1 for decode, 4 for up to 64 rows)
template <int WAVES, int KU, int MT_MAX, int NG, int KSPLIT, int ASRC, bool NORM, int EPI>
__global__ __launch_bounds__(WAVES * 64) void wgemm_kernel(WgemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NT = WAVES * 64;
  constexpr int UPW = WAVES / KSPLIT;  // units processed concurrently by one workgroup
  if ((int)blockIdx.x >= a.real_grid) {
    prefetch_role(a.pf.ptr, a.pf.bytes, blockIdx.x - a.real_grid, gridDim.x - a.real_grid);
    return;
  }
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int kpart = wave % KSPLIT;
  const int ugrp = wave / KSPLIT;
  const int M = a.M;
  const int mtn = (M + 15) >> 4;
  const int KT = a.K >> 5;
  const int units = (a.N >> 4) / NG;
  const int kt_per = KT / KSPLIT;
  const int kt0 = kpart * kt_per;
  const int kend = kt0 + kt_per;
  const int ldxs = a.K + 8;  // +16 B per row: the 16 A rows land on distinct LDS bank slots
  const int ustride = a.real_grid * UPW;

  bf16_t* xs = (bf16_t*)smem;
  const size_t xs_bytes = (ASRC != A_GLOBAL) ? (((size_t)M * ldxs * 2 + 15) & ~(size_t)15) : 0;
  float* red = (float*)(smem + xs_bytes);  // [WAVES][NG*MT_MAX*4][64] split-K partials
  float* scal = red + WAVES * NG * MT_MAX * 4 * 64;

  // ---- start the weight stream before anything else
  int u = blockIdx.x * UPW + ugrp;
  u32x4_t wb[KU][NG];
  auto wptr = [&](int uu, int g) {
    return (const u32x4_t*)(a.w + ((size_t)(uu * NG + g) * KT) * 512) + lane;
  };
  if (u < units) {
#pragma unroll
    for (int kk = 0; kk < KU; ++kk)
#pragma unroll
      for (int g = 0; g < NG; ++g) wb[kk][g] = __builtin_nontemporal_load(wptr(u, g) + (kt0 + kk) * 64);
  }

  // ---- prologue: A rows in LDS (plain, RMSNorm'ed, or combined from attention chunks)
  if constexpr (ASRC == A_LDS) {
    // rows in parallel: wave w stages rows w, w+WAVES, ... (DPP row reduction, no barrier)
    // One pass per row, all of a lane's 16-B chunks in flight at once (K <= 4096 for the
    // RMSNorm'ed rows; longer plain rows go in batches of 8 chunks).
    constexpr int CPL = 8;  // chunks per lane held in registers
    for (int m = wave; m < M; m += WAVES) {
      const bf16_t* xr = a.x + (size_t)m * a.ldx;
      for (int k0 = 0; k0 < a.K; k0 += 64 * 8 * CPL) {
        u32x4_t xv[CPL];
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int k = k0 + (c * 64 + lane) * 8;
          if (k < a.K) xv[c] = *(const u32x4_t*)(xr + k);
        }
        if constexpr (NORM) {  // (K <= 64*8*CPL: the whole row is in xv)
          float ss = 0.f;
#pragma unroll
          for (int c = 0; c < CPL; ++c) {
            if ((c * 64 + lane) * 8 < a.K) {
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const float lo = bf_lo(xv[c][q]), hi = bf_hi(xv[c][q]);
                ss += lo * lo + hi * hi;
              }
            }
          }
          ss = wave_sum_dpp(ss);
          const float r = 1.0f / sqrtf(ss / (float)a.K + a.eps);
#pragma unroll
          for (int c = 0; c < CPL; ++c) {
            const int k = (c * 64 + lane) * 8;
            if (k < a.K) {
              const u32x4_t g = *(const u32x4_t*)(a.normw + k);
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const float lo = rbf(bf_lo(g[q]) * rbf(bf_lo(xv[c][q]) * r));
                const float hi = rbf(bf_hi(g[q]) * rbf(bf_hi(xv[c][q]) * r));
                xv[c][q] = pack_bf2(lo, hi);
              }
            }
          }
        }
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int k = k0 + (c * 64 + lane) * 8;
          if (k < a.K) *(u32x4_t*)(xs + (size_t)m * ldxs + k) = xv[c];
        }
      }
    }
    __syncthreads();
  } else if constexpr (ASRC == A_ATTN) {
    // o[m][h*D+d] = sum_s o_s f_s,  f_s = e^(m_s - M) / sum_s' l_s' e^(m_s' - M)
    // phase 1: one thread per (row, head) turns the chunk statistics into factors (LDS);
    // phase 2: every thread merges its (row, head, dim) elements with independent loads.
    const int D = a.attn_D, H = a.K / D, NS = a.attn_nsplit;
    float* fac = (float*)(smem + xs_bytes) + WAVES * NG * MT_MAX * 4 * 64 + 64;
    for (int mh = threadIdx.x; mh < M * H; mh += NT) {
      const int m = mh / H;
      const int ns = (a.attn_pos[m] + a.attn_split) / a.attn_split;
      const float* ml = a.attn_ml + (size_t)mh * NS * 2;
      float mx = -INFINITY;
      for (int s = 0; s < ns; ++s) mx = fmaxf(mx, ml[2 * s]);
      float l = 0.f;
      for (int s = 0; s < ns; ++s) {
        const float f = expf(ml[2 * s] - mx);
        fac[mh * NS + s] = f;
        l += ml[2 * s + 1] * f;
      }
      const float il = 1.0f / l;
      for (int s = 0; s < ns; ++s) fac[mh * NS + s] *= il;
    }
    __syncthreads();
    // 8 consecutive dims per thread: two float4 loads per chunk, one 16-B LDS store
    for (int e = threadIdx.x; e < M * a.K / 8; e += NT) {
      const int m = (e * 8) / a.K, hd = (e * 8) % a.K, mh = m * H + hd / D, d = hd % D;
      const int ns = (a.attn_pos[m] + a.attn_split) / a.attn_split;
      const float* po = a.attn_o + (size_t)mh * NS * D + d;
      const float* f = fac + mh * NS;
      float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int s = 0; s < ns; ++s) {
        const float4 v0 = *(const float4*)(po + (size_t)s * D);
        const float4 v1 = *(const float4*)(po + (size_t)s * D + 4);
        const float fs = f[s];
        o[0] += v0.x * fs; o[1] += v0.y * fs; o[2] += v0.z * fs; o[3] += v0.w * fs;
        o[4] += v1.x * fs; o[5] += v1.y * fs; o[6] += v1.z * fs; o[7] += v1.w * fs;
      }
      u32x4_t pk;
#pragma unroll
      for (int q = 0; q < 4; ++q) pk[q] = pack_bf2(o[2 * q], o[2 * q + 1]);
      *(u32x4_t*)(xs + (size_t)m * ldxs + hd) = pk;
    }
    __syncthreads();
  }

  const int arow = lane & 15;
  const int akoff = 8 * (lane >> 4);

  // per-lane running argmax (EPI_LOGITS): rows m = mt*16 + 4*(lane>>4) + r
  float best_v[MT_MAX][4];
  int best_i[MT_MAX][4];
#pragma unroll
  for (int mt = 0; mt < MT_MAX; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) { best_v[mt][r] = -INFINITY; best_i[mt][r] = 0x7fffffff; }

  for (int ubase = blockIdx.x * UPW; ubase < units; ubase += ustride) {
    u = ubase + ugrp;
    const bool active = u < units;
    f32x4_t acc[NG][MT_MAX];
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int mt = 0; mt < MT_MAX; ++mt) acc[g][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    if (active) {
      const int unext = u + ustride;
      for (int kt = kt0; kt < kend; kt += KU) {
        // next stage: same unit, else the first stage of the wave's next unit
        int nu = u, nk = kt + KU;
        if (nk >= kend) { nu = unext; nk = kt0; }
        const bool has_next = nu < units;
        u32x4_t wn[KU][NG];
        if (has_next) {
#pragma unroll
          for (int kk = 0; kk < KU; ++kk)
#pragma unroll
            for (int g = 0; g < NG; ++g) wn[kk][g] = __builtin_nontemporal_load(wptr(nu, g) + (nk + kk) * 64);
        }

#pragma unroll
        for (int kk = 0; kk < KU; ++kk) {
          const int k = (kt + kk) * 32 + akoff;
#pragma unroll
          for (int mt = 0; mt < MT_MAX; ++mt) {
            if (mt < mtn) {
              const int m = mt * 16 + arow;
              u32x4_t av = u32x4_t{0u, 0u, 0u, 0u};
              if (m < M) {
                if constexpr (ASRC != A_GLOBAL) av = *(const u32x4_t*)(xs + (size_t)m * ldxs + k);
                else av = *(const u32x4_t*)(a.x + (size_t)m * a.ldx + k);
              }
              const bf16x8_t af = as_bf16x8(av);
#pragma unroll
              for (int g = 0; g < NG; ++g)
                acc[g][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, as_bf16x8(wb[kk][g]),
                                                                     acc[g][mt], 0, 0, 0);
            }
          }
        }
        if (has_next) {
#pragma unroll
          for (int kk = 0; kk < KU; ++kk)
#pragma unroll
            for (int g = 0; g < NG; ++g) wb[kk][g] = wn[kk][g];
        }
      }
    }

    // ---- split-K combine through LDS, fixed order (deterministic)
    if constexpr (KSPLIT > 1) {
      constexpr int PS = NG * MT_MAX * 4 * 64;
      float* myred = red + (size_t)wave * PS;
#pragma unroll
      for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int mt = 0; mt < MT_MAX; ++mt)
          if (mt < mtn) {
#pragma unroll
            for (int r = 0; r < 4; ++r) myred[((g * MT_MAX + mt) * 4 + r) * 64 + lane] = acc[g][mt][r];
          }
      __syncthreads();
      if (kpart == 0) {
#pragma unroll
        for (int p = 1; p < KSPLIT; ++p) {
          const float* o = red + (size_t)(wave + p) * PS;
#pragma unroll
          for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int mt = 0; mt < MT_MAX; ++mt)
              if (mt < mtn) {
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[g][mt][r] += o[((g * MT_MAX + mt) * 4 + r) * 64 + lane];
              }
        }
      }
      __syncthreads();
    }

    // ---- epilogue (lane owns column n, rows m = mt*16 + 4*(lane>>4) + r)
    if (kpart == 0 && active) {
      const int n = u * 16 + (lane & 15);
#pragma unroll
      for (int mt = 0; mt < MT_MAX; ++mt) {
        if (mt >= mtn) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = mt * 16 + 4 * (lane >> 4) + r;
          if (m >= M) continue;
          if constexpr (EPI == EPI_STORE) {
            a.out[(size_t)m * a.ldo + n] = f2bf(acc[0][mt][r]);
          } else if constexpr (EPI == EPI_RESID) {
            bf16_t* p = a.resid + (size_t)m * a.ldo + n;
            *p = f2bf(bf2f(*p) + rbf(acc[0][mt][r]));
          } else if constexpr (EPI == EPI_SWIGLU) {
            // unit u = (gate tile, up tile) pair for intermediate columns u*16 .. u*16+15
            const float gt = rbf(acc[0][mt][r]);
            const float up = rbf(acc[NG - 1][mt][r]);
            a.out[(size_t)m * a.ldo + n] = f2bf(rbf(silu_f(gt)) * up);
          } else if constexpr (EPI == EPI_LOGITS) {
            float v = rbf(acc[0][mt][r]);  // logits are materialised in bf16, then .float()
            const uint32_t bits = a.seen[(size_t)m * a.seen_stride + (n >> 5)];
            if ((bits >> (n & 31)) & 1u) v = (v < 0.f) ? v * a.penalty : v / a.penalty;
            if (n == a.eos_mask[m]) v = -INFINITY;
            argmax_merge(best_v[mt][r], best_i[mt][r], v, n);
          }
        }
      }
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
    __syncthreads();
    if (kpart == 0 && (lane & 15) == 0) {
#pragma unroll
      for (int mt = 0; mt < MT_MAX; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = mt * 16 + 4 * (lane >> 4) + r;
          rv[ugrp * MT_MAX * 16 + m] = best_v[mt][r];
          ri[ugrp * MT_MAX * 16 + m] = best_i[mt][r];
        }
    }
    __syncthreads();
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
// Launch shapes (WAVES, KU, KSPLIT): a small fixed table keeps the instantiation count low.
enum { CFG_WIDE = 0, CFG_K2 = 1, CFG_K8 = 3, CFG_K4 = 4, CFG_K4W8 = 5, CFG_K16 = 6 };

template <int WAVES, int KU, int NG, int KSPLIT, int ASRC, bool NORM, int EPI>
static void launch_one(const WgemmArgs& a, int grid, hipStream_t s) {
  const int mt = a.M <= 16 ? 1 : 4;
  size_t lds = (ASRC != A_GLOBAL) ? (((size_t)a.M * (a.K + 8) * 2 + 15) & ~(size_t)15) : 0;
  lds += (size_t)(WAVES * NG * mt * 4 * 64 + 64) * sizeof(float);
  if (ASRC == A_ATTN) lds += (size_t)a.M * (a.K / a.attn_D) * a.attn_nsplit * sizeof(float);
  if (mt == 1) {
    hipLaunchKernelGGL((wgemm_kernel<WAVES, KU, 1, NG, KSPLIT, ASRC, NORM, EPI>), dim3(grid),
                       dim3(WAVES * 64), lds, s, a);
  } else if constexpr (WAVES <= 8) {  // 16-wave shapes are planned for M <= 16 only
    hipLaunchKernelGGL((wgemm_kernel<WAVES, KU, 4, NG, KSPLIT, ASRC, NORM, EPI>), dim3(grid),
                       dim3(WAVES * 64), lds, s, a);
  }
}

template <int NG, int ASRC, bool NORM, int EPI>
static void launch_cfg(const WgemmArgs& a, int cfg, int grid, hipStream_t s) {
  switch (cfg) {
    case CFG_WIDE: launch_one<4, 8, NG, 1, ASRC, NORM, EPI>(a, grid, s); break;
    case CFG_K2: launch_one<4, 8, NG, 2, ASRC, NORM, EPI>(a, grid, s); break;
    case CFG_K8: launch_one<8, 8, NG, 8, ASRC, NORM, EPI>(a, grid, s); break;
    case CFG_K4W8: launch_one<8, 8, NG, 4, ASRC, NORM, EPI>(a, grid, s); break;
    case CFG_K16: launch_one<16, 8, NG, 16, ASRC, NORM, EPI>(a, grid, s); break;
    default: launch_one<4, 8, NG, 4, ASRC, NORM, EPI>(a, grid, s); break;
  }
}

// Chooses the launch shape so that every CU has work and enough bytes in flight: large-N
// GEMMs (lm_head, MLP) stream whole n-tiles per wave; small-N projections split K across
// the waves of a workgroup (and use 8-wave workgroups when only ~128 units exist).
WgemmPlan plan_wgemm(int M, int N, int K, int epi, int num_cu) {
  WgemmPlan p;
  const int NG = (epi == EPI_SWIGLU) ? 2 : 1;
  const int units = (N / 16) / NG;
  const int KT = K / 32;
  p.a_lds = ((size_t)M * (K + 8) * 2) <= 80 * 1024;
  int cfg, upw;
  if (units >= num_cu * 4) { cfg = CFG_WIDE; upw = 4; }
  else if (units >= num_cu * 2 && KT % 32 == 0) { cfg = CFG_K4W8; upw = 2; }
  else if (units >= num_cu * 2 && KT % 16 == 0) { cfg = CFG_K2; upw = 2; }
  else if (2 * units <= num_cu && KT % 128 == 0 && M <= 16) { cfg = CFG_K16; upw = 1; }
  else if (KT % 64 == 0) { cfg = CFG_K8; upw = 1; }
  else if (KT % 32 == 0) { cfg = CFG_K4; upw = 1; }
  else { cfg = CFG_WIDE; upw = 4; }
  // experiment hook (scripts/microbench.py): force a launch shape when it divides the shape
  static const int forced = getenv("TTS_WGEMM_CFG") ? atoi(getenv("TTS_WGEMM_CFG")) : -1;
  if (forced >= 0) {
    const int ks[] = {1, 2, 0, 8, 4, 4, 16};
    const int up[] = {4, 2, 0, 1, 1, 2, 1};
    if (forced <= 6 && ks[forced] && KT % (ks[forced] * 8) == 0 && (forced != CFG_K16 || M <= 16)) {
      cfg = forced;
      upw = up[forced];
    }
  }
  p.cfg = cfg;
  int grid = (units + upw - 1) / upw;
  const int cap = (epi == EPI_LOGITS) ? LOGITS_MAX_PARTS : num_cu * 8;
  if (grid > cap) grid = cap;
  p.grid = grid;
  return p;
}

bool wgemm_supported(int M, int N, int K, int epi) {
  const int NG = (epi == EPI_SWIGLU) ? 2 : 1;
  return M >= 1 && M <= 64 && (N % (16 * NG)) == 0 && (K % 256) == 0;
}

void launch_wgemm(const WgemmArgs& a_in, const WgemmPlan& p, int epi, bool norm, hipStream_t s) {
  WgemmArgs a = a_in;
  a.real_grid = p.grid;
  const int grid = p.grid + ((a.pf.bytes && a.pf.ptr) ? a.pf.wgs : 0);
  const int c = p.cfg;
  const bool attn = a.attn_o != nullptr;
  switch (epi) {
    case EPI_STORE:
      if (!p.a_lds) launch_cfg<1, A_GLOBAL, false, EPI_STORE>(a, c, grid, s);
      else if (norm) launch_cfg<1, A_LDS, true, EPI_STORE>(a, c, grid, s);
      else launch_cfg<1, A_LDS, false, EPI_STORE>(a, c, grid, s);
      break;
    case EPI_RESID:
      if (attn) launch_cfg<1, A_ATTN, false, EPI_RESID>(a, c, grid, s);
      else if (!p.a_lds) launch_cfg<1, A_GLOBAL, false, EPI_RESID>(a, c, grid, s);
      else launch_cfg<1, A_LDS, false, EPI_RESID>(a, c, grid, s);
      break;
    case EPI_SWIGLU:
      if (!p.a_lds) launch_cfg<2, A_GLOBAL, false, EPI_SWIGLU>(a, c, grid, s);
      else if (norm) launch_cfg<2, A_LDS, true, EPI_SWIGLU>(a, c, grid, s);
      else launch_cfg<2, A_LDS, false, EPI_SWIGLU>(a, c, grid, s);
      break;
    case EPI_LOGITS:  // the lm_head always carries the final RMSNorm (fused, or applied before)
      if (!p.a_lds || !norm) launch_cfg<1, A_GLOBAL, false, EPI_LOGITS>(a, c, grid, s);
      else launch_cfg<1, A_LDS, true, EPI_LOGITS>(a, c, grid, s);
      break;
  }
}

}  // namespace tts
