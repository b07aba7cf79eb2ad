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
constexpr int WG_THREADS = 256;
constexpr int KU = 8;  // k-tiles per pipeline stage (8 KiB of weights per wave per stage)

TTS_DEV bf16x8_t as_bf16x8(u32x4_t v) { return __builtin_bit_cast(bf16x8_t, v); }

// Better (value, index): larger value wins, lower index on ties (torch.argmax semantics).
TTS_DEV void argmax_merge(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}

template <int MT, int NG, int KSPLIT, bool A_LDS, bool NORM, int EPI>
__global__ __launch_bounds__(WG_THREADS) void wgemm_kernel(WgemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int UPW = 4 / KSPLIT;  // units processed concurrently by one workgroup
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int kpart = wave % KSPLIT;
  const int ugrp = wave / KSPLIT;
  const int M = a.M;
  const int KT = a.K >> 5;
  const int units = (a.N >> 4) / NG;
  const int kt_per = KT / KSPLIT;
  const int kt0 = kpart * kt_per;
  const int ldxs = a.K + 8;  // +16 B per row: the 16 A rows land on distinct LDS bank slots

  bf16_t* xs = (bf16_t*)smem;
  const size_t xs_bytes = A_LDS ? (((size_t)M * ldxs * 2 + 15) & ~(size_t)15) : 0;
  float* red = (float*)(smem + xs_bytes);  // [4 waves][NG*MT*4][64] split-K partials
  float* scal = red + 4 * NG * MT * 4 * 64;  // small scratch (block reductions)

  // ---- prologue: stage the A rows (optionally RMSNorm'ed) in LDS once per workgroup
  if constexpr (A_LDS) {
    for (int m = 0; m < M; ++m) {
      const bf16_t* xr = a.x + (size_t)m * a.ldx;
      float r = 1.0f;
      if constexpr (NORM) {
        float ss = 0.f;
        for (int k = threadIdx.x * 8; k < a.K; k += WG_THREADS * 8) {
          const u32x4_t v = *(const u32x4_t*)(xr + k);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float lo = bf_lo(v[q]), hi = bf_hi(v[q]);
            ss += lo * lo + hi * hi;
          }
        }
        ss = block_sum(ss, scal);
        r = 1.0f / sqrtf(ss / (float)a.K + a.eps);
      }
      for (int k = threadIdx.x * 8; k < a.K; k += WG_THREADS * 8) {
        u32x4_t v = *(const u32x4_t*)(xr + k);
        if constexpr (NORM) {
          const u32x4_t g = *(const u32x4_t*)(a.normw + k);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float lo = rbf(bf_lo(g[q]) * rbf(bf_lo(v[q]) * r));
            const float hi = rbf(bf_hi(g[q]) * rbf(bf_hi(v[q]) * r));
            v[q] = pack_bf2(lo, hi);
          }
        }
        *(u32x4_t*)(xs + (size_t)m * ldxs + k) = v;
      }
    }
    __syncthreads();
  }

  const int arow = lane & 15;
  const int akoff = 8 * (lane >> 4);

  // per-lane running argmax (EPI_LOGITS): rows m = mt*16 + 4*(lane>>4) + r
  float best_v[MT][4];
  int best_i[MT][4];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) { best_v[mt][r] = -INFINITY; best_i[mt][r] = 0x7fffffff; }

  for (int ubase = blockIdx.x * UPW; ubase < units; ubase += gridDim.x * UPW) {
    const int u = ubase + ugrp;
    const bool active = u < units;
    f32x4_t acc[NG][MT];
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[g][mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    if (active) {
      const u32x4_t* wt[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g)
        wt[g] = (const u32x4_t*)(a.w + ((size_t)(u * NG + g) * KT) * 512) + lane;
      const int kend = kt0 + kt_per;
      u32x4_t wb[KU][NG];
#pragma unroll
      for (int kk = 0; kk < KU; ++kk)
#pragma unroll
        for (int g = 0; g < NG; ++g) wb[kk][g] = __builtin_nontemporal_load(wt[g] + (kt0 + kk) * 64);

      for (int kt = kt0; kt < kend; kt += KU) {
        // prefetch the next stage (clamped: the last stage re-reads itself, never out of range)
        const int ktn = (kt + KU < kend) ? kt + KU : kt;
        u32x4_t wn[KU][NG];
#pragma unroll
        for (int kk = 0; kk < KU; ++kk)
#pragma unroll
          for (int g = 0; g < NG; ++g) wn[kk][g] = __builtin_nontemporal_load(wt[g] + (ktn + kk) * 64);

#pragma unroll
        for (int kk = 0; kk < KU; ++kk) {
          const int k = (kt + kk) * 32 + akoff;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const int m = mt * 16 + arow;
            u32x4_t av = u32x4_t{0u, 0u, 0u, 0u};
            if (m < M) {
              if constexpr (A_LDS) av = *(const u32x4_t*)(xs + (size_t)m * ldxs + k);
              else av = *(const u32x4_t*)(a.x + (size_t)m * a.ldx + k);
            }
            const bf16x8_t af = as_bf16x8(av);
#pragma unroll
            for (int g = 0; g < NG; ++g)
              acc[g][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, as_bf16x8(wb[kk][g]),
                                                                   acc[g][mt], 0, 0, 0);
          }
        }
#pragma unroll
        for (int kk = 0; kk < KU; ++kk)
#pragma unroll
          for (int g = 0; g < NG; ++g) wb[kk][g] = wn[kk][g];
      }
    }

    // ---- split-K combine through LDS, fixed order (deterministic)
    if constexpr (KSPLIT > 1) {
      float* myred = red + (size_t)wave * (NG * MT * 4 * 64);
#pragma unroll
      for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) myred[((g * MT + mt) * 4 + r) * 64 + lane] = acc[g][mt][r];
      __syncthreads();
      if (kpart == 0) {
#pragma unroll
        for (int p = 1; p < KSPLIT; ++p) {
          const float* o = red + (size_t)(wave + p) * (NG * MT * 4 * 64);
#pragma unroll
          for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
              for (int r = 0; r < 4; ++r) acc[g][mt][r] += o[((g * MT + mt) * 4 + r) * 64 + lane];
        }
      }
      __syncthreads();
    }

    // ---- epilogue (lane owns column n, rows m = mt*16 + 4*(lane>>4) + r)
    if (kpart == 0 && active) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = mt * 16 + 4 * (lane >> 4) + r;
          if (m >= M) continue;
          if constexpr (EPI == EPI_STORE) {
            const int n = u * 16 + (lane & 15);
            a.out[(size_t)m * a.ldo + n] = f2bf(acc[0][mt][r]);
          } else if constexpr (EPI == EPI_RESID) {
            const int n = u * 16 + (lane & 15);
            bf16_t* p = a.resid + (size_t)m * a.ldo + n;
            *p = f2bf(bf2f(*p) + rbf(acc[0][mt][r]));
          } else if constexpr (EPI == EPI_SWIGLU) {
            // unit u = (gate tile, up tile) pair for intermediate columns u*16 .. u*16+15
            const int n = u * 16 + (lane & 15);
            const float gt = rbf(acc[0][mt][r]);
            const float up = rbf(acc[1][mt][r]);
            a.out[(size_t)m * a.ldo + n] = f2bf(rbf(silu_f(gt)) * up);
          } else if constexpr (EPI == EPI_LOGITS) {
            const int n = u * 16 + (lane & 15);
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
    for (int mt = 0; mt < MT; ++mt)
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
    int* ri = (int*)(red + 4 * MT * 16);
    __syncthreads();
    if (kpart == 0 && (lane & 15) == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = mt * 16 + 4 * (lane >> 4) + r;
          rv[ugrp * MT * 16 + m] = best_v[mt][r];
          ri[ugrp * MT * 16 + m] = best_i[mt][r];
        }
    }
    __syncthreads();
    for (int m = threadIdx.x; m < M; m += WG_THREADS) {
      float v = rv[m];
      int i = ri[m];
      for (int g = 1; g < UPW; ++g) argmax_merge(v, i, rv[g * MT * 16 + m], ri[g * MT * 16 + m]);
      a.part_val[(size_t)m * a.part_stride + blockIdx.x] = v;
      a.part_idx[(size_t)m * a.part_stride + blockIdx.x] = i;
    }
  }
}

// ---------------------------------------------------------------- host dispatch -------
template <int MT, int NG, int KSPLIT, bool A_LDS, bool NORM, int EPI>
static void launch_one(const WgemmArgs& a, int grid, hipStream_t s) {
  size_t lds = A_LDS ? (((size_t)a.M * (a.K + 8) * 2 + 15) & ~(size_t)15) : 0;
  lds += (size_t)(4 * NG * MT * 4 * 64 + 64) * sizeof(float);
  hipLaunchKernelGGL((wgemm_kernel<MT, NG, KSPLIT, A_LDS, NORM, EPI>), dim3(grid),
                     dim3(WG_THREADS), lds, s, a);
}

template <int MT, int NG, bool A_LDS, bool NORM, int EPI>
static void launch_ks(const WgemmArgs& a, int ksplit, int grid, hipStream_t s) {
  if (ksplit == 4) launch_one<MT, NG, 4, A_LDS, NORM, EPI>(a, grid, s);
  else if (ksplit == 2) launch_one<MT, NG, 2, A_LDS, NORM, EPI>(a, grid, s);
  else launch_one<MT, NG, 1, A_LDS, NORM, EPI>(a, grid, s);
}

template <int NG, bool A_LDS, bool NORM, int EPI>
static void launch_mt(const WgemmArgs& a, int mt, int ksplit, int grid, hipStream_t s) {
  switch (mt) {
    case 1: launch_ks<1, NG, A_LDS, NORM, EPI>(a, ksplit, grid, s); break;
    case 2: launch_ks<2, NG, A_LDS, NORM, EPI>(a, ksplit, grid, s); break;
    case 3: launch_ks<3, NG, A_LDS, NORM, EPI>(a, ksplit, grid, s); break;
    default: launch_ks<4, NG, A_LDS, NORM, EPI>(a, ksplit, grid, s); break;
  }
}

// Picks split-K and grid so that small-N projections still cover the 256 CUs and
// large-N ones (lm_head, MLP) stream whole n-tiles per wave.
WgemmPlan plan_wgemm(int M, int N, int K, int epi, int num_cu) {
  WgemmPlan p;
  const int NG = (epi == EPI_SWIGLU) ? 2 : 1;
  const int units = (N / 16) / NG;
  const int KT = K / 32;
  p.a_lds = ((size_t)M * (K + 8) * 2) <= 80 * 1024;
  int ks = 1;
  // enough units for every wave of every CU to own whole tiles? else split K in-workgroup
  if (units < num_cu * 4) ks = 2;
  if (units < num_cu * 2) ks = 4;
  while (ks > 1 && (KT % (ks * KU)) != 0) ks >>= 1;
  p.ksplit = ks;
  const int upw = 4 / ks;
  int grid = (units + upw - 1) / upw;
  const int cap = (epi == EPI_LOGITS) ? LOGITS_MAX_PARTS : num_cu * 8;
  if (grid > cap) grid = cap;
  p.grid = grid;
  return p;
}

bool wgemm_supported(int M, int N, int K, int epi) {
  const int NG = (epi == EPI_SWIGLU) ? 2 : 1;
  return M >= 1 && M <= 64 && (N % (16 * NG)) == 0 && (K % (32 * KU)) == 0;
}

void launch_wgemm(const WgemmArgs& a, const WgemmPlan& p, int epi, bool norm, hipStream_t s) {
  const int mt = (a.M + 15) / 16;
  const bool lds = p.a_lds;
#define TTS_DISPATCH(NGV, EPIV)                                                        \
  do {                                                                                 \
    if (lds) {                                                                         \
      if (norm) launch_mt<NGV, true, true, EPIV>(a, mt, p.ksplit, p.grid, s);          \
      else launch_mt<NGV, true, false, EPIV>(a, mt, p.ksplit, p.grid, s);              \
    } else {                                                                           \
      launch_mt<NGV, false, false, EPIV>(a, mt, p.ksplit, p.grid, s);                  \
    }                                                                                  \
  } while (0)
  switch (epi) {
    case EPI_STORE: TTS_DISPATCH(1, EPI_STORE); break;
    case EPI_RESID: TTS_DISPATCH(1, EPI_RESID); break;
    case EPI_SWIGLU: TTS_DISPATCH(2, EPI_SWIGLU); break;
    case EPI_LOGITS: TTS_DISPATCH(1, EPI_LOGITS); break;
  }
#undef TTS_DISPATCH
}

}  // namespace tts
