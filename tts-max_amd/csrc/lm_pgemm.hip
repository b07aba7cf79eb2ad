// lm_pgemm.hip — prefill GEMM: out = epi(X[M][K] . W^T) for M >> 64 rows (prompt tokens of
// every sequence of the batch in one launch), bf16 in, fp32 accumulate, bf16 out.
//
// Reference semantics as lm_gemm.hip (transformers LlamaForCausalLM: nn.Linear rounded once
// to bf16; LlamaMLP silu(gate)*up with bf16 rounding per op, modeling_llama.py:163-176;
// decoder residual add rounded to bf16).
//
// MI355X design: the weights stay in the decode stream-plan layout (1 KiB MFMA B-fragment
// tiles, lm_gemm.hip) — the prefill reads the same copy, locating tile (nt, kt) with
// plan_tile().  A workgroup = 4 waves (2 x 2) owns a BM x BN output block; per K step of
// 64 (two k-tiles) the A rows (BM x 64 bf16) and the B tiles (BN/16 x 2 KiB) are staged
// through double-buffered LDS, each wave then runs MW x NW v_mfma_f32_16x16x32_bf16 per
// k-tile from LDS fragments.  The next step's global loads are in flight while the current
// step computes.  Rows beyond M are clamped on load and never stored.
//
// Canonical K chunks (round 6): every output is the sum, in chunk order, of its partial dot
// products over the fixed K chunks [0, 1024), [1024, 2048), ... (each one MFMA accumulation
// chain from zero).  A workgroup either sweeps all of K and keeps the running sum in
// registers (tall batched prefill: plenty of tiles), or takes ONE chunk (grid.y) and writes
// its fp32 partial, summed in the same order by pgemm_combine_kernel (a single prompt: a
// 202-row down projection has 64-224 tiles on 256 CUs and 128 dependent K steps each).  Both
// forms give the same bits, for every M and tile shape, so a prompt's rows are bit-identical
// prefilled alone or in any batch.
//
// Tile order (XCD-grouped, xcd_tile): the ≈64 workgroups resident on one XCD cover a compact
// block of output tiles, so the weight tiles and A rows they share are fetched into that
// XCD's L2 once.  The weight loads use the default cache policy (they are re-read by every
// m-block: MI355X_MICROARCH.md nt-weights, "never on slices that every CU re-reads").
#include "hip_common.h"
#include "lm_kernels.h"

#include <cstdlib>

namespace tts {

namespace {

TTS_DEV bf16x8_t as_bf16x8p(u32x4_t v) { return __builtin_bit_cast(bf16x8_t, v); }

constexpr int PK_KK = 2;                      // k-tiles per K step
constexpr int PK_LDA = PK_KK * 32 + 8;        // LDS row stride of A (bf16): +16 B spreads the rows' banks
constexpr int PK_GM = 8;                      // m-blocks per tile group of the XCD-grouped order
constexpr int PK_KCH = 1024;                  // canonical K chunk (elements)
constexpr int PK_CS = PK_KCH / (PK_KK * 32);  // K steps per chunk
constexpr int PK_PART = 99;                   // "epilogue" of the one-chunk form: fp32 partials

// XCD-grouped tile order (a.xcd_order): the dispatcher places workgroup b on XCD b % 8 (round
// robin; speed only, never correctness), so XCD x's workgroups are b = x, x + 8, ...  XCD x owns
// the n-blocks [x*nb/8, (x+1)*nb/8) and walks them in groups of PK_GM m-blocks, m fastest: the
// workgroups resident on one XCD at a time form a compact block of output tiles, whose A rows
// and weight tiles are fetched into that XCD's L2 once and re-read from there (the plain
// order put consecutive m-blocks on different XCDs: every XCD fetched every weight tile and A
// row block for itself).  mb < 0: no tile (the XCD's share is smaller than the grid's)
TTS_DEV void xcd_tile(int b, int mblocks, int nblocks, int& mb, int& nb) {
  const int x = b & 7, l = b >> 3;
  const int nlo = x * nblocks / 8, nn = (x + 1) * nblocks / 8 - nlo;
  if (l >= mblocks * nn) { mb = -1; nb = 0; return; }
  const int grp = l / (PK_GM * nn), m0 = grp * PK_GM, gm = min(PK_GM, mblocks - m0);
  const int li = l - grp * PK_GM * nn;
  mb = m0 + li % gm;
  nb = nlo + li / gm;
}

// The epilogue's arithmetic on a finished fp32 sum (shared by the GEMM and the combine, so
// both forms round identically)
TTS_DEV bf16_t swiglu_out(float gate, float up) { return f2bf(rbf(silu_f(rbf(gate))) * rbf(up)); }
TTS_DEV bf16_t resid_out(bf16_t r, float s) { return f2bf(bf2f(r) + rbf(s)); }

// EPI: EPI_STORE / EPI_RESID / EPI_SWIGLU, or PK_PART (one chunk = blockIdx.y, fp32 partial
// to a.part[chunk][M][N] in the GEMM's own column order)
template <int MW, int NW, int EPI, bool DEEP = (MW <= 2)>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void pgemm_kernel(PgemmArgs a) {
  constexpr bool SPLIT = EPI == PK_PART;
  constexpr int BM = 2 * MW * 16, BN = 2 * NW * 16;
  constexpr int NTB = BN / 16;                     // n-tiles per workgroup
  constexpr int ACH = BM * PK_KK * 4 / 256;        // A 16-B chunks per thread per step
  constexpr int BCH = NTB * PK_KK * 64 / 256;      // B 16-B chunks per thread per step
  static_assert(ACH >= 1 && BCH >= 1, "tile too small for 256 threads");
  __shared__ bf16_t As[2][BM * PK_LDA];
  __shared__ u32x4_t Bs[2][NTB * PK_KK * 64];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int mblocks = (a.M + BM - 1) / BM;
  int mb, nbk;
  if (a.xcd_order) {
    xcd_tile((int)blockIdx.x, mblocks, a.N / BN, mb, nbk);
    if (mb < 0) return;
  } else {
    mb = blockIdx.x % mblocks;
    nbk = blockIdx.x / mblocks;
  }
  const int m0 = mb * BM, nt0 = nbk * NTB;
  const int KT = a.K >> 5, steps = KT / PK_KK;
  // this workgroup's K steps: all of K, or one canonical chunk
  const int s_lo = SPLIT ? (int)blockIdx.y * PK_CS : 0;
  const int s_hi = SPLIT ? min(steps, s_lo + PK_CS) : steps;

  // Two register sets of staged operands: the global loads of step s+2 are issued while
  // step s computes (one step of MFMAs is shorter than an HBM round trip), and unconditional
  // (clamped step index) so the vmcnt waits stay exact.  Requires an even step count (per
  // chunk: K % 128 == 0, PK_CS even).
  u32x4_t ra[DEEP ? 2 : 1][ACH], rb[DEEP ? 2 : 1][BCH];
  auto load = [&](int s, u32x4_t (&xa)[ACH], u32x4_t (&xb)[BCH]) {
    s = min(s, s_hi - 1);
#pragma unroll
    for (int j = 0; j < ACH; ++j) {
      const int c = tid + j * 256, row = c / (PK_KK * 4), col = (c % (PK_KK * 4)) * 8;
      const int m = min(m0 + row, a.M - 1);
      xa[j] = *(const u32x4_t*)(a.x + (size_t)m * a.ldx + s * PK_KK * 32 + col);
    }
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      const int c = tid + j * 256, t = c >> 6, ln = c & 63;
      const int ntl = t / PK_KK, ktl = t % PK_KK;
      const long long tile =
          plan_tile(a.ng, a.ksplit, a.ku, a.ur, a.units, KT, a.kc, nt0 + ntl, s * PK_KK + ktl);
      xb[j] = *((const u32x4_t*)a.w + tile * 64 + ln);
    }
  };
  auto stash = [&](int buf, const u32x4_t (&xa)[ACH], const u32x4_t (&xb)[BCH]) {
#pragma unroll
    for (int j = 0; j < ACH; ++j) {
      const int c = tid + j * 256, row = c / (PK_KK * 4), col = (c % (PK_KK * 4)) * 8;
      *(u32x4_t*)(&As[buf][row * PK_LDA + col]) = xa[j];
    }
#pragma unroll
    for (int j = 0; j < BCH; ++j) Bs[buf][tid + j * 256] = xb[j];
  };

  f32x4_t acc[MW][NW];
  // running sum over the finished chunks: from +0, which adds exactly (a chain that starts at
  // +0 never ends at -0), so it equals the combine's part[0] + part[1] + ...
  f32x4_t tot[SPLIT ? 1 : MW][SPLIT ? 1 : NW];
#pragma unroll
  for (int i = 0; i < MW; ++i)
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      if constexpr (!SPLIT) tot[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }

  auto compute = [&](int buf) {
#pragma unroll
    for (int ktl = 0; ktl < PK_KK; ++ktl) {
      bf16x8_t bf[NW];
#pragma unroll
      for (int j = 0; j < NW; ++j) bf[j] = as_bf16x8p(Bs[buf][((wn * NW + j) * PK_KK + ktl) * 64 + lane]);
#pragma unroll
      for (int i = 0; i < MW; ++i) {
        const int row = (wm * MW + i) * 16 + (lane & 15);
        const bf16x8_t af =
            as_bf16x8p(*(const u32x4_t*)(&As[buf][row * PK_LDA + ktl * 32 + 8 * (lane >> 4)]));
#pragma unroll
        for (int j = 0; j < NW; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[j], acc[i][j], 0, 0, 0);
      }
    }
  };
  // end of a chunk (all-of-K form): fold its partial into the running sum, restart from zero
  auto fold = [&]() {
    if constexpr (!SPLIT) {
#pragma unroll
      for (int i = 0; i < MW; ++i)
#pragma unroll
        for (int j = 0; j < NW; ++j) {
          tot[i][j] += acc[i][j];
          acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        }
    }
  };

  if constexpr (!DEEP) {  // tall blocks: one step ahead (the second set would cost occupancy)
    load(s_lo, ra[0], rb[0]);
    stash(0, ra[0], rb[0]);
    __syncthreads();
    for (int c0 = s_lo; c0 < s_hi; c0 += PK_CS) {  // chunk by chunk
      const int c1 = min(c0 + PK_CS, s_hi);
#pragma nounroll
      for (int s = c0; s < c1; ++s) {
        const int buf = (s - s_lo) & 1;
        if (s + 1 < s_hi) load(s + 1, ra[0], rb[0]);
        compute(buf);
        if (s + 1 < s_hi) stash(buf ^ 1, ra[0], rb[0]);
        __syncthreads();
      }
      fold();
    }
  } else {
    load(s_lo, ra[0], rb[0]);
    load(s_lo + 1, ra[1], rb[1]);
    stash(0, ra[0], rb[0]);
    __syncthreads();
    load(s_lo + 2, ra[0], rb[0]);
    for (int s = s_lo; s < s_hi; s += 2) {
      compute(0);                    // step s (buffer 0); set 1 holds step s+1, set 0 step s+2
      stash(1, ra[1], rb[1]);
      __syncthreads();
      load(s + 3, ra[1], rb[1]);
      compute(1);                    // step s+1
      stash(0, ra[0], rb[0]);        // (after the last step: a clamped duplicate, never used)
      __syncthreads();
      load(s + 4, ra[0], rb[0]);
      if (!SPLIT && ((s + 2) % PK_CS == 0 || s + 2 == s_hi)) fold();
    }
  }

  // ---- epilogue: lane owns column (lane & 15) of each n-tile, rows 4*(lane>>4) + r
#pragma unroll
  for (int i = 0; i < MW; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + (wm * MW + i) * 16 + 4 * (lane >> 4) + r;
      if (m >= a.M) continue;
      if constexpr (SPLIT) {
        float* pr = a.part + ((size_t)blockIdx.y * a.M + m) * a.N;
#pragma unroll
        for (int j = 0; j < NW; ++j) pr[(nt0 + wn * NW + j) * 16 + (lane & 15)] = acc[i][j][r];
      } else if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
        for (int j = 0; j < NW; j += 2) {  // n-tiles (2u, 2u+1) = (gate, up) of unit u
          const int u = (nt0 + wn * NW + j) >> 1;
          a.out[(size_t)m * a.ldo + u * 16 + (lane & 15)] = swiglu_out(tot[i][j][r], tot[i][j + 1][r]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < NW; ++j) {
          const int n = (nt0 + wn * NW + j) * 16 + (lane & 15);
          if constexpr (EPI == EPI_RESID) {
            bf16_t* p = a.resid + (size_t)m * a.ldo + n;
            *p = resid_out(*p, tot[i][j][r]);
          } else {
            a.out[(size_t)m * a.ldo + n] = f2bf(tot[i][j][r]);
          }
        }
      }
    }
  }
}

// The one-chunk form's sum: out = epi(part[0] + part[1] + ... in chunk order), 4 output
// columns per thread.  SwiGLU: output column u*16 + c takes GEMM columns (2u)*16 + c (gate)
// and (2u+1)*16 + c (up), as the GEMM epilogue does.
template <int EPI>
__global__ __launch_bounds__(256) void pgemm_combine_kernel(PgemmArgs a, int nch) {
  const int NO = EPI == EPI_SWIGLU ? a.N / 2 : a.N, q = NO / 4;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)a.M * q) return;
  const int m = (int)(i / q), o = (int)(i % q) * 4;
  const size_t cs = (size_t)a.M * a.N;
  const float* pr = a.part + (size_t)m * a.N;
  if constexpr (EPI == EPI_SWIGLU) {
    const int gc = (o >> 4) * 32 + (o & 15);
    f32x4_t g = *(const f32x4_t*)(pr + gc), u = *(const f32x4_t*)(pr + gc + 16);
    for (int c = 1; c < nch; ++c) {
      g += *(const f32x4_t*)(pr + c * cs + gc);
      u += *(const f32x4_t*)(pr + c * cs + gc + 16);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) a.out[(size_t)m * a.ldo + o + t] = swiglu_out(g[t], u[t]);
  } else {
    f32x4_t sum = *(const f32x4_t*)(pr + o);
    for (int c = 1; c < nch; ++c) sum += *(const f32x4_t*)(pr + c * cs + o);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if constexpr (EPI == EPI_RESID) {
        bf16_t* p = a.resid + (size_t)m * a.ldo + o + t;
        *p = resid_out(*p, sum[t]);
      } else {
        a.out[(size_t)m * a.ldo + o + t] = f2bf(sum[t]);
      }
    }
  }
}

int pk_chunks(int K) { return (K + PK_KCH - 1) / PK_KCH; }

template <int MW, int NW>
int pk_tiles(const PgemmArgs& a) {
  constexpr int BM = 2 * MW * 16, BN = 2 * NW * 16;
  return ((a.M + BM - 1) / BM) * (a.N / BN);
}

template <int MW, int NW>
bool launch_pgemm_mn(const PgemmArgs& a, int epi, bool split, hipStream_t s) {
  constexpr int BM = 2 * MW * 16, BN = 2 * NW * 16;
  const int mblocks = (a.M + BM - 1) / BM, nblocks = a.N / BN;
  // (XCD-grouped order: 8 x the largest per-XCD share; the plain order: one per tile)
  const int gx = a.xcd_order ? 8 * mblocks * ((nblocks + 7) / 8) : mblocks * nblocks;
  if (split) {
    const int nch = pk_chunks(a.K);
    hipLaunchKernelGGL((pgemm_kernel<MW, NW, PK_PART>), dim3(gx, nch), dim3(256), 0, s, a);
    if (epi == EPI_RESID && a.next_norm && a.N <= 8192) {
      // the decode path's combine + next RMSNorm (one workgroup per row, chunks summed in order,
      // the canonical norm): the consumer GEMM then reads xn instead of a standalone norm pass
      launch_splitk_combine_norm(a.part, nch, a.M, a.N, a.N, a.resid, a.ldo, a.next_norm, a.eps, a.xn, a.N, s);
      return true;
    }
    const long long n4 = (long long)a.M * ((epi == EPI_SWIGLU ? a.N / 2 : a.N) / 4);
    const dim3 cg((unsigned)((n4 + 255) / 256));
    switch (epi) {
      case EPI_STORE: hipLaunchKernelGGL((pgemm_combine_kernel<EPI_STORE>), cg, dim3(256), 0, s, a, nch); break;
      case EPI_RESID: hipLaunchKernelGGL((pgemm_combine_kernel<EPI_RESID>), cg, dim3(256), 0, s, a, nch); break;
      case EPI_SWIGLU: hipLaunchKernelGGL((pgemm_combine_kernel<EPI_SWIGLU>), cg, dim3(256), 0, s, a, nch); break;
    }
    return false;
  }
  switch (epi) {
    case EPI_STORE: hipLaunchKernelGGL((pgemm_kernel<MW, NW, EPI_STORE>), dim3(gx), dim3(256), 0, s, a); break;
    case EPI_RESID: hipLaunchKernelGGL((pgemm_kernel<MW, NW, EPI_RESID>), dim3(gx), dim3(256), 0, s, a); break;
    case EPI_SWIGLU: hipLaunchKernelGGL((pgemm_kernel<MW, NW, EPI_SWIGLU>), dim3(gx), dim3(256), 0, s, a); break;
  }
  return false;
}

}  // namespace

bool pgemm_supported(int M, int N, int K, int epi) {
  return M >= 1 && (N % 64) == 0 && (K % (2 * PK_KK * 32)) == 0 &&  // (an even step count)
         (epi == EPI_STORE || epi == EPI_RESID || epi == EPI_SWIGLU);
}

size_t pgemm_part_bytes(int M, int N, int K) { return (size_t)pk_chunks(K) * M * N * 4; }

bool launch_pgemm(const PgemmArgs& a_in, int epi, int num_cu, hipStream_t s) {
  PgemmArgs a = a_in;
  // A/B switches (bit-identical either way): TTS_PGEMM_XCD=0 plain tile order (202-row prompt
  // 2.31 -> 2.46 ms, 32 prompts 20.8 -> 22.1 ms); TTS_PGEMM_SPLIT=0 never one chunk per
  // workgroup (2.31 -> 2.79 ms), =1 also for the SwiGLU gate/up, whose 512 tiles already cover
  // the CUs (2.19 -> 2.31 ms: the partials cost more than the shorter chains save;
  // profiles/r6i_prefill_ab.txt)
  static const bool xcd_env = !getenv("TTS_PGEMM_XCD") || atoi(getenv("TTS_PGEMM_XCD"));
  static const int split_env = getenv("TTS_PGEMM_SPLIT") ? atoi(getenv("TTS_PGEMM_SPLIT")) : 2;
  a.xcd_order = xcd_env;
  const StreamPlan sp = stream_plan(a.N, a.K, epi == EPI_SWIGLU ? 2 : 1, num_cu);
  a.ng = sp.ng; a.ksplit = sp.ksplit; a.ku = sp.ku; a.ur = sp.ur(); a.kc = sp.kc;
  a.units = (a.N / 16) / sp.ng;
  const bool wide = (a.N % 128) == 0;
  // 64-row blocks while that still leaves > 2 blocks per CU's worth of weight re-reads
  // unneeded (short prompts), 128-row blocks for long batched prefill
  const bool tall = a.M > 512;
  if (wide && tall) return launch_pgemm_mn<4, 4>(a, epi, false, s);
  if (tall) return launch_pgemm_mn<4, 2>(a, epi, false, s);
  // short prompts: too few tiles for the CUs, each a long chain of dependent K steps — one
  // canonical K chunk per workgroup (same bits) on the largest tile that then covers the CUs
  const int nch = pk_chunks(a.K);
  const bool split = split_env > 0 && nch > 1 && a.part && pgemm_part_bytes(a.M, a.N, a.K) <= a.part_bytes &&
                     (epi != EPI_SWIGLU || split_env == 1);
  if (split) {
    if (wide && pk_tiles<2, 4>(a) * nch >= num_cu) return launch_pgemm_mn<2, 4>(a, epi, true, s);
    if (pk_tiles<2, 2>(a) * nch >= num_cu) return launch_pgemm_mn<2, 2>(a, epi, true, s);
    if (pk_tiles<1, 2>(a) * nch >= num_cu || epi == EPI_SWIGLU) return launch_pgemm_mn<1, 2>(a, epi, true, s);
    return launch_pgemm_mn<1, 1>(a, epi, true, s);
  }
  // smaller blocks until the grid covers the CUs (a single prompt's QKV / o_proj / down gave
  // 64-96 workgroups)
  if (wide && pk_tiles<2, 4>(a) >= num_cu) return launch_pgemm_mn<2, 4>(a, epi, false, s);
  if (pk_tiles<2, 2>(a) >= num_cu) return launch_pgemm_mn<2, 2>(a, epi, false, s);
  if (pk_tiles<1, 2>(a) >= num_cu / 2 || epi == EPI_SWIGLU) return launch_pgemm_mn<1, 2>(a, epi, false, s);  // (SwiGLU: n-tile pairs)
  return launch_pgemm_mn<1, 1>(a, epi, false, s);
}

}  // namespace tts
