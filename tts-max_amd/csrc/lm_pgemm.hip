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
// step computes.  Rows beyond M are clamped on load and never stored.  Workgroups are
// ordered m-block fastest so the ones sharing a weight block run together (L2 / MALL reuse).
#include "hip_common.h"
#include "lm_kernels.h"

namespace tts {

namespace {

TTS_DEV bf16x8_t as_bf16x8p(u32x4_t v) { return __builtin_bit_cast(bf16x8_t, v); }

constexpr int PK_KK = 2;                // k-tiles per K step
constexpr int PK_LDA = PK_KK * 32 + 8;  // LDS row stride of A (bf16): +16 B spreads the rows' banks

template <int MW, int NW, int EPI, bool DEEP = (MW <= 2)>
__global__ __launch_bounds__(256) void pgemm_kernel(PgemmArgs a) {
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
  const int mb = blockIdx.x % mblocks, nbk = blockIdx.x / mblocks;
  const int m0 = mb * BM, nt0 = nbk * NTB;
  const int KT = a.K >> 5, steps = KT / PK_KK;

  // Two register sets of staged operands: the global loads of step s+2 are issued while
  // step s computes (one step of MFMAs is shorter than an HBM round trip), and unconditional
  // (clamped step index) so the vmcnt waits stay exact.  Requires an even step count.
  u32x4_t ra[DEEP ? 2 : 1][ACH], rb[DEEP ? 2 : 1][BCH];
  auto load = [&](int s, u32x4_t (&xa)[ACH], u32x4_t (&xb)[BCH]) {
    s = min(s, steps - 1);
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
      xb[j] = __builtin_nontemporal_load((const u32x4_t*)a.w + tile * 64 + ln);
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
#pragma unroll
  for (int i = 0; i < MW; ++i)
#pragma unroll
    for (int j = 0; j < NW; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

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

  if constexpr (!DEEP) {  // tall blocks: one step ahead (the second set would cost occupancy)
    load(0, ra[0], rb[0]);
    stash(0, ra[0], rb[0]);
    __syncthreads();
    for (int s = 0; s < steps; ++s) {
      const int buf = s & 1;
      if (s + 1 < steps) load(s + 1, ra[0], rb[0]);
      compute(buf);
      if (s + 1 < steps) stash(buf ^ 1, ra[0], rb[0]);
      __syncthreads();
    }
  } else {
  load(0, ra[0], rb[0]);
  load(1, ra[1], rb[1]);
  stash(0, ra[0], rb[0]);
  __syncthreads();
  load(2, ra[0], rb[0]);
  for (int s = 0; s < steps; s += 2) {
    compute(0);                    // step s (buffer 0); set 1 holds step s+1, set 0 step s+2
    stash(1, ra[1], rb[1]);
    __syncthreads();
    load(s + 3, ra[1], rb[1]);
    compute(1);                    // step s+1
    stash(0, ra[0], rb[0]);        // (after the last step: a clamped duplicate, never used)
    __syncthreads();
    load(s + 4, ra[0], rb[0]);
  }
  }

  // ---- epilogue: lane owns column (lane & 15) of each n-tile, rows 4*(lane>>4) + r
#pragma unroll
  for (int i = 0; i < MW; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + (wm * MW + i) * 16 + 4 * (lane >> 4) + r;
      if (m >= a.M) continue;
      if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
        for (int j = 0; j < NW; j += 2) {  // n-tiles (2u, 2u+1) = (gate, up) of unit u
          const int u = (nt0 + wn * NW + j) >> 1;
          const float gt = rbf(acc[i][j][r]), up = rbf(acc[i][j + 1][r]);
          a.out[(size_t)m * a.ldo + u * 16 + (lane & 15)] = f2bf(rbf(silu_f(gt)) * up);
        }
      } else {
#pragma unroll
        for (int j = 0; j < NW; ++j) {
          const int n = (nt0 + wn * NW + j) * 16 + (lane & 15);
          if constexpr (EPI == EPI_RESID) {
            bf16_t* p = a.resid + (size_t)m * a.ldo + n;
            *p = f2bf(bf2f(*p) + rbf(acc[i][j][r]));
          } else {
            a.out[(size_t)m * a.ldo + n] = f2bf(acc[i][j][r]);
          }
        }
      }
    }
  }
}

template <int MW, int NW>
void launch_pgemm_mn(const PgemmArgs& a, int epi, hipStream_t s) {
  constexpr int BM = 2 * MW * 16, BN = 2 * NW * 16;
  const dim3 grid(((a.M + BM - 1) / BM) * (a.N / BN));
  switch (epi) {
    case EPI_STORE: hipLaunchKernelGGL((pgemm_kernel<MW, NW, EPI_STORE>), grid, dim3(256), 0, s, a); break;
    case EPI_RESID: hipLaunchKernelGGL((pgemm_kernel<MW, NW, EPI_RESID>), grid, dim3(256), 0, s, a); break;
    case EPI_SWIGLU: hipLaunchKernelGGL((pgemm_kernel<MW, NW, EPI_SWIGLU>), grid, dim3(256), 0, s, a); break;
  }
}

}  // namespace

bool pgemm_supported(int M, int N, int K, int epi) {
  return M >= 1 && (N % 64) == 0 && (K % (2 * PK_KK * 32)) == 0 &&  // (an even step count)
         (epi == EPI_STORE || epi == EPI_RESID || epi == EPI_SWIGLU);
}

void launch_pgemm(const PgemmArgs& a_in, int epi, int num_cu, hipStream_t s) {
  PgemmArgs a = a_in;
  const StreamPlan sp = stream_plan(a.N, a.K, epi == EPI_SWIGLU ? 2 : 1, num_cu);
  a.ng = sp.ng; a.ksplit = sp.ksplit; a.ku = sp.ku; a.ur = sp.ur(); a.kc = sp.kc;
  a.units = (a.N / 16) / sp.ng;
  const bool wide = (a.N % 128) == 0;
  // 64-row blocks while that still leaves > 2 blocks per CU's worth of weight re-reads
  // unneeded (short prompts), 128-row blocks for long batched prefill
  const bool tall = a.M > 512;
  auto grid = [&](int bm, int bn) { return ((a.M + bm - 1) / bm) * (a.N / bn); };
  if (wide && tall) launch_pgemm_mn<4, 4>(a, epi, s);
  else if (wide && grid(64, 128) >= num_cu) launch_pgemm_mn<2, 4>(a, epi, s);
  else if (tall) launch_pgemm_mn<4, 2>(a, epi, s);
  // short prompts: smaller blocks until the grid covers the CUs (a single prompt's QKV /
  // o_proj / down gave 64-96 workgroups).  The block shape never changes an output's
  // k-order (one MFMA accumulation chain over K), so rows stay bit-identical across shapes
  else if (grid(64, 64) >= num_cu) launch_pgemm_mn<2, 2>(a, epi, s);
  else if (grid(32, 64) >= num_cu / 2 || epi == EPI_SWIGLU) launch_pgemm_mn<1, 2>(a, epi, s);  // (SwiGLU: n-tile pairs)
  else launch_pgemm_mn<1, 1>(a, epi, s);
}

}  // namespace tts
