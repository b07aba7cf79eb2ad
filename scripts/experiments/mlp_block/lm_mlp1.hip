// lm_mlp1.hip — the MLP half of a one-row decode layer as ONE launch (TTS-1 geometry:
// hidden 2048, ffn 8192, 256 CUs).  Reference semantics: LlamaMLP + the residual add of
// LlamaDecoderLayer (transformers modeling_llama.py:150-165, 318-322), as the launch path's
// gate/up (EPI_SWIGLU) + down (EPI_RESID) pair computes it: h = the residual stream after
// attention (row 0 of x), RMSNorm(h, ln2) in bf16, gate / up rounded to bf16, act =
// SiLU(gate) * up in bf16, x = h + down(act) (down rounded to bf16, bf16 add).
//
// Why one launch: as two launches the down projection starts cold after a launch boundary
// (9.1 us for 33.5 MB at one row, 3.7 TB/s).  Here workgroup c (one per CU, 8 waves):
//   * issues, at once, the loads of its gate/up rows (256 KiB: act outputs 32c .. 32c+31) into
//     registers and the LDS-DMA of its down K-slice (the 2048 x 32 columns that multiply those
//     same act values: 128 KiB) into LDS — the down weights stream in while gate/up computes;
//   * multiplies its own act slice into a 2048-wide fp32 partial, published as 8-byte
//     {payload, tag} granules (tag = position << 6 | layer) in owner-major order, so that the
//     owner of outputs 8c .. 8c+7 reads one contiguous 16 KiB run that nobody else reads (an
//     all-gather of act instead would have every CU read the same 32 KiB: a hot spot of a few
//     memory channels, ~10 us);
//   * wave w sums output 8c + w over the 256 producers in a fixed order and writes x = h +
//     down over h.
// Writing x over h in place is safe: an owner writes only after every CU published its
// partial, and every CU read all of h before that.
#include <stdexcept>

#include "hip_common.h"
#include "lm_kernels.h"

namespace tts {

namespace {

constexpr int NCU = 256, NW = 8, HID = 2048, FFN = 8192;
constexpr int GU_GROUP = 4 * HID * 2;               // 4 rows (gate 2j, 2j+1, up 2j, 2j+1): 16 KiB
constexpr int GU_BYTES = NW * 2 * GU_GROUP;          // per CU: 16 groups = 256 KiB
constexpr int D_BYTES = HID * 32 * 2;                // per CU: K-slice 32c .. 32c+31 of all 2048 rows
constexpr size_t PER_CU = (size_t)GU_BYTES + D_BYTES;
constexpr int L_ACT = D_BYTES;                       // LDS: down K-slice [4][2048][8], then act [32]
constexpr int LDS_BYTES = D_BYTES + 64;
constexpr int MAX_SPINS = 1 << 18;

typedef __attribute__((address_space(1))) uint64_t g64;
typedef __attribute__((address_space(1))) int gint;
TTS_DEV uint64_t gld(const uint64_t* p) { return __hip_atomic_load((const g64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
TTS_DEV void gst(uint64_t* p, uint32_t payload, uint32_t tag) {
  __hip_atomic_store((g64*)p, ((uint64_t)tag << 32) | payload, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

TTS_DEV float dot8(u32x4_t a, u32x4_t b, float acc) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    // element copies first: __builtin_bit_cast of a vector subscript reads element 0
    const uint32_t aq = a[q], bq = b[q];
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_cvt_t, aq), __builtin_bit_cast(bf16x2_cvt_t, bq), acc,
                                          false);
  }
  return acc;
}

}  // namespace

__global__ __launch_bounds__(NW * 64) void mlp1_kernel(Mlp1Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const char* wb = (const char*)a.w + ((size_t)a.layer * NCU + c) * PER_CU;

  // 1. loads, in the order they are needed: h and ln2 (this lane's k = 8 lane + 512 j), the
  //    wave's two gate/up groups, then its 16 KiB of the down rows by LDS-DMA
  u32x4_t xh[4], g[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    xh[j] = *(const u32x4_t*)(a.x + 8 * lane + 512 * j);
    g[j] = *(const u32x4_t*)(a.ln2 + 8 * lane + 512 * j);
  }
  u32x4_t wv[2][4][4] = {};
  if (!(a.dbg & 2))
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        wv[i][r][j] = __builtin_nontemporal_load(
            (const u32x4_t*)(wb + (size_t)(2 * w + i) * GU_GROUP + r * HID * 2 + j * 1024 + lane * 16));
  if (!(a.dbg & 1))
#pragma unroll
  for (int p = 0; p < D_BYTES / 1024 / NW; ++p) {
    const int chunk = (D_BYTES / 1024 / NW) * w + p;
    __builtin_amdgcn_global_load_lds((gptr_t)(wb + GU_BYTES + (size_t)chunk * 1024 + lane * 16),
                                     (lptr_t)(smem + chunk * 1024 + lane * 16), 16, 0, 2 /* nt */);
  }

  // 2. RMSNorm(h, ln2): fp32 mean of squares in the canonical order, x * r rounded to bf16,
  //    times the weight rounded to bf16
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) ss += wave_sum_dpp(chunk_sumsq(xh[j]));
  const float rr = 1.0f / sqrtf(ss / (float)HID + a.eps);
  u32x4_t xn[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      xn[j][q] = pack_bf2(rbf(bf_lo(g[j][q]) * rbf(bf_lo(xh[j][q]) * rr)), rbf(bf_hi(g[j][q]) * rbf(bf_hi(xh[j][q]) * rr)));

  // 3. gate / up rows -> act 32c + 2(2w + i), +1 into LDS
  bf16_t* act = (bf16_t*)(smem + L_ACT);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float y[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = dot8(wv[i][r][j], xn[j], acc);
      y[r] = wave_sum_dpp(acc);
    }
    if (lane == 0) {
      const float a0 = rbf(rbf(silu_f(rbf(y[0]))) * rbf(y[2])), a1 = rbf(rbf(silu_f(rbf(y[1]))) * rbf(y[3]));
      ((uint32_t*)act)[2 * w + i] = pack_bf2(a0, a1);
    }
  }
  // 4. every wave's act and down K-slice are in LDS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // 5. partial down over this CU's K-slice: wave w, lane -> outputs n = 256 w + lane + 64 q;
  //    LDS layout [i = k / 8][n][8] (16 consecutive bytes per lane)
  const uint32_t tag = ((uint32_t)a.row_pos[0] << 6) | (uint32_t)a.layer;
  u32x4_t av[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) av[i] = *(const u32x4_t*)(act + 8 * i);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n = 256 * w + lane + 64 * q;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc = dot8(*(const u32x4_t*)(smem + ((size_t)i * HID + n) * 16), av[i], acc);
    gst(a.gran + ((size_t)(n >> 3) * NCU + c) * 8 + (n & 7), __float_as_uint(acc), tag);
  }

  // 6. owner: output 8c + w = the 256 producers' partials (lane: producers 4 lane .. +3),
  //    re-swept together until every tag is this launch's
  const uint64_t* pd = a.gran + (size_t)c * NCU * 8 + w + lane * 32;
  uint64_t gv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) gv[k] = gld(pd + k * 8);
  uint32_t pending = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) pending |= ((uint32_t)(gv[k] >> 32) != tag && !(a.dbg & 4)) ? 1u << k : 0u;
  int spins = 0;
  while (pending) {
    if (++spins > MAX_SPINS) {  // bounded: the host sees err and fails the call
      __hip_atomic_store((gint*)a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (pending & (1u << k)) gv[k] = gld(pd + k * 8);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if ((uint32_t)(gv[k] >> 32) == tag) pending &= ~(1u << k);
  }
  const float d = wave_sum_dpp((__uint_as_float((uint32_t)gv[0]) + __uint_as_float((uint32_t)gv[1])) +
                               (__uint_as_float((uint32_t)gv[2]) + __uint_as_float((uint32_t)gv[3])));
  if (lane == 0) {
    const int n = 8 * c + w;
    a.x[n] = f2bf(bf2f(a.x[n]) + rbf(d));
  }
}

bool mlp1_supported(int hidden, int ffn, int num_cu) { return hidden == HID && ffn == FFN && num_cu == NCU; }
size_t mlp1_weight_bytes(int layers) { return (size_t)layers * NCU * PER_CU; }
size_t mlp1_gran_elems() { return (size_t)HID * NCU; }

void launch_mlp1(const Mlp1Args& a, hipStream_t s) {
  hipLaunchKernelGGL(mlp1_kernel, dim3(NCU), dim3(NW * 64), LDS_BYTES, s, a);
}

// Row-major gate / up [8192][2048] or down [2048][8192] of one layer -> this kernel's layout:
// per CU, 16 gate/up groups of 4 rows (gate 2j, 2j+1, up 2j, 2j+1; j = 16c + group), then
// the down K-slice 32c .. 32c+31 of every row.  kind 0 gate, 1 up, 2 down.  One thread = 16 bytes.
__global__ void mlp1_pack_kernel(const bf16_t* __restrict__ src, char* __restrict__ dst, int kind, int layer) {
  const long long n16 = (long long)FFN * HID / 8;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n16; i += (long long)gridDim.x * blockDim.x) {
    size_t off;
    if (kind == 2) {  // Wd[n][k]: CU k / 32, layout [i = (k % 32) / 8][n][8]
      const int n = (int)(i / (FFN / 8)), k = (int)(i % (FFN / 8)) * 8;
      off = ((size_t)layer * NCU + k / 32) * PER_CU + GU_BYTES + ((size_t)((k % 32) / 8) * HID + n) * 16;
    } else {  // Wg / Wu [row][k]: act pair j = row / 2, CU j / 16, group j % 16
      const int row = (int)(i / (HID / 8)), k = (int)(i % (HID / 8)) * 8;
      const int j = row / 2, r = (kind == 0 ? 0 : 2) + row % 2;
      off = ((size_t)layer * NCU + j / 16) * PER_CU + (size_t)(j % 16) * GU_GROUP + (size_t)r * HID * 2 +
            (size_t)k * 2;
    }
    *(u32x4_t*)(dst + off) = *(const u32x4_t*)(src + i * 8);
  }
}

void launch_mlp1_pack(const bf16_t* w, void* dst, int kind, int layer, hipStream_t s) {
  hipLaunchKernelGGL(mlp1_pack_kernel, dim3(4096), dim3(256), 0, s, w, (char*)dst, kind, layer);
}

}  // namespace tts
