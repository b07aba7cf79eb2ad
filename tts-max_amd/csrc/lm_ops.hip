// lm_ops.hip — small SpeechLM kernels: standalone RMSNorm (prefill chunks), token
// embedding gather, row gather, greedy finalize (argmax reduce + per-sequence bookkeeping),
// and the deterministic synthetic-weight generator shared with tts_amd/synth.py.
#include "hip_common.h"
#include "lm_kernels.h"
#include "lm_finalize.h"

namespace tts {

// LlamaRMSNorm (transformers modeling_llama.py:62-67) with bf16 in/out.
__global__ void rmsnorm_kernel(const bf16_t* __restrict__ x, int ldx, const bf16_t* __restrict__ w,
                               float eps, bf16_t* __restrict__ y, int ldy, int K) {
  __shared__ float segs[64];  // 512-value segment sums (K <= 32768)
  const bf16_t* xr = x + (size_t)blockIdx.x * ldx;
  bf16_t* yr = y + (size_t)blockIdx.x * ldy;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int nseg = (K + 511) / 512;
  for (int sg = wave; sg < nseg; sg += nw) {  // canonical order (chunk_sumsq)
    const int k = sg * 512 + lane * 8;
    const float s = wave_sum_dpp(k < K ? chunk_sumsq(*(const u32x4_t*)(xr + k)) : 0.f);
    if (lane == 0) segs[sg] = s;
  }
  __syncthreads();
  float ss = 0.f;
  for (int sg = 0; sg < nseg; ++sg) ss += segs[sg];
  const float r = 1.0f / sqrtf(ss / (float)K + eps);
  for (int k = threadIdx.x * 8; k < K; k += blockDim.x * 8) {
    u32x4_t v = *(const u32x4_t*)(xr + k);
    const u32x4_t g = *(const u32x4_t*)(w + k);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[q] = pack_bf2(bf_lo(g[q]) * rbf(bf_lo(v[q]) * r), bf_hi(g[q]) * rbf(bf_hi(v[q]) * r));
    *(u32x4_t*)(yr + k) = v;
  }
}

// The same normalisation with the row and the weight loaded once, both issued at entry
// (K <= 256 * 8 * RJ): one memory round trip instead of two.  Chunk c = tid + 256 j lands in
// 512-value segment c / 64 on wave (c / 64) % 4 exactly as above: identical sums and bits.
template <int RJ>
__global__ __launch_bounds__(256) void rmsnorm_reg_kernel(const bf16_t* __restrict__ x, int ldx,
                                                          const bf16_t* __restrict__ w, float eps,
                                                          bf16_t* __restrict__ y, int ldy, int K) {
  __shared__ float segs[64];
  const bf16_t* xr = x + (size_t)blockIdx.x * ldx;
  bf16_t* yr = y + (size_t)blockIdx.x * ldy;
  const int tid = threadIdx.x, lane = tid & 63;
  const int nch = K / 8;
  u32x4_t v[RJ], g[RJ];
#pragma unroll
  for (int j = 0; j < RJ; ++j) {  // unconditional (clamped) loads
    const int c = min(tid + 256 * j, nch - 1);
    v[j] = *(const u32x4_t*)(xr + c * 8);
    g[j] = *(const u32x4_t*)(w + c * 8);
  }
#pragma unroll
  for (int j = 0; j < RJ; ++j) {
    const int c0 = 256 * j + (tid & ~63);  // first chunk of this wave's segment
    if (c0 < nch) {                          // (wave-uniform)
      const float s = wave_sum_dpp(tid + 256 * j < nch ? chunk_sumsq(v[j]) : 0.f);
      if (lane == 0) segs[c0 >> 6] = s;
    }
  }
  __syncthreads();
  const int nseg = (K + 511) / 512;
  float ss = 0.f;
  for (int sg = 0; sg < nseg; ++sg) ss += segs[sg];
  const float r = 1.0f / sqrtf(ss / (float)K + eps);
#pragma unroll
  for (int j = 0; j < RJ; ++j) {
    const int c = tid + 256 * j;
    if (c < nch) {
      u32x4_t o;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        o[q] = pack_bf2(bf_lo(g[j][q]) * rbf(bf_lo(v[j][q]) * r), bf_hi(g[j][q]) * rbf(bf_hi(v[j][q]) * r));
      *(u32x4_t*)(yr + c * 8) = o;
    }
  }
}

void launch_rmsnorm(const bf16_t* x, int ldx, const bf16_t* w, float eps, bf16_t* y, int ldy,
                    int M, int K, hipStream_t s) {
  if (dry_record("rmsnorm")) return;
  if (K % 8 == 0 && K <= 2048)
    hipLaunchKernelGGL((rmsnorm_reg_kernel<1>), dim3(M), dim3(256), 0, s, x, ldx, w, eps, y, ldy, K);
  else if (K % 8 == 0 && K <= 4096)
    hipLaunchKernelGGL((rmsnorm_reg_kernel<2>), dim3(M), dim3(256), 0, s, x, ldx, w, eps, y, ldy, K);
  else if (K % 8 == 0 && K <= 8192)
    hipLaunchKernelGGL((rmsnorm_reg_kernel<4>), dim3(M), dim3(256), 0, s, x, ldx, w, eps, y, ldy, K);
  else
    hipLaunchKernelGGL(rmsnorm_kernel, dim3(M), dim3(256), 0, s, x, ldx, w, eps, y, ldy, K);
}

__global__ void embed_kernel(const int* __restrict__ tokens, const bf16_t* __restrict__ table,
                             bf16_t* __restrict__ x, int hidden) {
  const int t = tokens[blockIdx.x];
  const u32x4_t* src = (const u32x4_t*)(table + (size_t)t * hidden);
  u32x4_t* dst = (u32x4_t*)(x + (size_t)blockIdx.x * hidden);
  for (int i = threadIdx.x; i < hidden / 8; i += blockDim.x) dst[i] = src[i];
}

void launch_embed(const int* tokens, const bf16_t* table, bf16_t* x, int M, int hidden,
                  hipStream_t s) {
  hipLaunchKernelGGL(embed_kernel, dim3(M), dim3(256), 0, s, tokens, table, x, hidden);
}

__global__ void gather_rows_kernel(const bf16_t* __restrict__ x, int ld, const int* __restrict__ rows,
                                   bf16_t* __restrict__ y, int hidden) {
  const u32x4_t* src = (const u32x4_t*)(x + (size_t)rows[blockIdx.x] * ld);
  u32x4_t* dst = (u32x4_t*)(y + (size_t)blockIdx.x * hidden);
  for (int i = threadIdx.x; i < hidden / 8; i += blockDim.x) dst[i] = src[i];
}

void launch_gather_rows(const bf16_t* x, int ld, const int* rows, bf16_t* y, int M, int hidden,
                        hipStream_t s) {
  hipLaunchKernelGGL(gather_rows_kernel, dim3(M), dim3(256), 0, s, x, ld, rows, y, hidden);
}

// --------------------------------------------------------------- greedy finalize -------
// One workgroup per sequence (lm_finalize.h finalize_row).
__global__ void finalize_greedy_kernel(const float* __restrict__ pv, const int* __restrict__ pi,
                                       int part_stride, int nparts, StepState st,
                                       const bf16_t* __restrict__ embed, bf16_t* __restrict__ x,
                                       int hidden) {
  __shared__ int lds[16];
  const int b = blockIdx.x;
  // the step counter (norm-once hand-off tags, WgemmArgs::nw_epoch): +1 per step, every step
  if (b == 0 && threadIdx.x == 0 && st.epoch) __hip_atomic_fetch_add(st.epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  finalize_row<256, false>(pv + (size_t)b * part_stride, pi + (size_t)b * part_stride, nparts, st, b, embed, x,
                           hidden, lds);
}

__global__ void bump_epoch_kernel(uint32_t* epoch) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

void launch_bump_epoch(uint32_t* epoch, hipStream_t s) {
  if (dry_record("bump_epoch_kernel")) return;
  hipLaunchKernelGGL(bump_epoch_kernel, dim3(1), dim3(64), 0, s, epoch);
}

void launch_finalize_greedy(const float* part_val, const int* part_idx, int part_stride,
                            int nparts, StepState st, int B, const bf16_t* embed, bf16_t* x,
                            int hidden, hipStream_t s) {
  if (dry_record("finalize_greedy_kernel")) return;
  hipLaunchKernelGGL(finalize_greedy_kernel, dim3(B), dim3(256), 0, s, part_val, part_idx,
                     part_stride, nparts, st, embed, x, hidden);
}

// --------------------------------------------------------------- synthetic weights -----
// Counter-based generator (splitmix64 of seed + index): value = (2u - 1) * scale with
// u = top 24 bits / 2^24.  Bit-identical to tts_amd/synth.py (numpy), so the GPU box can
// regenerate the exact weights the golden fixtures were produced with.
TTS_DEV float synth_value(unsigned long long seed, unsigned long long idx, float scale) {
  unsigned long long z = seed + (idx + 1ull) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  const float u = (float)(unsigned)(z >> 40) * (1.0f / 16777216.0f);
  const float t = __fsub_rn(__fmul_rn(u, 2.0f), 1.0f);
  return __fmul_rn(t, scale);
}

__global__ void synth_fill_kernel(void* dst, int dtype, long long n, unsigned long long seed,
                                  float scale) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const float v = synth_value(seed, (unsigned long long)i, scale);
    if (dtype == 0) ((float*)dst)[i] = v;
    else ((bf16_t*)dst)[i] = f2bf(v);
  }
}

void launch_synth_fill(void* dst, int dtype, long long n, unsigned long long seed, float scale,
                       hipStream_t s) {
  long long g = (n + 255) / 256;
  int grid = (int)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
  hipLaunchKernelGGL(synth_fill_kernel, dim3(grid), dim3(256), 0, s, dst, dtype, n, seed, scale);
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

// K-sliced GEMM epilogue: the chunk partials of one output element summed in chunk order,
// rounded once to bf16 (as nn.Linear), then stored or added to the residual stream (rounded
// again, modeling_llama.py decoder residual).  8 columns per thread.
__global__ void splitk_combine_kernel(const float* __restrict__ part, int kc, int M, int N, int ldp,
                                      bf16_t* __restrict__ out, bf16_t* __restrict__ resid, int ldo) {
  const int per_row = N / 8;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * per_row) return;
  const int m = i / per_row, n = (i - m * per_row) * 8;
  float v[8];
  {
    const float4* p = (const float4*)(part + (size_t)m * ldp + n);
    const float4 a = p[0], b = p[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  for (int c = 1; c < kc; ++c) {
    const float4* p = (const float4*)(part + ((size_t)c * M + m) * ldp + n);
    const float4 a = p[0], b = p[1];
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
  }
  u32x4_t pk;
  if (resid) {
    bf16_t* r = resid + (size_t)m * ldo + n;
    const u32x4_t old = *(const u32x4_t*)r;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      pk[q] = pack_bf2(bf_lo(old[q]) + rbf(v[2 * q]), bf_hi(old[q]) + rbf(v[2 * q + 1]));
    *(u32x4_t*)r = pk;
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) pk[q] = pack_bf2(v[2 * q], v[2 * q + 1]);
    *(u32x4_t*)(out + (size_t)m * ldo + n) = pk;
  }
}

// The same combine for a residual epilogue, one workgroup per row, followed by the NEXT
// RMSNorm of the updated row (LlamaRMSNorm, canonical sum order of chunk_sumsq): writes the
// residual stream and its normalised copy, so the consumer GEMM stages plain rows.
__global__ __launch_bounds__(256) void splitk_combine_norm_kernel(
    const float* __restrict__ part, int kc, int M, int N, int ldp, bf16_t* __restrict__ resid, int ldo,
    const bf16_t* __restrict__ normw, float eps, bf16_t* __restrict__ xn, int ldn) {
  __shared__ float segs[64];
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nchunk = N / 8;  // 8-column chunks; wave w takes 512-value segments w, w + 4, ...
  bf16_t* r = resid + (size_t)m * ldo;
  constexpr int IT = 4;      // N <= 8192: the updated chunks stay in registers for the norm
  u32x4_t keep[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int base = wave * 64 + it * 256;
    if (base >= nchunk) break;  // wave-uniform: full DPP rows
    const int c = base + lane;
    float s = 0.f;
    if (c < nchunk) {
      const int n = c * 8;
      float v[8];
      {
        const float4* p = (const float4*)(part + (size_t)m * ldp + n);
        const float4 a = p[0], b = p[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      }
      for (int k = 1; k < kc; ++k) {
        const float4* p = (const float4*)(part + ((size_t)k * M + m) * ldp + n);
        const float4 a = p[0], b = p[1];
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
      }
      const u32x4_t old = *(const u32x4_t*)(r + n);
      u32x4_t pk;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        pk[q] = pack_bf2(bf_lo(old[q]) + rbf(v[2 * q]), bf_hi(old[q]) + rbf(v[2 * q + 1]));
      *(u32x4_t*)(r + n) = pk;
      keep[it] = pk;
      s = chunk_sumsq(pk);
    }
    s = wave_sum_dpp(s);
    if (lane == 0) segs[base >> 6] = s;
  }
  __syncthreads();
  float ss = 0.f;
  for (int sg = 0; sg < (nchunk + 63) / 64; ++sg) ss += segs[sg];
  const float rs = 1.0f / sqrtf(ss / (float)N + eps);
#pragma unroll
  for (int it = 0; it < IT; ++it) {  // the chunks this thread wrote
    const int c = wave * 64 + it * 256 + lane;
    if (c >= nchunk) break;
    const int n = c * 8;
    u32x4_t v = keep[it];
    const u32x4_t g = *(const u32x4_t*)(normw + n);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[q] = pack_bf2(bf_lo(g[q]) * rbf(bf_lo(v[q]) * rs), bf_hi(g[q]) * rbf(bf_hi(v[q]) * rs));
    *(u32x4_t*)(xn + (size_t)m * ldn + n) = v;
  }
}

// The same arithmetic with every load in flight at once (the KC chunk partials, the residual
// and the norm weight of the thread's IT chunks, issued before the first add): N = IT * 2048,
// kc = KC.  TTS-1's down at 17..32 rows (4 chunks) and TTS-1-Max's (7 chunks, N 4096).
template <int KC, int IT>
__global__ __launch_bounds__(256) void splitk_combine_norm_fixed_kernel(
    const float* __restrict__ part, int M, int ldp, bf16_t* __restrict__ resid, int ldo,
    const bf16_t* __restrict__ normw, float eps, bf16_t* __restrict__ xn, int ldn) {
  __shared__ float segs[64];
  constexpr int N = IT * 2048;
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  bf16_t* r = resid + (size_t)m * ldo;
  float4 pa[IT][KC], pb[IT][KC];
  u32x4_t old[IT], g[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int n = (wave * 64 + it * 256 + lane) * 8;  // (the generic kernel's chunk order)
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const float4* q = (const float4*)(part + ((size_t)k * M + m) * ldp + n);
      pa[it][k] = q[0];
      pb[it][k] = q[1];
    }
    old[it] = *(const u32x4_t*)(r + n);
    g[it] = *(const u32x4_t*)(normw + n);
  }
  u32x4_t keep[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    float v[8] = {pa[it][0].x, pa[it][0].y, pa[it][0].z, pa[it][0].w, pb[it][0].x, pb[it][0].y, pb[it][0].z, pb[it][0].w};
#pragma unroll
    for (int k = 1; k < KC; ++k) {  // chunk order, as the generic kernel
      v[0] += pa[it][k].x; v[1] += pa[it][k].y; v[2] += pa[it][k].z; v[3] += pa[it][k].w;
      v[4] += pb[it][k].x; v[5] += pb[it][k].y; v[6] += pb[it][k].z; v[7] += pb[it][k].w;
    }
    u32x4_t pk;
#pragma unroll
    for (int q = 0; q < 4; ++q) pk[q] = pack_bf2(bf_lo(old[it][q]) + rbf(v[2 * q]), bf_hi(old[it][q]) + rbf(v[2 * q + 1]));
    *(u32x4_t*)(r + (wave * 64 + it * 256 + lane) * 8) = pk;
    keep[it] = pk;
    const float ssum = wave_sum_dpp(chunk_sumsq(pk));
    if (lane == 0) segs[wave + 4 * it] = ssum;
  }
  __syncthreads();
  float ss = 0.f;
#pragma unroll
  for (int sg = 0; sg < N / 512; ++sg) ss += segs[sg];
  const float rs = 1.0f / sqrtf(ss / (float)N + eps);
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    u32x4_t v = keep[it];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[q] = pack_bf2(bf_lo(g[it][q]) * rbf(bf_lo(v[q]) * rs), bf_hi(g[it][q]) * rbf(bf_hi(v[q]) * rs));
    *(u32x4_t*)(xn + (size_t)m * ldn + (wave * 64 + it * 256 + lane) * 8) = v;
  }
}

void launch_splitk_combine_norm(const float* part, int kc, int M, int N, int ldp, bf16_t* resid, int ldo,
                                const bf16_t* normw, float eps, bf16_t* xn, int ldn, hipStream_t s) {
  static const bool fixed = !(getenv("TTS_COMBINE_FIXED") && !atoi(getenv("TTS_COMBINE_FIXED")));
  if (dry_record("splitk_combine_norm")) return;
  if (fixed && N == 2048 && kc == 4)
    hipLaunchKernelGGL((splitk_combine_norm_fixed_kernel<4, 1>), dim3(M), dim3(256), 0, s, part, M, ldp, resid, ldo,
                       normw, eps, xn, ldn);
  else if (fixed && N == 4096 && kc == 7)
    hipLaunchKernelGGL((splitk_combine_norm_fixed_kernel<7, 2>), dim3(M), dim3(256), 0, s, part, M, ldp, resid, ldo,
                       normw, eps, xn, ldn);
  else
    hipLaunchKernelGGL(splitk_combine_norm_kernel, dim3(M), dim3(256), 0, s, part, kc, M, N, ldp, resid, ldo,
                       normw, eps, xn, ldn);
}

void launch_splitk_combine(const float* part, int kc, int M, int N, int ldp, bf16_t* out,
                           bf16_t* resid, int ldo, hipStream_t s) {
  if (dry_record("splitk_combine")) return;
  const int n = M * (N / 8);
  hipLaunchKernelGGL(splitk_combine_kernel, dim3((n + 255) / 256), dim3(256), 0, s, part, kc, M, N, ldp,
                     out, resid, ldo);
}

void launch_f32_to_bf16(const float* x, bf16_t* y, long long n, hipStream_t s) {
  long long g = (n + 255) / 256;
  int grid = (int)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid), dim3(256), 0, s, x, y, n);
}

// fp16 checkpoints (the serving CLI loads the LM with torch_dtype=float16,
// tools/serving/inference.py:103-107): f16 -> f32 is exact, then one RNE rounding to bf16
// (exact for f16 values with at most 8 significant bits, i.e. normal-range f16 images of bf16
// weights; f16 subnormals carrying more bits are rounded).
__global__ void f16_to_bf16_kernel(const _Float16* __restrict__ x, bf16_t* __restrict__ y, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    y[i] = f2bf((float)x[i]);
}

void launch_f16_to_bf16(const void* x, bf16_t* y, long long n, hipStream_t s) {
  long long g = (n + 255) / 256;
  int grid = (int)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
  hipLaunchKernelGGL(f16_to_bf16_kernel, dim3(grid), dim3(256), 0, s, (const _Float16*)x, y, n);
}

}  // namespace tts
