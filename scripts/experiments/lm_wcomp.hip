// lm_wcomp.hip — exponent-coded weight stream for the one-row decode GEMVs (lossless).
//
// The one-row decode step is a stream of 2.7 GB of bf16 weights (HBM-bound: DESIGN §3).  A
// trained or random-init weight matrix uses few exponents: nearly every 1 KiB tile's 512
// values have their bf16 exponent field inside one window of 16 values [eb, eb + 15].  Such a
// tile is stored as 768 B — per value the sign + 7 mantissa bits (a byte) and a 4-bit code
// e - eb — and decoded in registers back to the exact bf16 bits (hip_common.h wc_decode: one
// v_perm, an and and two adds per pair), so the MFMA sees the same operands and every sum is
// bit-identical to the plain stream.  A tile with any exponent outside the window (zeros,
// subnormals, tiny outliers: ~1-2 % of tiles for uniform weights) is kept raw (1 KiB) in a
// side buffer; a per-tile meta word (0 = coded, else 1 + slot) tells the kernel which, read
// a ring depth ahead of the stage (lm_gemm_kernel.h).  eb is chosen per matrix to cover the
// most tiles (lm_engine.cpp build_wcomp).
//
// Coded lane record (12 B, lane l of tile t at rec + (t * 64 + l) * 12): d0 = bytes of values
// 0..3, d1 = values 4..7, n = codes (value 2q at bits 4q.., value 2q+1 at bits 16+4q..).
#include "hip_common.h"
#include "lm_kernels.h"

namespace tts {

// one wave per tile: min / max exponent field over its 512 values
__global__ void wcomp_stats_kernel(const bf16_t* __restrict__ w, long long ntiles, uint8_t* emin, uint8_t* emax) {
  const int lane = threadIdx.x & 63;
  const long long waves = (long long)gridDim.x * (blockDim.x >> 6);
  for (long long t = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6); t < ntiles; t += waves) {
    const u32x4_t v = *(const u32x4_t*)(w + (size_t)(t * 64 + lane) * 8);
    int lo = 255, hi = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e0 = (v[q] >> 7) & 0xFF, e1 = (v[q] >> 23) & 0xFF;
      lo = min(lo, min(e0, e1));
      hi = max(hi, max(e0, e1));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, __shfl_xor(lo, o, 64));
      hi = max(hi, __shfl_xor(hi, o, 64));
    }
    if (lane == 0) { emin[t] = (uint8_t)lo; emax[t] = (uint8_t)hi; }
  }
}

__global__ void wcomp_encode_kernel(const bf16_t* __restrict__ w, long long ntiles, uint32_t eb,
                                    const uint32_t* __restrict__ meta, uint32_t* __restrict__ rec,
                                    bf16_t* __restrict__ esc) {
  const int lane = threadIdx.x & 63;
  const long long waves = (long long)gridDim.x * (blockDim.x >> 6);
  for (long long t = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6); t < ntiles; t += waves) {
    const u32x4_t v = *(const u32x4_t*)(w + (size_t)(t * 64 + lane) * 8);
    const uint32_t m = meta[t];
    uint32_t* r = rec + (size_t)(t * 64 + lane) * 3;
    if (m) {  // raw tile in the side buffer; its coded record is never read
      *(u32x4_t*)(esc + (size_t)(m - 1) * 512 + lane * 8) = v;
      r[0] = 0; r[1] = 0; r[2] = 0;
      continue;
    }
    uint32_t d[2] = {0u, 0u}, n = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t h = (j & 1) ? (v[j >> 1] >> 16) : (v[j >> 1] & 0xFFFFu);
      const uint32_t byte = ((h >> 8) & 0x80u) | (h & 0x7Fu);
      const uint32_t c = ((h >> 7) & 0xFFu) - eb;  // 0..15 (the tile fits the window)
      d[j >> 2] |= byte << (8 * (j & 3));
      n |= c << ((j & 1) ? 16 + 4 * (j >> 1) : 4 * (j >> 1));
    }
    r[0] = d[0]; r[1] = d[1]; r[2] = n;
  }
}

__global__ void wcomp_decode_kernel(const uint32_t* __restrict__ rec, const uint32_t* __restrict__ meta,
                                    const bf16_t* __restrict__ esc, uint32_t eb, long long ntiles,
                                    bf16_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint32_t eb2 = (eb << 7) | (eb << 23);
  const long long waves = (long long)gridDim.x * (blockDim.x >> 6);
  for (long long t = blockIdx.x * (long long)(blockDim.x >> 6) + (threadIdx.x >> 6); t < ntiles; t += waves) {
    const uint32_t m = meta[t];
    u32x4_t v;
    if (m) {
      v = *(const u32x4_t*)(esc + (size_t)(m - 1) * 512 + lane * 8);
    } else {
      const uint32_t* r = rec + (size_t)(t * 64 + lane) * 3;
      v = wc_decode(u32x4_t{r[0], r[1], r[2], 0u}, eb2);
    }
    *(u32x4_t*)(out + (size_t)(t * 64 + lane) * 8) = v;
  }
}

static int wcomp_grid(long long ntiles) {
  long long g = (ntiles + 3) / 4;
  return (int)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

void launch_wcomp_stats(const bf16_t* tiled, long long ntiles, uint8_t* emin, uint8_t* emax, hipStream_t s) {
  hipLaunchKernelGGL(wcomp_stats_kernel, dim3(wcomp_grid(ntiles)), dim3(256), 0, s, tiled, ntiles, emin, emax);
}
void launch_wcomp_encode(const bf16_t* tiled, long long ntiles, uint32_t eb, const uint32_t* meta,
                         uint32_t* rec, bf16_t* esc, hipStream_t s) {
  hipLaunchKernelGGL(wcomp_encode_kernel, dim3(wcomp_grid(ntiles)), dim3(256), 0, s, tiled, ntiles, eb, meta, rec,
                     esc);
}
void launch_wcomp_decode(const uint32_t* rec, const uint32_t* meta, const bf16_t* esc, uint32_t eb,
                         long long ntiles, bf16_t* out, hipStream_t s) {
  hipLaunchKernelGGL(wcomp_decode_kernel, dim3(wcomp_grid(ntiles)), dim3(256), 0, s, rec, meta, esc, eb, ntiles,
                     out);
}

}  // namespace tts
