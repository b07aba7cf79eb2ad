// hip_common.h — shared device helpers for the gfx950 kernels (wave64, bf16 bit tricks).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;  // raw bf16 bits; all arithmetic is done in fp32
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

#define TTS_DEV __device__ __forceinline__
// Diagnostic build only (make stamps: -DTTS_STAMPS, scripts/stamp_probe.py): thread 0 of a
// workgroup writes the chip-wide 100 MHz clock to stamps[slot].  Compiled out otherwise.
#ifdef TTS_STAMPS
#define TTS_STAMP(buf, slot) \
  do { if ((buf) && threadIdx.x == 0) (buf)[slot] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define TTS_STAMP_WAVE(buf, slot) \
  do { if ((buf) && (threadIdx.x & 63) == 0) (buf)[slot] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define TTS_STAMP(buf, slot) do {} while (0)
#define TTS_STAMP_WAVE(buf, slot) do {} while (0)
#endif
// Timing-diagnostic switches of the GEMM kernel (WgemmArgs::diag, TTS_WGEMM_DIAG) exist in the
// diagnostic build only.  In the product build they must not exist even as untaken branches:
// a branch that skips the LDS-DMA landing wait leaves the DMA "pending" on one path, and the
// compiler's wait insertion merges paths pessimistically, i.e. puts s_waitcnt vmcnt(0) (drain
// the whole weight ring) before the first LDS read of the prologue.
#ifdef TTS_STAMPS
constexpr int kWgemmDiagMask = ~0;
#else
constexpr int kWgemmDiagMask = 0;
#endif

// bf16 -> fp32 is exact: the bf16 bits are the top half of the fp32 pattern.
// Workgroup barrier ordering LDS only: unlike __syncthreads (which waits for every
// outstanding global load first, vmcnt(0)), the weight stream a wave has in flight stays in
// flight across it.  For hand-offs through LDS only.
TTS_DEV void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
TTS_DEV float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
TTS_DEV float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
TTS_DEV float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// fp32 -> bf16 round-to-nearest-even (same rounding as torch's .to(bfloat16)): gfx950's
// v_cvt_pk_bf16_f32.  (A software RNE with a NaN test compiles to an exec-mask branch per
// element: ~25 instructions, which made the RMSNorm prologues the cost of a whole GEMV.)
typedef __attribute__((ext_vector_type(2))) float f32x2_cvt_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_cvt_t;
TTS_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
// Round an fp32 value to the nearest bf16 value, returned as fp32 (torch bf16 op semantics:
// every bf16 elementwise op computes in fp32 and rounds its result once).
TTS_DEV float rbf(float f) { return bf2f(f2bf(f)); }
TTS_DEV uint32_t pack_bf2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_cvt_t){lo, hi}, bf16x2_cvt_t));
}

// ---- DPP wave reductions (VALU speed; __shfl_xor lowers to ds_bpermute = LDS latency)
template <int CTRL, int ROW_MASK = 0xf>
TTS_DEV float dpp_mov(float old, float src) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), CTRL,
                                                    ROW_MASK, 0xf, false));
}
// quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror, row_bcast:15 (rows
// 1,3), row_bcast:31 (rows 2,3): lane 63 ends with the full reduction; read it uniformly.
TTS_DEV float wave_sum_dpp(float v) {
  v += dpp_mov<0xB1>(0.f, v);
  v += dpp_mov<0x4E>(0.f, v);
  v += dpp_mov<0x141>(0.f, v);
  v += dpp_mov<0x140>(0.f, v);
  v += dpp_mov<0x142, 0xA>(0.f, v);
  v += dpp_mov<0x143, 0xC>(0.f, v);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
// LDS-DMA operand pointer types (__builtin_amdgcn_global_load_lds)
typedef __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
// s_waitcnt immediates (gfx9 encoding: vmcnt [3:0]+[15:14], expcnt [6:4], lgkmcnt [11:8])
constexpr int waitcnt_vm(int n) { return (n & 15) | (((n >> 4) & 3) << 14) | (7 << 4) | (15 << 8); }
constexpr int waitcnt_lgkm0() { return 15 | (3 << 14) | (7 << 4); }

// RMSNorm sum of squares, canonical order shared by every implementation (fused prologue,
// LDS prologue, standalone kernel) so all of them round identically: per 16-B chunk of 8
// values, then a DPP wave sum over each 512-value segment, then the segments in order.
TTS_DEV float chunk_sumsq(u32x4_t v) {
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float lo = bf_lo(v[q]), hi = bf_hi(v[q]);
    s += lo * lo + hi * hi;
  }
  return s;
}
TTS_DEV float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(-INFINITY, v));
  v = fmaxf(v, dpp_mov<0x4E>(-INFINITY, v));
  v = fmaxf(v, dpp_mov<0x141>(-INFINITY, v));
  v = fmaxf(v, dpp_mov<0x140>(-INFINITY, v));
  v = fmaxf(v, dpp_mov<0x142, 0xA>(-INFINITY, v));
  v = fmaxf(v, dpp_mov<0x143, 0xC>(-INFINITY, v));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

TTS_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
TTS_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024).  `red` is >= 16 floats of LDS.
TTS_DEV float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum_dpp(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];  // fixed order: deterministic
  return t;
}
TTS_DEV float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max_dpp(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

TTS_DEV float silu_f(float x) { return x / (1.0f + expf(-x)); }

