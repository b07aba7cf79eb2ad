// chain_probe.hip — what does one batch-1 TTS-1 decode layer cost as a chain of dependent
// weight-streaming launches, by launch geometry?  Four GEMVs per layer (QKV 3072x2048,
// o_proj 2048x2048, gate/up 16384x2048, down 2048x8192; MFMA-tiled 1 KiB tiles as in the
// engine), each reading the vector the previous launch wrote, 16 layers of distinct weights
// (HBM-cold) captured into one hipGraph.  Variants: the full chain, the chain without weight
// loads (dependency + launch floor), and per-kernel geometry sweeps.
// build: hipcc -O3 --offload-arch=gfx950 scripts/chain_probe.hip -o scripts/chain_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef unsigned short bf16_t;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((unsigned)h) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

// One wave = TPW consecutive k-tiles of one 16-column tile; KS = KT / TPW waves per column
// tile; XW workgroups share a column tile (XW = 2: fp32 atomic pair + arrival ticket, the
// second arriver finishes; a+b is order-free for two terms).  NORM: every wave computes the
// RMS statistic of x itself (no barrier).  MODE 0: full; 1: no weight loads; 2: no x read.
template <int WAVES, int TPW, int XW, bool NORM, int MODE>
__global__ __launch_bounds__(WAVES * 64) void gv_kernel(const u32x4_t* __restrict__ W, const bf16_t* x, bf16_t* y,
                                                       int KT, float* acc2, int* tick) {
  __shared__ float red[WAVES][16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int KS = KT / TPW;            // waves per column tile (whole grid)
  const int KSW = KS / XW;            // of them in this workgroup
  const int CPW = WAVES / KSW;        // column tiles per workgroup
  const int ctl = wave / KSW, kp = (blockIdx.x % XW) * KSW + wave % KSW;
  const int ct = (blockIdx.x / XW) * CPW + ctl;
  const u32x4_t* wp = W + ((size_t)ct * KT + (size_t)kp * TPW) * 64 + lane;
  u32x4_t w[TPW];
  if (MODE != 1) {
#pragma unroll
    for (int t = 0; t < TPW; ++t) w[t] = __builtin_nontemporal_load(wp + t * 64);
  }
  u32x4_t xv[TPW];
  float r = 1.f;
  if (MODE != 2) {
#pragma unroll
    for (int t = 0; t < TPW; ++t) xv[t] = *(const u32x4_t*)(x + (kp * TPW + t) * 32 + 8 * (lane >> 4));
    if (NORM) {
      const int K = KT * 32;
      float ss = 0.f;
      for (int k = lane * 8; k < K; k += 512) {
        const u32x4_t v = *(const u32x4_t*)(x + k);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float lo = __uint_as_float(v[q] << 16), hi = __uint_as_float(v[q] & 0xffff0000u);
          ss += lo * lo + hi * hi;
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
      r = 1.0f / sqrtf(ss / (float)K + 1e-5f);
    }
  } else {
#pragma unroll
    for (int t = 0; t < TPW; ++t) xv[t] = u32x4_t{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};
  }
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    u32x4_t a = xv[t];
    if (NORM) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float lo = __uint_as_float(a[q] << 16) * r, hi = __uint_as_float(a[q] & 0xffff0000u) * r;
        a[q] = (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
      }
    }
    const u32x4_t b = MODE == 1 ? a : w[t];
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                 acc, 0, 0, 0);
  }
  // row 0 of the 16x16 result lives in lanes 0..15, acc[0]
  if (lane < 16) red[wave][lane] = acc[0];
  __syncthreads();
  if (wave % KSW == 0 && lane < 16) {
    float s = 0.f;
    for (int i = 0; i < KSW; ++i) s += red[wave + i][lane];
    const int n = ct * 16 + lane;
    if (XW == 1) {
      y[n] = f2bf(s * 0.03f);
    } else {
      atomicAdd(acc2 + n, s);
      __threadfence();
      const int prev = atomicAdd(tick + n, 1);
      if (prev == XW - 1) {
        const float t = __hip_atomic_load(acc2 + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        y[n] = f2bf(t * 0.03f);
        acc2[n] = 0.f;
        tick[n] = 0;
      }
    }
  }
}

struct Geo { int waves, tpw, xw; };

template <int WAVES, int TPW, int XW, bool NORM, int MODE>
static void launch_t(const u32x4_t* W, const bf16_t* x, bf16_t* y, int N, int KT, float* acc2, int* tick, hipStream_t s) {
  const int NCT = N / 16, KS = KT / TPW, KSW = KS / XW;
  if (KS % XW || WAVES % KSW) { printf("bad geo N %d KT %d waves %d tpw %d xw %d\n", N, KT, WAVES, TPW, XW); exit(1); }
  const int grid = NCT * XW / (WAVES / KSW);
  hipLaunchKernelGGL((gv_kernel<WAVES, TPW, XW, NORM, MODE>), dim3(grid), dim3(WAVES * 64), 0, s, W, x, y, KT, acc2, tick);
}

template <bool NORM, int MODE>
static void launch(Geo g, const u32x4_t* W, const bf16_t* x, bf16_t* y, int N, int KT, float* acc2, int* tick, hipStream_t s) {
#define G(WV, TP, XW) if (g.waves == WV && g.tpw == TP && g.xw == XW) return launch_t<WV, TP, XW, NORM, MODE>(W, x, y, N, KT, acc2, tick, s);
  G(4, 16, 1) G(8, 8, 1) G(16, 4, 1) G(16, 2, 2)
  G(4, 8, 2) G(8, 4, 2) G(16, 16, 1) G(8, 16, 2) G(16, 8, 2)
  printf("geo not instantiated %d %d %d\n", g.waves, g.tpw, g.xw);
  exit(1);
}

int main(int argc, char** argv) {
  const int L = 16;
  const int Ns[4] = {3072, 2048, 16384, 2048}, Ks[4] = {2048, 2048, 2048, 8192};
  std::vector<u32x4_t*> Wb(4 * L);
  for (int l = 0; l < L; ++l)
    for (int j = 0; j < 4; ++j) {
      CK(hipMalloc(&Wb[l * 4 + j], (size_t)Ns[j] * Ks[j] * 2));
      CK(hipMemset(Wb[l * 4 + j], 0x11, (size_t)Ns[j] * Ks[j] * 2));
    }
  bf16_t* vec[5];
  for (int i = 0; i < 5; ++i) { CK(hipMalloc(&vec[i], 16384 * 2)); CK(hipMemset(vec[i], 0x3f, 16384 * 2)); }
  float* acc2;
  int* tick;
  CK(hipMalloc(&acc2, 16384 * 4 * 4));
  CK(hipMalloc(&tick, 16384 * 4 * 4));
  CK(hipMemset(acc2, 0, 16384 * 16));
  CK(hipMemset(tick, 0, 16384 * 16));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  // per-kernel geometry sets: {qkv, o, gu, down}
  struct Cfg { const char* name; Geo g[4]; };
  std::vector<Cfg> cfgs = {
      {"engine-like 16w", {{16, 4, 1}, {16, 4, 1}, {16, 4, 1}, {16, 16, 1}}},
      {"8w tpw8", {{8, 8, 1}, {8, 8, 1}, {8, 8, 1}, {8, 16, 2}}},
      {"4w tpw16", {{4, 16, 1}, {4, 16, 1}, {4, 16, 1}, {8, 16, 2}}},
      {"8w tpw4 x2", {{8, 4, 2}, {8, 4, 2}, {8, 8, 1}, {8, 16, 2}}},
      {"4w tpw8 x2", {{4, 8, 2}, {4, 8, 2}, {4, 16, 1}, {8, 16, 2}}},
      {"mix a", {{16, 4, 1}, {8, 4, 2}, {8, 8, 1}, {16, 16, 1}}},
      {"mix b", {{8, 8, 1}, {8, 4, 2}, {4, 16, 1}, {8, 16, 2}}},
      {"mix c", {{4, 8, 2}, {4, 8, 2}, {8, 8, 1}, {16, 8, 2}}},
      {"16w tpw2 x2", {{16, 2, 2}, {16, 2, 2}, {16, 4, 1}, {16, 16, 1}}},
  };
  for (int mode = 0; mode < 3; ++mode) {
    for (auto& c : cfgs) {
      auto body = [&]() {
        for (int l = 0; l < L; ++l) {
          const bf16_t* x = vec[0];
          for (int j = 0; j < 4; ++j) {
            const bool norm = j == 0 || j == 2;
            bf16_t* y = vec[j + 1];
            float* a2 = acc2 + j * 16384;
            int* tk = tick + j * 16384;
            const int KT = Ks[j] / 32;
            if (j == 3) y = vec[0];
            if (mode == 0) { if (norm) launch<true, 0>(c.g[j], Wb[l * 4 + j], x, y, Ns[j], KT, a2, tk, s); else launch<false, 0>(c.g[j], Wb[l * 4 + j], x, y, Ns[j], KT, a2, tk, s); }
            if (mode == 1) { if (norm) launch<true, 1>(c.g[j], Wb[l * 4 + j], x, y, Ns[j], KT, a2, tk, s); else launch<false, 1>(c.g[j], Wb[l * 4 + j], x, y, Ns[j], KT, a2, tk, s); }
            if (mode == 2) launch<false, 2>(c.g[j], Wb[l * 4 + j], x, y, Ns[j], KT, a2, tk, s);
            x = y;
          }
        }
      };
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      body();
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
      const int reps = 20;
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us_layer = ms * 1000.0 / reps / L;
      printf("mode %d (%s) %-16s  %7.2f us/layer  %6.1f GB/s\n", mode, mode == 0 ? "full" : mode == 1 ? "no-weights" : "no-dep",
             c.name, us_layer, 121.6e6 / us_layer / 1e3);
      fflush(stdout);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  // per-kernel isolated timing (each kernel repeated over the 16 layers' weights, graph)
  for (int j = 0; j < 4; ++j) {
    for (auto& c : cfgs) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int l = 0; l < L; ++l)
        launch<false, 0>(c.g[j], Wb[l * 4 + j], vec[1], vec[2 + (l & 1)], Ns[j], Ks[j] / 32, acc2, tick, s);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
      const int reps = 20;
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1000.0 / reps / L;
      printf("kernel %d (%5dx%5d) %-16s geo %2dw tpw %2d xw %d: %7.2f us  %6.1f GB/s\n", j, Ns[j], Ks[j], c.name,
             c.g[j].waves, c.g[j].tpw, c.g[j].xw, us, (double)Ns[j] * Ks[j] * 2 / us / 1e3);
      fflush(stdout);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
