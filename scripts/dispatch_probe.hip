// dispatch_probe.hip — the per-launch floor of a decode-sized kernel as a function of its
// shape: empty launches and 8 MiB slab reads (one slab per workgroup, warm in L2 from the
// previous launch) at grid x block = 256 x {64, 256, 512, 1024}, 128 x 1024, 512 x 256.
// Durations come from the kernel trace: run under rocprofv3 --kernel-trace (each shape is
// launched 20 times in a row; the kernel's template arguments name the shape).
// Then the 128 x 1024 slab read (one o_proj unit of 64 KiB per workgroup) with the pieces a
// decode GEMM adds one at a time: 80 KiB of dynamic LDS, a 1 KiB kernel-argument struct, a
// split-K style reduction (16 wave partials through LDS, a barrier, one wave sums and stores).
// build: hipcc -O3 --offload-arch=gfx950 scripts/dispatch_probe.hip -o scripts/dispatch_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

template <int GRID, int BLOCK>
__global__ __launch_bounds__(BLOCK) void empty_kernel(unsigned* sink) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && sink == nullptr) sink[0] = 1;
}

template <int GRID, int BLOCK>
__global__ __launch_bounds__(BLOCK) void slab_kernel(const u32x4_t* __restrict__ p, size_t slab16, unsigned* sink) {
  const u32x4_t* q = p + (size_t)blockIdx.x * slab16;
  u32x4_t acc = {0u, 0u, 0u, 0u};
  for (size_t i = threadIdx.x; i < slab16; i += 4 * BLOCK) {
    u32x4_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const size_t k = i + j * BLOCK;
      v[j] = q[k < slab16 ? k : i];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= v[j];
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[0] = 1;
}

struct BigArgs {
  const u32x4_t* p;
  size_t slab16;
  unsigned* sink;
  float* out;
  long long pad[124];
};

// FLAGS: 1 dynamic LDS (launch), 2 big kernarg, 4 LDS reduction + store
template <int FLAGS>
__global__ __launch_bounds__(1024) void gemmish_kernel(BigArgs a) {
  extern __shared__ float red[];
  const u32x4_t* q = a.p + (size_t)blockIdx.x * a.slab16;
  u32x4_t acc = {0u, 0u, 0u, 0u};
  for (size_t i = threadIdx.x; i < a.slab16; i += 4 * 1024) {
    u32x4_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const size_t k = i + j * 1024;
      v[j] = q[k < a.slab16 ? k : i];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= v[j];
  }
  if constexpr (FLAGS & 4) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    red[wave * 64 + lane] = (float)(acc[0] ^ acc[1] ^ acc[2] ^ acc[3]);
    __syncthreads();
    if (wave == 0) {
      float t = 0.f;
      for (int w = 0; w < 16; ++w) t += red[w * 64 + lane];
      a.out[blockIdx.x * 64 + lane] = t;
    }
  } else {
    if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) a.sink[0] = 1;
  }
}

template <int FLAGS>
static void run_g(const char* w, size_t bytes, unsigned* sink, float* out, hipStream_t s) {
  BigArgs a;
  a.p = (const u32x4_t*)w;
  a.slab16 = bytes / 16 / 128;
  a.sink = sink;
  a.out = out;
  const size_t lds = (FLAGS & 1) ? 80 * 1024 : ((FLAGS & 4) ? 4096 : 0);
  for (int r = 0; r < 20; ++r) hipLaunchKernelGGL((gemmish_kernel<FLAGS>), dim3(128), dim3(1024), lds, s, a);
  (void)hipStreamSynchronize(s);
}

template <int GRID, int BLOCK>
static void run(const char* w, size_t bytes, unsigned* sink, hipStream_t s) {
  for (int r = 0; r < 20; ++r) hipLaunchKernelGGL((empty_kernel<GRID, BLOCK>), dim3(GRID), dim3(BLOCK), 0, s, sink);
  for (int r = 0; r < 20; ++r)
    hipLaunchKernelGGL((slab_kernel<GRID, BLOCK>), dim3(GRID), dim3(BLOCK), 0, s, (const u32x4_t*)w,
                       bytes / 16 / GRID, sink);
  (void)hipStreamSynchronize(s);
}

int main() {
  const size_t S = (size_t)8 << 20;
  char* w;
  unsigned* sink;
  if (hipMalloc(&w, S) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  (void)hipMemset(w, 1, S);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  run<256, 64>(w, S, sink, s);
  run<256, 256>(w, S, sink, s);
  run<256, 512>(w, S, sink, s);
  run<256, 1024>(w, S, sink, s);
  run<128, 1024>(w, S, sink, s);
  run<512, 256>(w, S, sink, s);
  run<128, 512>(w, S, sink, s);
  float* out;
  if (hipMalloc(&out, 128 * 64 * 4) != hipSuccess) return 1;
  (void)hipFuncSetAttribute((const void*)gemmish_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
  (void)hipFuncSetAttribute((const void*)gemmish_kernel<7>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
  run_g<0>(w, S, sink, out, s);
  run_g<1>(w, S, sink, out, s);
  run_g<4>(w, S, sink, out, s);
  run_g<7>(w, S, sink, out, s);
  printf("done\n");
  return 0;
}
