// cu_bw_probe.hip — streaming read bandwidth when only G of the 256 CUs stream (one
// 1024-thread workgroup per CU, LPT 16-B loads in flight per lane, non-temporal): how much
// of HBM can half the chip pull (the persistent step's stream / chain CU split)?
// build: hipcc -O3 --offload-arch=gfx950 scripts/cu_bw_probe.hip -o scripts/cu_bw_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
template <int LPT>
__global__ __launch_bounds__(1024) void stream_kernel(const u32x4_t* __restrict__ p, size_t n16, unsigned* sink) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  u32x4_t acc = {0u, 0u, 0u, 0u};
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += LPT * stride) {
    u32x4_t v[LPT];
#pragma unroll
    for (int j = 0; j < LPT; ++j) { const size_t k = i + j * stride; v[j] = __builtin_nontemporal_load(p + (k < n16 ? k : i)); }
#pragma unroll
    for (int j = 0; j < LPT; ++j) acc ^= v[j];
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[0] = 1;
}
int main() {
  const size_t bytes = (size_t)100 << 20, pool = (size_t)1600 << 20;
  char* buf; unsigned* sink;
  hipMalloc(&buf, pool); hipMalloc(&sink, 64); hipMemset(buf, 1, pool);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int copies = (int)(pool / bytes);
  for (int lpt : {4, 8, 16}) for (int G : {32, 64, 96, 128, 192, 256}) {
    auto launch = [&](int c) {
      const u32x4_t* p = (const u32x4_t*)(buf + (size_t)c * bytes);
      if (lpt == 4) hipLaunchKernelGGL(stream_kernel<4>, dim3(G), dim3(1024), 0, 0, p, bytes / 16, sink);
      else if (lpt == 8) hipLaunchKernelGGL(stream_kernel<8>, dim3(G), dim3(1024), 0, 0, p, bytes / 16, sink);
      else hipLaunchKernelGGL(stream_kernel<16>, dim3(G), dim3(1024), 0, 0, p, bytes / 16, sink);
    };
    for (int i = 0; i < 3; ++i) launch(i % copies);
    hipEventRecord(a, 0);
    for (int i = 0; i < 24; ++i) launch(i % copies);
    hipEventRecord(b, 0); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1000.0 / 24;
    printf("lpt %2d CUs %3d: %8.1f us per 100 MiB  %7.1f GB/s total  %6.1f GB/s per CU\n", lpt, G, us, bytes / us / 1e3,
           bytes / us / 1e3 / G);
  }
  return 0;
}
