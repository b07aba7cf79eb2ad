// mall_probe.hip — can the Infinity Cache (256 MiB, memory-side) pre-stage a decode layer's
// weights?  (1) a full-chip stream of a 121 MB buffer (one TTS-1 layer) from cold caches vs
// right after another read of it; (2) a latency chain (dependent short launches, standing for
// a layer's hand-offs) followed by the stream, with and without a prefetch kernel reading the
// same buffer on a second stream while the chain runs.
// build: hipcc -O3 --offload-arch=gfx950 scripts/mall_probe.hip -o scripts/mall_probe
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
    for (int j = 0; j < LPT; ++j) {
      const size_t k = i + j * stride;
      v[j] = p[k < n16 ? k : i];
    }
#pragma unroll
    for (int j = 0; j < LPT; ++j) acc ^= v[j];
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[0] = 1;
}

__global__ void spin_kernel(unsigned* sink, int loops) {  // a short dependent launch
  for (int i = 0; i < loops; ++i) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0 && blockIdx.x == 0 && loops < 0) sink[1] = 1;
}

int main() {
  const size_t W = (size_t)121 << 20, F = (size_t)1024 << 20;
  char *w, *f;
  unsigned* sink;
  hipMalloc(&w, W);
  hipMalloc(&f, F);
  hipMalloc(&sink, 64);
  hipMemset(w, 1, W);
  hipMemset(f, 2, F);
  hipStream_t sa, sb;
  hipStreamCreateWithFlags(&sa, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&sb, hipStreamNonBlocking);
  hipEvent_t a, b, fork;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventCreate(&fork);
  auto stream = [&](const char* p, size_t bytes, int grid, hipStream_t s) {
    hipLaunchKernelGGL(stream_kernel<8>, dim3(grid), dim3(1024), 0, s, (const u32x4_t*)p, bytes / 16, sink);
  };
  auto flush = [&]() { stream(f, F, 256, sa); };
  auto timed = [&](auto&& body) {
    float best = 1e9f, sum = 0.f;
    for (int r = 0; r < 6; ++r) {
      body(true);  // setup (untimed part inside body before the event)
      hipEventRecord(b, sa);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (r > 0) { sum += ms; best = ms < best ? ms : best; }
    }
    return sum / 5 * 1000.f;
  };
  // (1) cold vs warm full-chip stream
  float cold = timed([&](bool) { flush(); hipEventRecord(a, sa); stream(w, W, 256, sa); });
  float warm = timed([&](bool) { stream(w, W, 256, sa); hipEventRecord(a, sa); stream(w, W, 256, sa); });
  printf("stream 121 MiB, 256 CUs: cold %.1f us (%.0f GB/s), after a read %.1f us (%.0f GB/s)\n", cold, W / cold / 1e3,
         warm, W / warm / 1e3);
  // (2) chain of short launches, then the stream; prefetch on stream b during the chain
  for (int spin : {200, 400, 800}) {
    for (int pg : {0, 32, 64, 128, 256}) {
      float t = timed([&](bool) {
        flush();
        hipEventRecord(a, sa);
        if (pg > 0) {
          hipEventRecord(fork, sa);
          hipStreamWaitEvent(sb, fork, 0);
          stream(w, W, pg, sb);
        }
        for (int i = 0; i < 4; ++i) hipLaunchKernelGGL(spin_kernel, dim3(256), dim3(64), 0, sa, sink, spin);
        stream(w, W, 256, sa);
      });
      float chain = timed([&](bool) {
        flush();
        hipEventRecord(a, sa);
        for (int i = 0; i < 4; ++i) hipLaunchKernelGGL(spin_kernel, dim3(256), dim3(64), 0, sa, sink, spin);
      });
      printf("chain(spin %4d) %7.1f us; chain + stream: prefetch on %3d CUs -> %7.1f us (stream part %7.1f)\n", spin,
             chain, pg, t, t - chain);
      hipStreamSynchronize(sb);
    }
  }
  return 0;
}
