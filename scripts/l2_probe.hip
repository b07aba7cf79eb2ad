// l2_probe.hip — does a decode-sized weight read (4..32 MiB, one slab per workgroup) run
// faster when an EARLIER kernel already read the same bytes?  Per size: one launch timed with
// events (a) after a 1 GiB flush (cold), (b) right after the same launch (same workgroup ->
// slab map, so each slab was last read on the same XCD: L2 and Infinity Cache warm), (c) right
// after a launch that reads slab b from workgroup b+1 (another XCD: only the memory-side
// Infinity Cache can hold it), and (d) an empty launch (the floor of the event pair).  Also the
// kernel's own span: first workgroup start to last workgroup end (s_memrealtime, 100 MHz).
// build: hipcc -O3 --offload-arch=gfx950 scripts/l2_probe.hip -o scripts/l2_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

// workgroup b reads slab (b + shift) % gridDim.x, 16 B per lane per load, 4 loads in flight
__global__ __launch_bounds__(1024) void slab_kernel(const u32x4_t* __restrict__ p, size_t slab16, int shift,
                                                    unsigned* sink, unsigned long long* tm) {
  if (threadIdx.x == 0) tm[2 * blockIdx.x] = wall_clock64();
  const int b = (blockIdx.x + shift) % gridDim.x;
  const u32x4_t* q = p + (size_t)b * slab16;
  u32x4_t acc = {0u, 0u, 0u, 0u};
  for (size_t i = threadIdx.x; i < slab16; i += 4 * blockDim.x) {
    u32x4_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const size_t k = i + j * blockDim.x;
      v[j] = q[k < slab16 ? k : i];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= v[j];
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[0] = 1;
  __syncthreads();
  if (threadIdx.x == 0) tm[2 * blockIdx.x + 1] = wall_clock64();
}

__global__ void empty_kernel(unsigned* sink) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && sink == nullptr) sink[0] = 1;
}

int main() {
  const size_t F = (size_t)1024 << 20, MAXS = (size_t)32 << 20;
  char *w, *f;
  unsigned* sink;
  unsigned long long* tm;
  if (hipMalloc(&w, MAXS) != hipSuccess || hipMalloc(&f, F) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess ||
      hipMalloc(&tm, 2 * 256 * 8) != hipSuccess)
    return 1;
  unsigned long long htm[512];
  (void)hipMemset(w, 1, MAXS);
  (void)hipMemset(f, 2, F);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int grid = 256;
  auto launch = [&](const char* p, size_t bytes, int shift) {
    hipLaunchKernelGGL(slab_kernel, dim3(grid), dim3(1024), 0, s, (const u32x4_t*)p, bytes / 16 / grid, shift, sink, tm);
  };
  auto flush = [&]() { launch(f, F, 0); };
  // setup() then one timed launch; median-ish: best and mean of 9 repetitions
  // span of the last launch (us): max end - min start over its workgroups
  auto span = [&]() {
    (void)hipMemcpy(htm, tm, sizeof(htm), hipMemcpyDeviceToHost);
    unsigned long long lo = ~0ull, hi = 0;
    for (int i = 0; i < grid; ++i) {
      lo = htm[2 * i] < lo ? htm[2 * i] : lo;
      hi = htm[2 * i + 1] > hi ? htm[2 * i + 1] : hi;
    }
    return (hi - lo) * 0.01f;
  };
  float span_sum = 0.f;
  auto timed = [&](auto&& setup, auto&& body, float& best, float& mean) {
    best = 1e9f;
    float sum = 0.f;
    span_sum = 0.f;
    for (int r = 0; r < 9; ++r) {
      setup();
      (void)hipEventRecord(a, s);
      body();
      (void)hipEventRecord(b, s);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      best = ms < best ? ms : best;
      sum += ms;
      span_sum += span();
    }
    mean = sum / 9;
  };
  float eb, em;
  timed([&] { flush(); }, [&] { hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(1024), 0, s, sink); }, eb, em);
  printf("empty launch (256 x 1024): best %.2f us, mean %.2f us\n", eb * 1e3f, em * 1e3f);
  for (size_t S : {(size_t)4 << 20, (size_t)8 << 20, (size_t)16 << 20, (size_t)32 << 20}) {
    float cb, cm, wb, wm, xb, xm, cs, ws, xs;
    timed([&] { flush(); }, [&] { launch(w, S, 0); }, cb, cm);
    cs = span_sum / 9;
    timed([&] { flush(); launch(w, S, 0); }, [&] { launch(w, S, 0); }, wb, wm);
    ws = span_sum / 9;
    timed([&] { flush(); launch(w, S, 1); }, [&] { launch(w, S, 0); }, xb, xm);
    xs = span_sum / 9;
    printf("%2zu MiB events best/mean: cold %.2f/%.2f | warm same XCD %.2f/%.2f | warm other XCD %.2f/%.2f us\n",
           S >> 20, cb * 1e3f, cm * 1e3f, wb * 1e3f, wm * 1e3f, xb * 1e3f, xm * 1e3f);
    printf("%2zu MiB in-kernel span (mean): cold %.2f | warm same XCD %.2f | warm other XCD %.2f us\n", S >> 20, cs,
           ws, xs);
  }
  (void)hipStreamSynchronize(s);
  return 0;
}
