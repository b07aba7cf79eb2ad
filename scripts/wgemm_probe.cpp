// wgemm_probe.cpp — per-launch time of the decode-step GEMVs through the C ABI, from C++
// (no Python in the launch loop), rotating over > 600 MB of weight copies (HBM-cold).
// With TTS_WGEMM_DIAG=1/2/4/... the kernel skips prologue / epilogue / MFMA (diagnostics).
// build: hipcc -O2 scripts/wgemm_probe.cpp -Iinclude -Ltts-max_amd/tts_amd -ltts_mi355x
//        -Wl,-rpath,'$ORIGIN/../tts-max_amd/tts_amd' -o scripts/wgemm_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "tts_mi355x_ops.h"

int main() {
  struct Shape { const char* name; int N, K, epi; bool norm; };
  const Shape shapes[] = {{"qkv", 3072, 2048, 0, true}, {"o_proj", 2048, 2048, 1, false},
                          {"gate_up", 16384, 2048, 2, true}, {"down", 2048, 8192, 1, false},
                          {"lm_head", 193856, 2048, 0, true}};
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (const Shape& s : shapes) {
    const size_t wb = (size_t)s.N * s.K * 2;
    const int R = (int)(700e6 / wb) + 2;
    std::vector<void*> w(R);
    void *x, *out, *nw, *tmp;
    hipMalloc(&x, 64 * 8192 * 2);
    hipMalloc(&out, (size_t)64 * s.N * 2);
    hipMalloc(&nw, 8192 * 2);
    hipMalloc(&tmp, wb);
    tts_synth_fill(x, 1, 8192, 7, 1.0f, nullptr);
    tts_synth_fill(nw, 1, 8192, 8, 1.0f, nullptr);
    tts_synth_fill(out, 1, (int64_t)s.N, 9, 1.0f, nullptr);
    tts_synth_fill(tmp, 1, (int64_t)s.N * s.K, 10, 0.02f, nullptr);
    for (int r = 0; r < R; ++r) {
      hipMalloc(&w[r], wb);
      tts_op_retile(tmp, w[r], s.N, s.K, s.epi, nullptr);
    }
    hipDeviceSynchronize();
    const int ldo = s.epi == 2 ? s.N / 2 : s.N;
    auto launch = [&](int i) {
      tts_op_wgemm(x, 1, s.K, s.K, w[i % R], s.N, s.norm ? nw : nullptr, 1e-5f, s.epi == 1 ? nullptr : out, ldo,
                   s.epi == 1 ? out : nullptr, s.epi, nullptr);
    };
    for (int i = 0; i < 8; ++i) launch(i);
    const int iters = 96;
    hipEventRecord(a, nullptr);
    for (int i = 0; i < iters; ++i) launch(i);
    hipEventRecord(b, nullptr);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1000.0 / iters;
    printf("%-8s %8.1f MB %8.2f us %8.1f GB/s  %s\n", s.name, wb / 1e6, us, wb / us / 1e3, tts_last_error());
    for (int r = 0; r < R; ++r) hipFree(w[r]);
    hipFree(x); hipFree(out); hipFree(nw); hipFree(tmp);
  }
  return 0;
}
