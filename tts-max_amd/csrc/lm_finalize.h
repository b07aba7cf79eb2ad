// lm_finalize.h — the greedy step's row finalize (finalize_greedy_kernel, lm_ops.hip: one
// workgroup per sequence): reduce the lm_head partial argmaxes (lowest index on ties), append the
// token, update the repetition-penalty id set, stop on EOS / length, and gather the next
// step's input embedding.  Reference: GenerationMixin._sample (generation/utils.py:2894-2936).
#pragma once
#include "hip_common.h"
#include "lm_kernels.h"

namespace tts {

// Called by every thread of a workgroup of NT threads (barriers inside; uniform `b`).
// lds: >= NT / 64 * 2 + 1 words of LDS.  (A last-arriving lm_head workgroup running this on
// write-through partials, SC1, measured no faster than the separate launch: DESIGN §3.)
template <int NT, bool SC1>
TTS_DEV void finalize_row(const float* pv, const int* pi, int nparts, const StepState& st, int b,
                          const bf16_t* embed, bf16_t* x, int hidden, int* lds) {
  float* sv = (float*)lds;
  int* si = lds + NT / 64;
  int* stok = lds + 2 * (NT / 64);
  const int tid = threadIdx.x;
  // the row's state is read with the partials (one round trip), not after the reduction
  const int done = st.done[b];
  int g0 = 0, lim = 0, pos0 = 0;
  if (tid == 0) { g0 = st.gen_count[b]; lim = st.limit[b]; pos0 = st.pos[b]; }
  float v = -INFINITY;
  int i = 0x7fffffff;
  for (int p = tid; p < nparts; p += NT) {
    float v2;
    int i2;
    if constexpr (SC1) {
      v2 = __hip_atomic_load(pv + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      i2 = __hip_atomic_load(pi + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      v2 = pv[p];
      i2 = pi[p];
    }
    if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
  }
  if (done) return;  // (uniform)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(v, o, 64);
    const int i2 = __shfl_xor(i, o, 64);
    if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
  }
  if ((tid & 63) == 0) { sv[tid >> 6] = v; si[tid >> 6] = i; }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < NT / 64; ++w)
      if (sv[w] > v || (sv[w] == v && si[w] < i)) { v = sv[w]; i = si[w]; }
    // all-(-inf) rows cannot happen (only EOS is masked); guard anyway
    const int tok = (i == 0x7fffffff) ? 0 : i;
    const int g = g0;
    st.out_ids[(size_t)b * st.out_stride + g] = tok;
    st.gen_count[b] = g + 1;
    st.seen[(size_t)b * st.seen_stride + (tok >> 5)] |= 1u << (tok & 31);
    if (st.counts) st.counts[(size_t)b * st.seen_stride * 32 + tok] += 1;
    st.tokens[b] = tok;
    st.pos[b] = pos0 + 1;
    const bool stop = (tok == st.eos_id) || (g + 1 >= lim);
    st.eos_mask[b] = (g + 1 < st.min_new) ? st.eos_id : -1;
    if (stop) {
      st.done[b] = 1;
      atomicSub(st.n_active, 1);
    }
    *stok = tok;
  }
  __syncthreads();
  const u32x4_t* src = (const u32x4_t*)(embed + (size_t)(*stok) * hidden);
  u32x4_t* dst = (u32x4_t*)(x + (size_t)b * hidden);
  for (int k = tid; k < hidden / 8; k += NT) dst[k] = src[k];
}

}  // namespace tts
