// lm_sample.hip — the sampling head of GenerationMixin._sample (transformers, pinned 4.53.2
// by uv.lock:4610; the settings of tts/inference/inferencing.py:94-104, defaults
// InferenceSettings inferencing.py:15-40: temperature 0.8, top_p 1.0, HF top_k 50):
//   scores  = processed logits (bf16-rounded, repetition penalty, min-new EOS mask: the
//             lm_head epilogue, lm_gemm_kernel.h EPI_LOGITS)
//   TemperatureLogitsWarper (logits_process.py:238-300): scores / T        (T != 1 only)
//   TopKLogitsWarper        (logits_process.py:542-580): scores < topk(scores, k)[-1] -> -inf
//   TopPLogitsWarper        (logits_process.py:473-540): ascending sort, softmax, cumsum,
//                            remove cum <= 1 - p, always keep the largest        (p < 1 only)
//   probs = softmax(scores); next = multinomial(probs)   (generation/utils.py:2918-2923)
// The draw uses this engine's counter-based RNG (splitmix64 of seed, row, step), so token
// ids match torch only in distribution, never bitwise (torch's Philox stream is not
// reproducible outside torch).  The filtered distribution itself is exact to fp32 rounding.
//
// MI355X design: one 1024-thread workgroup per row.  Candidates for the top-k are the
// values >= the k-th largest of the lm_head workgroups' maxima (a lower bound of the true
// k-th value: those maxima are k members of the row), found in ONE pass over the row and
// appended to LDS; an exact 64-bit bitonic sort (value desc, index desc) of the few
// candidates gives top-k, top-p and the inverse-CDF draw.  If the bound admits too many
// candidates (adversarial rows), an exact 4-pass radix select on the row replaces it.
#include "hip_common.h"
#include "lm_kernels.h"

namespace tts {

namespace {

constexpr int SMP_THREADS = 1024;
constexpr int SMP_CMAX = 2048;  // LDS candidates

TTS_DEV uint32_t okey(float f) {  // order-preserving float -> uint
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
TTS_DEV float okey_inv(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

TTS_DEV float rng_uniform(unsigned long long seed, int row, int step) {
  unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (((unsigned long long)row << 32) + (unsigned)step + 1ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  return (float)(z >> 40) * (1.0f / 16777216.0f);  // [0, 1)
}

// bitonic sort, descending, of n (power of two) 64-bit keys in LDS
TTS_DEV void bitonic_desc(unsigned long long* a, int n) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += SMP_THREADS) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long x = a[i], y = a[ixj];
          const bool desc = (i & k) == 0;
          if (desc ? (x < y) : (x > y)) { a[i] = y; a[ixj] = x; }
        }
      }
      __syncthreads();
    }
  }
}

__global__ __launch_bounds__(SMP_THREADS) void sample_kernel(SampleArgs a) {
  __shared__ unsigned long long cand[SMP_CMAX];
  __shared__ unsigned hist[256];
  __shared__ int s_cnt;
  __shared__ uint32_t s_thr;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (a.done && a.done[b]) return;
  const float* l = a.logits + (size_t)b * a.ldl;
  const int V = a.V;
  const bool scale = a.temperature != 1.0f;
  auto sval = [&](int i) { const float v = l[i]; return scale ? v / a.temperature : v; };
  const int k = (a.top_k > 0 && a.top_k < V) ? a.top_k : V;

  // ---- threshold: k-th largest of the lm_head partial maxima (a lower bound), or exact
  uint32_t thr = 0u;  // keep keys >= thr
  bool exact = false;
  if (k < V && a.part_val != nullptr && a.nparts >= k && a.nparts <= SMP_CMAX) {
    int np2 = 64;
    while (np2 < a.nparts) np2 <<= 1;
    for (int i = tid; i < np2; i += SMP_THREADS) {
      const float v = i < a.nparts ? a.part_val[(size_t)b * a.part_stride + i] : -INFINITY;
      cand[i] = ((unsigned long long)okey(scale ? v / a.temperature : v) << 32) | (unsigned)i;
    }
    __syncthreads();
    bitonic_desc(cand, np2);
    thr = (uint32_t)(cand[k - 1] >> 32);
    __syncthreads();
  } else if (k < V) {
    exact = true;
  }

  for (int attempt = 0; attempt < 2; ++attempt) {
    if (exact && k < V) {
      // exact k-th largest key: 4 passes of 8-bit digits, most significant first
      uint32_t prefix = 0u, pmask = 0u;
      int kr = k;
      for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = tid; i < 256; i += SMP_THREADS) hist[i] = 0u;
        __syncthreads();
        for (int i = tid; i < V; i += SMP_THREADS) {
          const uint32_t key = okey(sval(i));
          if ((key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (tid == 0) {
          int cum = 0, d = 255;
          for (; d > 0; --d) {
            if (cum + (int)hist[d] >= kr) break;
            cum += (int)hist[d];
          }
          kr -= cum;
          s_thr = prefix | ((uint32_t)d << shift);
        }
        __syncthreads();
        prefix = s_thr;
        pmask |= 255u << shift;
        __syncthreads();
      }
      thr = prefix;
    }
    // ---- collect candidates (scaled key >= thr) into LDS
    if (tid == 0) s_cnt = 0;
    __syncthreads();
    for (int i = tid; i < V; i += SMP_THREADS) {
      const uint32_t key = okey(sval(i));
      if (key >= thr) {
        const int c = atomicAdd(&s_cnt, 1);
        if (c < SMP_CMAX) cand[c] = ((unsigned long long)key << 32) | (unsigned)i;
      }
    }
    __syncthreads();
    if (s_cnt <= SMP_CMAX || exact) break;
    exact = true;  // the bound admitted too many: exact select, then collect again
    __syncthreads();
  }
  const int cnt = min(s_cnt, SMP_CMAX);
  int n2 = 64;
  while (n2 < cnt) n2 <<= 1;
  for (int i = cnt + tid; i < n2; i += SMP_THREADS) cand[i] = 0ull;
  __syncthreads();
  // value desc, ties index desc: read backwards this is torch.sort's (stable) ascending order,
  // which decides which tied ids TopPLogitsWarper removes first
  bitonic_desc(cand, n2);

  if (tid == 0) {
    // top-k: keep every candidate >= the k-th value (ties kept, as `scores < kth` removes)
    int nk = cnt;
    if (k < V && cnt >= k) {
      const uint32_t kth = (uint32_t)(cand[k - 1] >> 32);
      nk = k;
      while (nk < cnt && (uint32_t)(cand[nk] >> 32) == kth) ++nk;
    }
    const float mx = okey_inv((uint32_t)(cand[0] >> 32));
    float z = 0.f;
    for (int i = 0; i < nk; ++i) z += expf(okey_inv((uint32_t)(cand[i] >> 32)) - mx);
    // top-p over the ascending order: drop while the cumulative probability <= 1 - p,
    // never the largest
    int nkeep = nk;
    if (a.top_p < 1.0f) {
      float cum = 0.f;
      int first_kept = 0;  // in ascending order: index nk-1-i
      for (int i = nk - 1; i >= 1; --i) {
        cum += expf(okey_inv((uint32_t)(cand[i] >> 32)) - mx) / z;
        if (cum <= 1.0f - a.top_p) first_kept = nk - i;
        else break;
      }
      nkeep = nk - first_kept;
    }
    float z2 = 0.f;
    for (int i = 0; i < nkeep; ++i) z2 += expf(okey_inv((uint32_t)(cand[i] >> 32)) - mx);
    const int step = a.step ? a.step[b] : a.step0;
    const float u = (a.row_seed ? rng_uniform(a.row_seed[b], 0, step) : rng_uniform(a.seed, b, step)) * z2;
    float acc = 0.f;
    int pick = nkeep - 1;
    for (int i = 0; i < nkeep; ++i) {
      acc += expf(okey_inv((uint32_t)(cand[i] >> 32)) - mx);
      if (acc > u) { pick = i; break; }
    }
    const int tok = (int)(uint32_t)cand[pick];
    if (a.probs) {
      for (int i = 0; i < nkeep; ++i) {
        const int id = (int)(uint32_t)cand[i];
        a.probs[(size_t)b * a.ldl + id] = expf(okey_inv((uint32_t)(cand[i] >> 32)) - mx) / z2;
      }
    }
    if (a.out_part_idx) {
      a.out_part_val[(size_t)b * a.part_stride] = 0.f;
      a.out_part_idx[(size_t)b * a.part_stride] = tok;
    }
    if (a.tokens) a.tokens[b] = tok;
  }
}

}  // namespace

void launch_sample(const SampleArgs& a, int B, hipStream_t s) {
  if (dry_record("sample_kernel")) return;
  hipLaunchKernelGGL(sample_kernel, dim3(B), dim3(SMP_THREADS), 0, s, a);
}

}  // namespace tts
