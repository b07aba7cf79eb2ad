// lm_attn.hip — SpeechLM attention for decode and prefill (GQA 4:1, causal, KV cache).
//
// Reference: LlamaAttention.forward (transformers modeling_llama.py:217-281) with
// apply_rotary_pos_emb (:138-160: q*cos + rotate_half(q)*sin, every op rounded to bf16,
// cos/sin materialised in bf16), DynamicCache.update (append), and the SDPA interface
// (scale = head_dim^-0.5, fp32 softmax).  The prompt rows of a prefill and the one new row
// of each sequence in a decode step are the same "query row" here: a row has a KV slot and
// an absolute position and attends to positions 0..pos of its slot (ragged batching: no
// padding, each sequence computed as in a batch-1 generate).
//
// MI355X layout: the KV cache of a layer is [slot][kv_head][max_seq][head_dim] bf16, so the
// K/V rows a workgroup streams are contiguous; a wave reads 64/(D/8) positions x D bf16 =
// 1 KiB per instruction.  Long contexts are split into chunks (split-K over positions) to
// put enough workgroups on the 256 CUs at batch 1; the chunks are merged by
// attn_combine_kernel with the usual (max, sum) rescaling.
#include "hip_common.h"
#include "lm_kernels.h"

namespace tts {

constexpr int GQA = 4;  // q heads per kv head (TTS-1: 32/8, TTS-1-Max: 32/8)

template <int D>
TTS_DEV float rope_elem(const bf16_t* v, int d, const bf16_t* cosr, const bf16_t* sinr) {
  constexpr int H2 = D / 2;
  const float c = bf2f(cosr[d]), s = bf2f(sinr[d]);
  const float x = bf2f(v[d]);
  const float rot = (d < H2) ? -bf2f(v[d + H2]) : bf2f(v[d - H2]);
  return rbf(rbf(x * c) + rbf(rot * s));
}

// Prefill: rope q -> q_rot, rope k and append k, v into the cache for every row.
template <int D>
__global__ void rope_append_kernel(AttnArgs a) {
  const int row = blockIdx.x;
  const int slot = a.row_slot[row], pos = a.row_pos[row];
  const bf16_t* base = a.qkv + (size_t)row * a.ld_qkv;
  const bf16_t* cosr = a.rope_cos + (size_t)pos * D;
  const bf16_t* sinr = a.rope_sin + (size_t)pos * D;
  const int HD = a.H * D, KD = a.KVH * D;
  for (int i = threadIdx.x; i < HD + 2 * KD; i += blockDim.x) {
    if (i < HD) {
      const int h = i / D, d = i % D;
      a.q_rot[(size_t)row * HD + i] = f2bf(rope_elem<D>(base + h * D, d, cosr, sinr));
    } else if (i < HD + KD) {
      const int j = i - HD, h = j / D, d = j % D;
      const size_t off = (((size_t)slot * a.KVH + h) * a.max_seq + pos) * D + d;
      a.kcache[off] = f2bf(rope_elem<D>(base + HD + h * D, d, cosr, sinr));
    } else {
      const int j = i - HD - KD, h = j / D, d = j % D;
      const size_t off = (((size_t)slot * a.KVH + h) * a.max_seq + pos) * D + d;
      a.vcache[off] = base[HD + KD + j];
    }
  }
}

template <int D, bool FUSED>
__global__ __launch_bounds__(256) void attn_kernel(AttnArgs a) {
  constexpr int LPP = D / 8;     // lanes per position: 16 B of K/V each
  constexpr int PPW = 64 / LPP;  // positions per wave-instruction
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int row = blockIdx.x / a.KVH, kvh = blockIdx.x % a.KVH, sp = blockIdx.y;
  const int slot = a.row_slot[row], pos = a.row_pos[row], ctx = pos + 1;
  const int t0 = sp * a.split;
  if (t0 >= ctx) return;
  const int t1 = min(t0 + a.split, ctx);
  const int n = t1 - t0;
  float* qs = sm;             // [GQA][D]
  float* kn = qs + GQA * D;   // [D] new k (roped)
  float* vn = kn + D;         // [D] new v
  float* s = vn + D;          // [GQA][split] scores -> probabilities
  float* ml = s + GQA * a.split;  // [GQA][2]
  float* ored = ml + 2 * GQA;     // [4 waves][GQA][D]
  const size_t cbase = ((size_t)slot * a.KVH + kvh) * a.max_seq * D;
  const bf16_t* kc = a.kcache + cbase;
  const bf16_t* vc = a.vcache + cbase;
  const bool has_new = FUSED && pos >= t0 && pos < t1;
  const bf16_t* cosr = a.rope_cos + (size_t)pos * D;
  const bf16_t* sinr = a.rope_sin + (size_t)pos * D;

  for (int i = threadIdx.x; i < GQA * D; i += blockDim.x) {
    const int g = i / D, d = i % D, h = kvh * GQA + g;
    if constexpr (FUSED) qs[i] = rope_elem<D>(a.qkv + (size_t)row * a.ld_qkv + h * D, d, cosr, sinr);
    else qs[i] = bf2f(a.q_rot[(size_t)row * a.H * D + h * D + d]);
  }
  if (has_new) {
    const bf16_t* kin = a.qkv + (size_t)row * a.ld_qkv + a.H * D + kvh * D;
    const bf16_t* vin = kin + a.KVH * D;
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
      const float kr = rope_elem<D>(kin, d, cosr, sinr);
      kn[d] = kr;
      vn[d] = bf2f(vin[d]);
      a.kcache[cbase + (size_t)pos * D + d] = f2bf(kr);
      a.vcache[cbase + (size_t)pos * D + d] = vin[d];
    }
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane % LPP, pg = lane / LPP;
  float qr[GQA][8];
#pragma unroll
  for (int g = 0; g < GQA; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) qr[g][j] = qs[g * D + c * 8 + j];

  // ---- scores
  for (int tb = t0 + wave * PPW; tb < t1; tb += 4 * PPW) {
    const int t = tb + pg;
    const bool valid = t < t1;
    float kv[8];
    if (valid && has_new && t == pos) {
#pragma unroll
      for (int j = 0; j < 8; ++j) kv[j] = kn[c * 8 + j];
    } else if (valid) {
      const u32x4_t v = *(const u32x4_t*)(kc + (size_t)t * D + c * 8);
#pragma unroll
      for (int q = 0; q < 4; ++q) { kv[2 * q] = bf_lo(v[q]); kv[2 * q + 1] = bf_hi(v[q]); }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) kv[j] = 0.f;
    }
    float part[GQA];
#pragma unroll
    for (int g = 0; g < GQA; ++g) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += qr[g][j] * kv[j];
      part[g] = acc;
    }
#pragma unroll
    for (int o = 1; o < LPP; o <<= 1)
#pragma unroll
      for (int g = 0; g < GQA; ++g) part[g] += __shfl_xor(part[g], o, 64);
    if (c == 0 && valid) {
#pragma unroll
      for (int g = 0; g < GQA; ++g) s[g * a.split + (t - t0)] = part[g] * a.scale;
    }
  }
  __syncthreads();

  // ---- softmax statistics of this chunk (one wave per q head)
  for (int g = wave; g < GQA; g += 4) {
    float m = -INFINITY;
    for (int i = lane; i < n; i += 64) m = fmaxf(m, s[g * a.split + i]);
    m = wave_max(m);
    // flash numerics: the normaliser sums the fp32 p, the P.V product sees p rounded to
    // bf16 (torch's CPU flash kernel and FA2 both feed bf16 P to the second GEMM)
    float l = 0.f;
    for (int i = lane; i < n; i += 64) {
      const float p = expf(s[g * a.split + i] - m);
      s[g * a.split + i] = rbf(p);
      l += p;
    }
    l = wave_sum(l);
    if (lane == 0) { ml[2 * g] = m; ml[2 * g + 1] = l; }
  }
  __syncthreads();

  // ---- P.V
  float o[GQA][8];
#pragma unroll
  for (int g = 0; g < GQA; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) o[g][j] = 0.f;
  for (int tb = t0 + wave * PPW; tb < t1; tb += 4 * PPW) {
    const int t = tb + pg;
    if (t < t1) {
      float vv[8];
      if (has_new && t == pos) {
#pragma unroll
        for (int j = 0; j < 8; ++j) vv[j] = vn[c * 8 + j];
      } else {
        const u32x4_t v = *(const u32x4_t*)(vc + (size_t)t * D + c * 8);
#pragma unroll
        for (int q = 0; q < 4; ++q) { vv[2 * q] = bf_lo(v[q]); vv[2 * q + 1] = bf_hi(v[q]); }
      }
#pragma unroll
      for (int g = 0; g < GQA; ++g) {
        const float p = s[g * a.split + (t - t0)];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[g][j] += p * vv[j];
      }
    }
  }
#pragma unroll
  for (int off = LPP; off < 64; off <<= 1)
#pragma unroll
    for (int g = 0; g < GQA; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) o[g][j] += __shfl_xor(o[g][j], off, 64);
  if (pg == 0) {
#pragma unroll
    for (int g = 0; g < GQA; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) ored[(wave * GQA + g) * D + c * 8 + j] = o[g][j];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < GQA * D; i += blockDim.x) {
    const int g = i / D, d = i % D, h = kvh * GQA + g;
    const float sum = ored[(0 * GQA + g) * D + d] + ored[(1 * GQA + g) * D + d] +
                      ored[(2 * GQA + g) * D + d] + ored[(3 * GQA + g) * D + d];
    const size_t pidx = ((size_t)row * a.H + h) * a.nsplit + sp;
    a.part_o[pidx * D + d] = sum;
    if (d == 0) { a.part_ml[pidx * 2] = ml[2 * g]; a.part_ml[pidx * 2 + 1] = ml[2 * g + 1]; }
  }
}

template <int D>
__global__ void attn_combine_kernel(AttnArgs a) {
  const int row = blockIdx.x / a.H, h = blockIdx.x % a.H;
  const int ctx = a.row_pos[row] + 1;
  const int ns = (ctx + a.split - 1) / a.split;
  const size_t pbase = ((size_t)row * a.H + h) * a.nsplit;
  float m = -INFINITY;
  for (int i = 0; i < ns; ++i) m = fmaxf(m, a.part_ml[(pbase + i) * 2]);
  float l = 0.f;
  for (int i = 0; i < ns; ++i) l += a.part_ml[(pbase + i) * 2 + 1] * expf(a.part_ml[(pbase + i) * 2] - m);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float o = 0.f;
    for (int i = 0; i < ns; ++i) o += a.part_o[(pbase + i) * D + d] * expf(a.part_ml[(pbase + i) * 2] - m);
    a.out[(size_t)row * a.H * D + h * D + d] = f2bf(o / l);
  }
}

static size_t attn_lds_bytes(const AttnArgs& a) {
  return (size_t)(GQA * a.D + 2 * a.D + GQA * a.split + 2 * GQA + 4 * GQA * a.D) * sizeof(float);
}

void launch_rope_append(const AttnArgs& a, hipStream_t s) {
  if (a.D == 64) hipLaunchKernelGGL(rope_append_kernel<64>, dim3(a.rows), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(rope_append_kernel<128>, dim3(a.rows), dim3(256), 0, s, a);
}

void launch_attn_decode(const AttnArgs& a, bool fused, hipStream_t s) {
  dim3 grid(a.rows * a.KVH, a.nsplit);
  const size_t lds = attn_lds_bytes(a);
  if (a.D == 64) {
    if (fused) hipLaunchKernelGGL((attn_kernel<64, true>), grid, dim3(256), lds, s, a);
    else hipLaunchKernelGGL((attn_kernel<64, false>), grid, dim3(256), lds, s, a);
  } else {
    if (fused) hipLaunchKernelGGL((attn_kernel<128, true>), grid, dim3(256), lds, s, a);
    else hipLaunchKernelGGL((attn_kernel<128, false>), grid, dim3(256), lds, s, a);
  }
}

// The same merge with every chunk statistic and partial of a (row, head) issued at once
// (NSX chunks, clamped; a runtime-length loop would serialise one L2 round trip per chunk
// and pass): one wave per head, four heads per workgroup.  Same formula and order as
// attn_combine_kernel, so the bits are identical.
template <int D, int NSX>
__global__ __launch_bounds__(256) void attn_combine_wide_kernel(AttnArgs a) {
  constexpr int DPL = D / 64;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rh = blockIdx.x * 4 + wave;  // (row, head)
  if (rh >= a.rows * a.H) return;
  const int row = rh / a.H, h = rh % a.H;
  const int ctx = a.row_pos[row] + 1;
  const int ns = (ctx + a.split - 1) / a.split;
  const size_t pbase = ((size_t)row * a.H + h) * a.nsplit;
  float2 ml[NSX];
  float ov[NSX][DPL];
#pragma unroll
  for (int i = 0; i < NSX; ++i) {
    const size_t pi = pbase + min(i, ns - 1);
    ml[i] = *(const float2*)(a.part_ml + pi * 2);
#pragma unroll
    for (int e = 0; e < DPL; ++e) ov[i][e] = a.part_o[pi * D + lane + 64 * e];
  }
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < NSX; ++i) if (i < ns) m = fmaxf(m, ml[i].x);
  float l = 0.f;
#pragma unroll
  for (int i = 0; i < NSX; ++i) if (i < ns) l += ml[i].y * expf(ml[i].x - m);
#pragma unroll
  for (int e = 0; e < DPL; ++e) {
    float o = 0.f;
#pragma unroll
    for (int i = 0; i < NSX; ++i) if (i < ns) o += ov[i][e] * expf(ml[i].x - m);
    a.out[(size_t)row * a.H * D + h * D + lane + 64 * e] = f2bf(o / l);
  }
}

void launch_attn_combine(const AttnArgs& a, hipStream_t s) {
  // (every row's chunk count <= 8 whenever the allocated chunk count is)
  if (a.nsplit <= 8) {
    const dim3 g((a.rows * a.H + 3) / 4);
    if (a.D == 64) hipLaunchKernelGGL((attn_combine_wide_kernel<64, 8>), g, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((attn_combine_wide_kernel<128, 8>), g, dim3(256), 0, s, a);
    return;
  }
  if (a.D == 64) hipLaunchKernelGGL(attn_combine_kernel<64>, dim3(a.rows * a.H), dim3(64), 0, s, a);
  else hipLaunchKernelGGL(attn_combine_kernel<128>, dim3(a.rows * a.H), dim3(128), 0, s, a);
}

}  // namespace tts
