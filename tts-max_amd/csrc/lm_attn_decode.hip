// lm_attn_decode.hip — decode-step attention (one new query row per sequence, GQA 4:1),
// with RoPE of the new q/k and the KV-cache append fused in.
//
// Reference: LlamaAttention.forward (transformers modeling_llama.py:217-281) at decode time:
// apply_rotary_pos_emb in bf16 (:138-160), DynamicCache.update (append), SDPA with
// scale D^-0.5 and flash numerics (p = exp(s - max) in fp32, P rounded to bf16 for P.V,
// fp32 normaliser; see oracle/lm_oracle.py).
//
// MI355X design.  One workgroup = one (sequence, kv head, chunk of SPLIT positions).  Every
// K/V byte of the chunk is loaded at kernel entry by its four waves (one HBM round trip) and
// parked in padded LDS tiles; then one wave computes the four q heads of the GQA group on
// the matrix cores (lm_attn_chunk.h: S^T = K.Q^T, chunk softmax, O^T = V^T.P^T with the V
// tile read transposed by ds_read_b64_tr_b16).  Chunks of one sequence are merged later
// (o_proj prologue or attn_combine_kernel).
#include "hip_common.h"
#include "lm_kernels.h"
#include "lm_attn_chunk.h"

namespace tts {

namespace {
constexpr int G = 4;  // q heads per kv head = waves per workgroup

}  // namespace

template <int D, int SPLIT>
__global__ __launch_bounds__(256) void attn_decode2_kernel(AttnArgs a) {
  constexpr int KROW = D + 8;                 // bf16 row stride: 16-B pad, conflict-free b128
  constexpr int CH = D / 8;                   // 16-B chunks per row
  constexpr int LOADS = SPLIT * CH / 256;     // 16-B loads per thread per tile
  constexpr int PPL = SPLIT / 64;             // positions per lane (scores)
  constexpr int DPL = D / 64;                 // dims per lane (P.V)
  __shared__ __attribute__((aligned(16))) bf16_t Ks[SPLIT * KROW];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[SPLIT * KROW];
  __shared__ __attribute__((aligned(16))) float qs[G * D];

  const int nrk = a.rows * a.KVH, nb = nrk * a.nsplit;
  if ((int)blockIdx.x >= nb) return;
  const int rk = blockIdx.x % nrk, sp = blockIdx.x / nrk;
  const int row = rk / a.KVH, kvh = rk % a.KVH;
  const int slot = a.row_slot[row], pos = a.row_pos[row], ctx = pos + 1;
  const int t0 = sp * SPLIT;
  if (t0 >= ctx) return;
  const int t1 = min(t0 + SPLIT, ctx);
  const int n = t1 - t0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const size_t cbase = ((size_t)slot * a.KVH + kvh) * a.max_seq * D;
  const bf16_t* kc = a.kcache + cbase;
  const bf16_t* vc = a.vcache + cbase;

  // 1. RoPE operands first, then the whole chunk's K and V: vmcnt retires in issue order,
  //    so the rotation below waits only for its own operands, not for the K/V stream.
  constexpr int QPT = G * D / 256;  // query elements per thread
  constexpr int H2 = D / 2;
  const bf16_t* cosr = a.rope_cos + (size_t)pos * D;
  const bf16_t* sinr = a.rope_sin + (size_t)pos * D;
  const bf16_t* qrow = a.qkv + (size_t)row * a.ld_qkv;
  const bf16_t* kin = qrow + a.H * D + kvh * D;
  const bf16_t* vin = kin + a.KVH * D;
  bf16_t qx[QPT], qr[QPT], qc[QPT], qsn[QPT];
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    const int i = tid + 256 * j, g = i / D, d = i % D;
    const bf16_t* v = qrow + (kvh * G + g) * D;
    qx[j] = v[d];
    qr[j] = v[d < H2 ? d + H2 : d - H2];
    qc[j] = cosr[d];
    qsn[j] = sinr[d];
  }
  const int dk = tid % D;  // new-position k/v element of this thread (used by tid < D)
  const bf16_t kx = kin[dk], kr = kin[dk < H2 ? dk + H2 : dk - H2], vx = vin[dk];
  u32x4_t kr4[LOADS], vr4[LOADS];
#pragma unroll
  for (int i = 0; i < LOADS; ++i) {  // unconditional (clamped row): no branch around loads
    const int q = tid + i * 256, tl = q / CH, c = q % CH;
    const int t = (t0 + tl < t1) ? t0 + tl : t0;
    kr4[i] = *(const u32x4_t*)(kc + (size_t)t * D + c * 8);
    vr4[i] = *(const u32x4_t*)(vc + (size_t)t * D + c * 8);
  }
  // 2. RoPE (HF apply_rotary_pos_emb in bf16: q*cos + rotate_half(q)*sin, each op rounded)
#pragma unroll
  for (int j = 0; j < QPT; ++j) {
    const int i = tid + 256 * j, d = i % D;
    const float rot = (d < H2) ? -bf2f(qr[j]) : bf2f(qr[j]);
    qs[i] = rbf(rbf(bf2f(qx[j]) * bf2f(qc[j])) + rbf(rot * bf2f(qsn[j])));
  }
  if (pos >= t0 && pos < t1 && tid < D) {  // the new position: roped k and v to cache + LDS
    const float c = bf2f(qc[0]), sn = bf2f(qsn[0]);  // (tid < D: element 0 is dimension dk)
    const float rot = (dk < H2) ? -bf2f(kr) : bf2f(kr);
    const bf16_t kb = f2bf(rbf(rbf(bf2f(kx) * c) + rbf(rot * sn)));
    Ks[(pos - t0) * KROW + dk] = kb;
    Vs[(pos - t0) * KROW + dk] = vx;
  }
  // 3. registers -> LDS tiles (rows past the chunk's end zeroed: their p is 0 and 0 * NaN
  //    from stale LDS would poison P.V)
  const u32x4_t z4 = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < LOADS; ++i) {
    const int q = tid + i * 256, tl = q / CH, c = q % CH, t = t0 + tl;
    if (t != pos) {
      *(u32x4_t*)(Ks + tl * KROW + c * 8) = t < t1 ? kr4[i] : z4;
      *(u32x4_t*)(Vs + tl * KROW + c * 8) = t < t1 ? vr4[i] : z4;
    }
  }
  __syncthreads();
  // the new position's k and v to the cache after the barrier (stores before it would be
  // waited for inside it)
  if (pos >= t0 && pos < t1 && tid < D) {
    a.kcache[cbase + (size_t)pos * D + dk] = Ks[(pos - t0) * KROW + dk];
    a.vcache[cbase + (size_t)pos * D + dk] = vx;
  }

  // 4-6. scores, chunk softmax statistics and P.V of the four q heads on the matrix cores
  if (wave == 0) {
    const size_t pidx = ((size_t)row * a.H + kvh * G) * a.nsplit + sp;
    attn_chunk_mfma<D, SPLIT>(Ks, Vs, qs, n, a.scale, lane, a.part_o + pidx * D, a.part_ml + pidx * 2,
                              a.nsplit * D, a.nsplit * 2);
  }
}

int decode_split(int D) { return D == 64 ? 128 : 64; }

void launch_attn_decode_step(const AttnArgs& a, hipStream_t s) {
  dim3 grid(a.rows * a.KVH * a.nsplit);
  if (a.D == 64) hipLaunchKernelGGL((attn_decode2_kernel<64, 128>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((attn_decode2_kernel<128, 64>), grid, dim3(256), 0, s, a);
}

}  // namespace tts
