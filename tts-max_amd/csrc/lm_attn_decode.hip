// lm_attn_decode.hip — decode-step attention (one new query row per sequence, GQA 4:1),
// with RoPE of the new q/k and the KV-cache append fused in.
//
// Reference: LlamaAttention.forward (transformers modeling_llama.py:217-281) at decode time:
// apply_rotary_pos_emb in bf16 (:138-160), DynamicCache.update (append), SDPA with
// scale D^-0.5 and flash numerics (p = exp(s - max) in fp32, P rounded to bf16 for P.V,
// fp32 normaliser; see oracle/lm_oracle.py).
//
// MI355X design.  One workgroup = one (sequence, kv head, chunk of SPLIT positions); its
// four waves are the four q heads of the GQA group.  Every K/V byte of the chunk is loaded
// at kernel entry (one HBM round trip), parked in padded LDS tiles, and the math runs
// lane-per-position (scores) and lane-per-dimension (P.V) out of LDS, so there are no
// cross-lane shuffles: the softmax statistics use DPP reductions (VALU speed) instead of
// __shfl_xor, which lowers to ds_bpermute and serialises on LDS latency.  Chunks of one
// sequence are merged later (o_proj prologue or attn_combine_kernel).
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
  __shared__ float ps[G * SPLIT];

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
  // 3. registers -> LDS tiles
#pragma unroll
  for (int i = 0; i < LOADS; ++i) {
    const int q = tid + i * 256, tl = q / CH, c = q % CH, t = t0 + tl;
    if (t < t1 && t != pos) {
      *(u32x4_t*)(Ks + tl * KROW + c * 8) = kr4[i];
      *(u32x4_t*)(Vs + tl * KROW + c * 8) = vr4[i];
    }
  }
  __syncthreads();
  // the new position's k and v to the cache after the barrier (stores before it would be
  // waited for inside it)
  if (pos >= t0 && pos < t1 && tid < D) {
    a.kcache[cbase + (size_t)pos * D + dk] = Ks[(pos - t0) * KROW + dk];
    a.vcache[cbase + (size_t)pos * D + dk] = vx;
  }

  // 4-6. scores (lane = position), chunk softmax statistics, P.V (lane = dimension)
  const int g = wave;
  float m, l;
  attn_chunk_softmax<D, SPLIT>(Ks, qs + g * D, n, a.scale, lane, ps + g * SPLIT, m, l);
  __syncthreads();
  const size_t pidx = ((size_t)row * a.H + kvh * G + g) * a.nsplit + sp;
  attn_chunk_pv_store<D, SPLIT>(Vs, ps + g * SPLIT, n, lane, m, l, a.part_o + pidx * D, a.part_ml + pidx * 2);
}

int decode_split(int D) { return D == 64 ? 128 : 64; }

void launch_attn_decode_step(const AttnArgs& a, hipStream_t s) {
  dim3 grid(a.rows * a.KVH * a.nsplit);
  if (a.D == 64) hipLaunchKernelGGL((attn_decode2_kernel<64, 128>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((attn_decode2_kernel<128, 64>), grid, dim3(256), 0, s, a);
}

// --------------------------------------------------------------------------------------
// attn_decode3: one workgroup per (row, kv head) does the whole decode attention of its
// GQA group and writes the merged bf16 output, so the o_proj that follows streams its
// weights with a plain 4-KiB A row instead of merging chunk partials (that merge read
// 32 KiB of fp32 partials per o_proj workgroup under the weight stream).  16 waves =
// 4 position groups x 4 q heads.  Positions are cut into tiles of T (the old kernel's
// chunk); group cg takes tiles cg, cg+4, ... with an online-softmax rescale across its
// tiles, and the four groups merge through LDS in tile order: for ctx <= 4T the result is
// bit-identical to the chunked kernel + o_proj merge (same chunks, same merge formula).
namespace {
template <int D> struct Dec3 {
  static constexpr int T = 8192 / D;            // positions per tile
  static constexpr int NGRP = 4;                // position groups
  static constexpr int KROW = D + 8;            // bf16 row stride (16-B pad)
  static constexpr int CH = D / 8;              // 16-B chunks per row
  static constexpr int LOADS = T * CH / 256;    // 16-B K (and V) loads per group thread
  static constexpr int PPL = T / 64;            // positions per lane (scores)
  static constexpr int DPL = D / 64;            // dims per lane (P.V)
  static constexpr size_t kv_bytes = (size_t)NGRP * T * KROW * 2;        // K or V tiles
  static constexpr size_t lds = 2 * kv_bytes + G * D * 4 + NGRP * G * T * 2 + D * 2;
};
}  // namespace

template <int D>
__global__ __launch_bounds__(1024) void attn_decode3_kernel(AttnArgs a) {
  using C = Dec3<D>;
  constexpr int T = C::T, KROW = C::KROW, CH = C::CH, LOADS = C::LOADS, PPL = C::PPL, DPL = C::DPL;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* Ks_all = (bf16_t*)smem;
  bf16_t* Vs_all = (bf16_t*)(smem + C::kv_bytes);
  float* qs = (float*)(smem + 2 * C::kv_bytes);
  bf16_t* ps_all = (bf16_t*)(qs + G * D);
  bf16_t* knew = ps_all + C::NGRP * G * T;  // roped k of the new position
  float* comb = (float*)smem;  // after the tile loop: [NGRP][G][D + 2] (reuses the K tiles)

  const int row = blockIdx.x / a.KVH, kvh = blockIdx.x % a.KVH;
  const int slot = a.row_slot[row], pos = a.row_pos[row], ctx = pos + 1;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = wave >> 2, g = wave & 3, gt = tid & 255;  // group, q head, thread in group
  bf16_t* Ks = Ks_all + (size_t)cg * T * KROW;
  bf16_t* Vs = Vs_all + (size_t)cg * T * KROW;
  bf16_t* ps = ps_all + (size_t)cg * G * T;
  const size_t cbase = ((size_t)slot * a.KVH + kvh) * a.max_seq * D;
  const bf16_t* kc = a.kcache + cbase;
  const bf16_t* vc = a.vcache + cbase;
  const int ntiles = (ctx + T - 1) / T;
  const int iters = (ntiles + C::NGRP - 1) / C::NGRP;  // uniform across the workgroup

  // 1. RoPE operands first (threads 0..G*D-1), then this group's first tile of K and V
  constexpr int H2 = D / 2;
  const bf16_t* cosr = a.rope_cos + (size_t)pos * D;
  const bf16_t* sinr = a.rope_sin + (size_t)pos * D;
  const bf16_t* qrow = a.qkv + (size_t)row * a.ld_qkv;
  const bf16_t* kin = qrow + a.H * D + kvh * D;
  const bf16_t* vin = kin + a.KVH * D;
  const int qi = min(tid, G * D - 1), qh = qi / D, qd = qi % D;
  const bf16_t* qv = qrow + (kvh * G + qh) * D;
  const bf16_t qx = qv[qd], qr = qv[qd < H2 ? qd + H2 : qd - H2], qc = cosr[qd], qsn = sinr[qd];
  const int dk = tid % D;
  const bf16_t kx = kin[dk], kr = kin[dk < H2 ? dk + H2 : dk - H2], vx = vin[dk];
  u32x4_t kr4[LOADS], vr4[LOADS];
  auto load_tile = [&](int t) {
    const int t0 = t * T;
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {  // unconditional (clamped position)
      const int q = gt + i * 256, tl = q / CH, c = q % CH;
      const int p = min(t0 + tl, ctx - 1);
      kr4[i] = *(const u32x4_t*)(kc + (size_t)p * D + c * 8);
      vr4[i] = *(const u32x4_t*)(vc + (size_t)p * D + c * 8);
    }
  };
  load_tile(min(cg, ntiles - 1));

  // 2. RoPE (HF apply_rotary_pos_emb in bf16), new k to the cache
  if (tid < G * D) {
    const float rot = (qd < H2) ? -bf2f(qr) : bf2f(qr);
    qs[tid] = rbf(rbf(bf2f(qx) * bf2f(qc)) + rbf(rot * bf2f(qsn)));
  }
  if (tid < D) {
    bf16_t kb;
    const float c = bf2f(cosr[dk]), sn = bf2f(sinr[dk]);
    const float rot = (dk < H2) ? -bf2f(kr) : bf2f(kr);
    kb = f2bf(rbf(rbf(bf2f(kx) * c) + rbf(rot * sn)));
    knew[dk] = kb;
    a.kcache[cbase + (size_t)pos * D + dk] = kb;
    a.vcache[cbase + (size_t)pos * D + dk] = vx;
  }

  // 3. tiles: scores (lane = position), chunk softmax, P.V (lane = dim), online rescale
  float m_run = -INFINITY, l_run = 0.f, o[DPL];
#pragma unroll
  for (int e = 0; e < DPL; ++e) o[e] = 0.f;
  const float* qg = qs + g * D;
  for (int it = 0; it < iters; ++it) {
    const int t = cg + it * C::NGRP;
    const bool live = t < ntiles;  // uniform per group
    const int t0 = t * T, n = live ? min(T, ctx - t0) : 0;
    __syncthreads();  // previous tile's readers are done (and qs is visible)
    if (live) {
#pragma unroll
      for (int i = 0; i < LOADS; ++i) {
        const int q = gt + i * 256, tl = q / CH, c = q % CH, p = t0 + tl;
        if (tl < n && p != pos) {
          *(u32x4_t*)(Ks + tl * KROW + c * 8) = kr4[i];
          *(u32x4_t*)(Vs + tl * KROW + c * 8) = vr4[i];
        }
      }
      if (pos >= t0 && pos < t0 + T && gt < D) {  // the new position (roped k, v) in the tile
        Ks[(pos - t0) * KROW + gt] = knew[gt];
        Vs[(pos - t0) * KROW + gt] = vx;
      }
    }
    __syncthreads();
    if (it + 1 < iters) load_tile(min(t + C::NGRP, ntiles - 1));  // next tile in flight
    if (live) {
      float sc[PPL];
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < PPL; ++j) {
        const int tl = lane + 64 * j;
        float acc = 0.f;
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          const u32x4_t kv = *(const u32x4_t*)(Ks + tl * KROW + c * 8);
          const float4 q0 = *(const float4*)(qg + c * 8);
          const float4 q1 = *(const float4*)(qg + c * 8 + 4);
          acc += q0.x * bf_lo(kv[0]) + q0.y * bf_hi(kv[0]) + q0.z * bf_lo(kv[1]) + q0.w * bf_hi(kv[1]) +
                 q1.x * bf_lo(kv[2]) + q1.y * bf_hi(kv[2]) + q1.z * bf_lo(kv[3]) + q1.w * bf_hi(kv[3]);
        }
        sc[j] = (tl < n) ? acc * a.scale : -INFINITY;
        mx = fmaxf(mx, sc[j]);
      }
      const float m = wave_max_dpp(mx);  // this tile's max (the chunk statistics)
      float lsum = 0.f;
#pragma unroll
      for (int j = 0; j < PPL; ++j) {
        const float p = (lane + 64 * j < n) ? expf(sc[j] - m) : 0.f;
        lsum += p;
        ps[g * T + lane + 64 * j] = f2bf(p);
      }
      const float l = wave_sum_dpp(lsum);
      float ot[DPL];
#pragma unroll
      for (int e = 0; e < DPL; ++e) ot[e] = 0.f;
      const bf16_t* pg = ps + g * T;
      // (ps written by this wave only: a wave-local LDS round trip needs no barrier)
#pragma unroll 4
      for (int tl = 0; tl < n; ++tl) {
        const float p = bf2f(pg[tl]);
        if constexpr (DPL == 1) {
          ot[0] += p * bf2f(Vs[tl * KROW + lane]);
        } else {
          const uint32_t v2 = *(const uint32_t*)(Vs + tl * KROW + 2 * lane);
          ot[0] += p * bf_lo(v2);
          ot[1] += p * bf_hi(v2);
        }
      }
      if (it == 0) {
        m_run = m; l_run = l;
#pragma unroll
        for (int e = 0; e < DPL; ++e) o[e] = ot[e];
      } else {  // online rescale across this group's tiles (ctx > 4T only)
        const float mn = fmaxf(m_run, m), f0 = expf(m_run - mn), f1 = expf(m - mn);
        l_run = l_run * f0 + l * f1;
#pragma unroll
        for (int e = 0; e < DPL; ++e) o[e] = o[e] * f0 + ot[e] * f1;
        m_run = mn;
      }
    }
  }
  // 4. merge the four groups (tile order), as attn_combine / the o_proj merge did
  __syncthreads();
  float* cm = comb + (size_t)(cg * G + g) * (D + 2);
#pragma unroll
  for (int e = 0; e < DPL; ++e) cm[lane * DPL + e] = o[e];
  if (lane == 0) { cm[D] = m_run; cm[D + 1] = l_run; }
  __syncthreads();
  if (cg == 0) {
    const int ng = min(ntiles, C::NGRP);
    float M = -INFINITY;
    for (int c = 0; c < ng; ++c) M = fmaxf(M, comb[(size_t)(c * G + g) * (D + 2) + D]);
    float L = 0.f;
    for (int c = 0; c < ng; ++c) {
      const float* q = comb + (size_t)(c * G + g) * (D + 2);
      L += q[D + 1] * expf(q[D] - M);
    }
    const float il = 1.0f / L;
    float r[DPL];
#pragma unroll
    for (int e = 0; e < DPL; ++e) r[e] = 0.f;
    for (int c = 0; c < ng; ++c) {
      const float* q = comb + (size_t)(c * G + g) * (D + 2);
      const float f = expf(q[D] - M) * il;
#pragma unroll
      for (int e = 0; e < DPL; ++e) r[e] += q[lane * DPL + e] * f;
    }
    const int h = kvh * G + g;
    bf16_t* out = a.out + (size_t)row * a.H * D + h * D + lane * DPL;
#pragma unroll
    for (int e = 0; e < DPL; ++e) out[e] = f2bf(r[e]);
  }
}

void launch_attn_decode_merged(const AttnArgs& a, hipStream_t s) {
  dim3 grid(a.rows * a.KVH);
  if (a.D == 64)
    hipLaunchKernelGGL((attn_decode3_kernel<64>), grid, dim3(1024), Dec3<64>::lds, s, a);
  else
    hipLaunchKernelGGL((attn_decode3_kernel<128>), grid, dim3(1024), Dec3<128>::lds, s, a);
}

}  // namespace tts
