// lm_attn_chunk.h — the per-chunk math of decode attention (scores, chunk softmax
// statistics, P.V on the matrix cores), shared by the standalone decode kernel
// (lm_attn_decode.hip) and the attention workgroups fused into the QKV projection launch
// (lm_gemm_kernel.h), so both produce bit-identical chunk partials.
//
// Reference numerics (transformers SDPA at decode, see oracle/lm_oracle.py): scores in
// fp32 from the roped bf16 q / k, p = exp(s - chunk max) in fp32, P rounded to bf16 for
// P.V, fp32 normaliser.  The chunks are merged by the o_proj prologue (or attn_combine).
#pragma once
#include "hip_common.h"

namespace tts {

// One wave computes the chunk for all G = 4 q heads of the kv group on the matrix cores
// (v_mfma_f32_16x16x32_bf16; products of bf16 operands are exact in fp32, so only the
// fp32 summation order differs from a scalar loop):
//   S^T[pos][head] = K . Q^T   A = K rows straight from the LDS tile (16 positions x 32 dims
//                              per fragment, one conflict-free ds_read_b128 per lane),
//                              B = the group's roped q (columns 4..15 duplicate heads 0..3
//                              and are discarded);
//   chunk softmax statistics per head: lanes with (lane & 15) = head hold its 4 x MT x 4
//                              scores; m = max, l = sum of fp32 p = exp(s - m);
//   O^T[dim][head] = V^T . P^T A = V^T by ds_read_b64_tr_b16 (4 positions x 16 dims per
//                              16-lane group, delivered column-major), B = P^T straight from
//                              the S^T accumulators rounded to bf16: k-step ps's element e
//                              of lane group g is position 32 ps + 16 (e >> 2) + 4 g + (e & 3)
//                              on BOTH operands, which is where the accumulators hold it.
// Ks / Vs: the chunk's n (<= SPLIT) rows of D + 8 bf16 (16-B pad), rows n.. SPLIT-1 of Vs
// finite (zeros): their p is 0, and 0 * NaN would poison the sum.  qs: the G heads' roped q
// (fp32 holding bf16 values).  Output: head g's partial o at po + g * o_hstride (D floats)
// and its (m, l) at pml + g * ml_hstride.  Call with the whole wave active (EXEC all ones:
// the transposed read gathers across lanes).
template <int D, int SPLIT>
TTS_DEV void attn_chunk_mfma(const bf16_t* Ks, const bf16_t* Vs, const float* qs, int n, float scale,
                             int lane, float* po, float* pml, int o_hstride, int ml_hstride) {
  typedef __attribute__((ext_vector_type(4))) short v4i16_t;
  typedef __attribute__((address_space(3))) v4i16_t lds_v4i16_t;
  constexpr int KROW = D + 8, MT = SPLIT / 16, KS = D / 32, PS = SPLIT / 32, DT = D / 16;
  const int c = lane & 15, g = lane >> 4, h = c & 3;
  bf16x8_t qb[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const float4 a = *(const float4*)(qs + h * D + 32 * ks + 8 * g);
    const float4 b = *(const float4*)(qs + h * D + 32 * ks + 8 * g + 4);
    const u32x4_t w = {pack_bf2(a.x, a.y), pack_bf2(a.z, a.w), pack_bf2(b.x, b.y), pack_bf2(b.z, b.w)};
    qb[ks] = __builtin_bit_cast(bf16x8_t, w);
  }
  f32x4_t s[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    s[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u32x4_t kf = *(const u32x4_t*)(Ks + (16 * mt + c) * KROW + 32 * ks + 8 * g);
      s[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, kf), qb[ks], s[mt], 0, 0, 0);
    }
  }
  // lane holds S^T[pos 16 mt + 4 g + r][head c]
  float mx = -INFINITY;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = (16 * mt + 4 * g + r < n) ? s[mt][r] * scale : -INFINITY;
      s[mt][r] = v;
      mx = fmaxf(mx, v);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float lsum = 0.f;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = (16 * mt + 4 * g + r < n) ? expf(s[mt][r] - mx) : 0.f;
      lsum += p;
      s[mt][r] = p;
    }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  f32x4_t o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int q = c >> 2, pp = c & 3;  // this lane's address in the transposed read: row q, columns 4 pp..
#pragma unroll
  for (int ps = 0; ps < PS; ++ps) {
    const u32x4_t pw = {pack_bf2(s[2 * ps][0], s[2 * ps][1]), pack_bf2(s[2 * ps][2], s[2 * ps][3]),
                        pack_bf2(s[2 * ps + 1][0], s[2 * ps + 1][1]), pack_bf2(s[2 * ps + 1][2], s[2 * ps + 1][3])};
    const bf16x8_t pb = __builtin_bit_cast(bf16x8_t, pw);
    const bf16_t* v0 = Vs + (32 * ps + 4 * g + q) * KROW + 4 * pp;
    const bf16_t* v1 = v0 + 16 * KROW;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const v4i16_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t*)(v0 + 16 * dt));
      const v4i16_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16_t*)(v1 + 16 * dt));
      typedef __attribute__((ext_vector_type(8))) short v8i16_t;
      const v8i16_t vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, vv), pb, o[dt], 0, 0, 0);
    }
  }
  // lane holds O^T[dim 16 dt + 4 g + r][head c]
  if (c < 4) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
      *(float4*)(po + c * o_hstride + 16 * dt + 4 * g) = make_float4(o[dt][0], o[dt][1], o[dt][2], o[dt][3]);
    if (g == 0) {
      pml[c * ml_hstride] = mx;
      pml[c * ml_hstride + 1] = lsum;
    }
  }
}

// RoPE of one element (HF apply_rotary_pos_emb in bf16: x*cos + rotate_half(x)*sin, each
// op rounded to bf16): x = element d, xr = element d +- D/2 (its rotate_half partner)
TTS_DEV float rope_elem(bf16_t x, bf16_t xr, bool lower_half, float c, float sn) {
  const float rot = lower_half ? -bf2f(xr) : bf2f(xr);
  return rbf(rbf(bf2f(x) * c) + rbf(rot * sn));
}

}  // namespace tts
