// lm_attn_chunk.h — the per-chunk math of decode attention (scores, chunk softmax
// statistics, P.V), shared by the standalone decode kernel (lm_attn_decode.hip) and the
// attention workgroups fused into the QKV projection launch (lm_gemm_kernel.h), so both
// produce bit-identical chunk partials.
//
// Reference numerics (transformers SDPA at decode, see oracle/lm_oracle.py): scores in
// fp32 from the roped bf16 q / k, p = exp(s - chunk max) in fp32, P rounded to bf16 for
// P.V, fp32 normaliser.  The chunks are merged by the o_proj prologue (or attn_combine).
#pragma once
#include "hip_common.h"

namespace tts {

// One wave = one q head over the chunk's n (<= SPLIT) positions held in LDS (rows of
// D + 8 bf16).  qg: the roped query (fp32, LDS); psg: this head's P row (fp32, LDS,
// written and read by this wave only, so no barrier is needed between the two calls).
template <int D, int SPLIT>
TTS_DEV void attn_chunk_softmax(const bf16_t* Ks, const float* qg, int n, float scale, int lane,
                                float* psg, float& m_out, float& l_out) {
  constexpr int KROW = D + 8, CH = D / 8, PPL = SPLIT / 64;
  float sc[PPL];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < PPL; ++j) {  // lane = position
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
    sc[j] = (tl < n) ? acc * scale : -INFINITY;
    mx = fmaxf(mx, sc[j]);
  }
  const float m = wave_max_dpp(mx);
  float lsum = 0.f;
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const float p = (lane + 64 * j < n) ? expf(sc[j] - m) : 0.f;
    lsum += p;
    psg[lane + 64 * j] = rbf(p);
  }
  m_out = m;
  l_out = wave_sum_dpp(lsum);
}

// P.V for one head (lane = head dimension(s)): the chunk partial o of the lane's dimensions.
template <int D, int SPLIT>
TTS_DEV void attn_chunk_pv(const bf16_t* Vs, const float* pg, int n, int lane, float (&o)[D / 64]) {
  constexpr int KROW = D + 8, DPL = D / 64;
#pragma unroll
  for (int e = 0; e < DPL; ++e) o[e] = 0.f;
#pragma unroll 8
  for (int tl = 0; tl < n; ++tl) {
    const float p = pg[tl];
    if constexpr (DPL == 1) {
      o[0] += p * bf2f(Vs[tl * KROW + lane]);
    } else {
      const uint32_t v2 = *(const uint32_t*)(Vs + tl * KROW + 2 * lane);
      o[0] += p * bf_lo(v2);
      o[1] += p * bf_hi(v2);
    }
  }
}

// ... and stores it with the chunk's (m, l)
template <int D, int SPLIT>
TTS_DEV void attn_chunk_pv_store(const bf16_t* Vs, const float* pg, int n, int lane, float m, float l,
                                 float* part_o, float* part_ml) {
  constexpr int DPL = D / 64;
  float o[DPL];
  attn_chunk_pv<D, SPLIT>(Vs, pg, n, lane, o);
#pragma unroll
  for (int e = 0; e < DPL; ++e) part_o[lane * DPL + e] = o[e];
  if (lane == 0) {
    part_ml[0] = m;
    part_ml[1] = l;
  }
}

// RoPE of one element (HF apply_rotary_pos_emb in bf16: x*cos + rotate_half(x)*sin, each
// op rounded to bf16): x = element d, xr = element d +- D/2 (its rotate_half partner)
TTS_DEV float rope_elem(bf16_t x, bf16_t xr, bool lower_half, float c, float sn) {
  const float rot = lower_half ? -bf2f(xr) : bf2f(xr);
  return rbf(rbf(bf2f(x) * c) + rbf(rot * sn));
}

}  // namespace tts
