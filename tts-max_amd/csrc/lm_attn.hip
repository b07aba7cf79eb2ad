// lm_attn.hip — SpeechLM attention for decode and prefill (GQA 4:1, causal, KV cache), on
// the matrix cores.
//
// Reference: LlamaAttention.forward (transformers modeling_llama.py:217-281) with
// apply_rotary_pos_emb (:138-160: q*cos + rotate_half(q)*sin, every op rounded to bf16,
// cos/sin materialised in bf16), DynamicCache.update (append), and SDPA (scale
// head_dim^-0.5, fp32 softmax; bf16 probabilities into P.V, fp32 normaliser: the flash
// numerics of oracle/lm_oracle.py:95-107).  The prompt rows of a prefill and the one new row
// of each sequence in a decode step are the same "query row": a row has a KV slot and an
// absolute position and attends to positions 0..pos of its slot (ragged batching: no
// padding, each sequence computed as in a batch-1 generate).
//
// KV cache of a layer (lm_attn_core.h): K [slot][kv head][S][D], V^T [slot][kv head] in 16 x 32 tiles —
// the A-operand layouts of S^T = K.Q^T and O^T = V^T.P^T on v_mfma_f32_16x16x32_bf16, so the
// kernels load every fragment straight into registers.  Both kernels write the attention
// output (bf16, [rows][H*D]) directly: no chunk partials, no merge pass.
#include <stdexcept>

#include "hip_common.h"
#include "lm_kernels.h"
#include "lm_attn_core.h"

namespace tts {

template <int D>
TTS_DEV float rope_at(const bf16_t* v, int d, const bf16_t* cosr, const bf16_t* sinr) {
  constexpr int H2 = D / 2;
  return rope_elem(v[d], v[d < H2 ? d + H2 : d - H2], d < H2, bf2f(cosr[d]), bf2f(sinr[d]));
}

// Prefill: rope q -> q_rot, rope k -> K rows, v -> V^T columns.  Workgroups [0, rows): the
// rope of one row's q and k.  Workgroups [rows, rows + nblocks): the V^T columns of one query
// block (up to 16 consecutive positions of one sequence, a.blocks) — a row's V lands in a
// different 64-B row of every V^T tile, so writing it row by row stored 2 B per 64-B segment
// (a 32-prompt prefill's appends took 38 us a layer, most of it this write amplification);
// the block's V rows are staged in LDS and written with consecutive lanes on consecutive
// positions (16 positions = 32 contiguous bytes of a V^T tile row).
template <int D>
__global__ __launch_bounds__(256) void rope_append_kernel(AttnArgs a) {
  constexpr int VLD = 8 * D + 8;  // staged V row stride (bf16, KVH <= 8): +16 B spreads the rows' banks
  __shared__ __attribute__((aligned(16))) bf16_t vs[16 * VLD];
  const int HD = a.H * D, KD = a.KVH * D;
  if ((int)blockIdx.x < a.rows) {
    const int row = blockIdx.x;
    const int slot = a.row_slot[row], pos = a.row_pos[row];
    const bf16_t* base = a.qkv + (size_t)row * a.ld_qkv;
    const bf16_t* cosr = a.rope_cos + (size_t)pos * D;
    const bf16_t* sinr = a.rope_sin + (size_t)pos * D;
    for (int i = threadIdx.x; i < HD + KD; i += blockDim.x) {
      if (i < HD) {
        const int h = i / D, d = i % D;
        a.q_rot[(size_t)row * HD + i] = f2bf(rope_at<D>(base + h * D, d, cosr, sinr));
      } else {
        const int j = i - HD, h = j / D, d = j % D;
        a.kcache[(((size_t)slot * a.KVH + h) * a.max_seq + pos) * D + d] = f2bf(rope_at<D>(base + HD + h * D, d, cosr, sinr));
      }
    }
    return;
  }
  const int4 blk = a.blocks[blockIdx.x - a.rows];  // {first row, rows, slot, first position}
  const int r0 = blk.x, nr = blk.y, slot = blk.z, p0 = blk.w;
  for (int e = threadIdx.x; e < nr * (KD / 8); e += blockDim.x) {  // the block's V rows, 16 B a thread
    const int rr = e / (KD / 8), c = e - rr * (KD / 8);
    *(u32x4_t*)(vs + rr * VLD + c * 8) = *(const u32x4_t*)(a.qkv + (size_t)(r0 + rr) * a.ld_qkv + HD + KD + c * 8);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < KD * 16; e += blockDim.x) {
    const int j = e >> 4, pl = e & 15, h = j / D, d = j % D;
    if (pl < nr)
      a.vtcache[((size_t)slot * a.KVH + h) * D * a.max_seq + vt_off(a.max_seq, d, p0 + pl)] = vs[pl * VLD + j];
  }
}

// ------------------------------------------------------------------------ decode ------
// One workgroup = one (row, kv head), dec_nw waves (lm_attn_core.h dec_attend): the row's RoPE of
// q / k, the attention over pos + 1 positions, the bf16 output of the group's four heads, and
// the KV append of the new position.
template <int D>
__global__ __launch_bounds__(dec_nw<D>() * 64) void attn_decode_kernel(AttnArgs a) {
  constexpr int PW = dec_pw<D>(), NW = dec_nw<D>();
  using C = DecShape<D, PW>;
  __shared__ __attribute__((aligned(16))) float qs[DEC_G * D];
  __shared__ __attribute__((aligned(16))) bf16_t knew[D];
  __shared__ __attribute__((aligned(16))) bf16_t vnew[D];
  __shared__ __attribute__((aligned(16))) float red[dec_red_floats<D, NW>()];
  const int row = blockIdx.x / a.KVH, kvh = blockIdx.x % a.KVH;
  const int slot = a.row_slot[row], pos = a.row_pos[row], ctx = pos + 1;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const size_t kvbase = ((size_t)slot * a.KVH + kvh) * a.max_seq * D;
  const bf16_t* kc = a.kcache + kvbase;
  const bf16_t* vtc = a.vtcache + kvbase;
  unsigned long long* stp = a.stamps ? a.stamps + 16384 + (size_t)blockIdx.x * 8 : nullptr;
  TTS_STAMP(stp, 0);
  // this wave's first-pass fragments before anything else (vmcnt retires in issue order).
  // Head dim 64 addresses them with 32-bit offsets (the 64-bit ones spilled across the later
  // passes); at 128 the 64-bit form allocates without spills.  (Loading q|k|v and the RoPE
  // terms ahead of the fragments was measured slower again in round 5: 32 rows 10.1 -> 12.5 us,
  // profiles/r5h_ab_32.txt)
  u32x4_t kf[C::MT][C::KS], vf[C::PS][C::DT];
  if (wave * PW < ctx) {
    dec_load_k<D, PW, D == 64>(kc, wave * PW, ctx, lane, kf);
    dec_load_v<D, PW, D == 64>(vtc, a.max_seq, wave * PW, lane, vf);
  }
  // RoPE of the group's q heads and of the new k (HF apply_rotary_pos_emb in bf16)
  const bf16_t* qrow = a.qkv + (size_t)row * a.ld_qkv;
  const bf16_t* cosr = a.rope_cos + (size_t)pos * D;
  const bf16_t* sinr = a.rope_sin + (size_t)pos * D;
  // the group's q | k | v: columns of the qkv row, or sums of a K-sliced launch's partials
  __shared__ __attribute__((aligned(16))) bf16_t raw[DEC_G * D + 2 * D];
  const bf16_t* qsrc = qrow + kvh * DEC_G * D;
  const bf16_t* ksrc = qrow + a.H * D + kvh * D;
  const bf16_t* vsrc = qrow + a.H * D + a.KVH * D + kvh * D;
  if (a.qkv_part) {
    for (int i = tid; i < DEC_G * D + 2 * D; i += NW * 64) {
      const int col = i < DEC_G * D ? kvh * DEC_G * D + i
                    : (i < DEC_G * D + D ? a.H * D + kvh * D + i - DEC_G * D
                                         : a.H * D + a.KVH * D + kvh * D + i - DEC_G * D - D);
      float v = 0.f;
      for (int sl = 0; sl < a.qkv_nsl; ++sl) v += a.qkv_part[((size_t)sl * a.rows + row) * a.ld_qkv + col];
      raw[i] = f2bf(v);
    }
    lds_barrier();
    qsrc = raw;
    ksrc = raw + DEC_G * D;
    vsrc = raw + DEC_G * D + D;
  }
  for (int i = tid; i < DEC_G * D + D; i += NW * 64) {
    if (i < DEC_G * D) {
      const int g = i / D, d = i % D;
      qs[i] = rope_at<D>(qsrc + g * D, d, cosr, sinr);
    } else {
      const int d = i - DEC_G * D;
      knew[d] = f2bf(rope_at<D>(ksrc, d, cosr, sinr));
      vnew[d] = vsrc[d];
    }
  }
  lds_barrier();
  TTS_STAMP(stp, 2);
  dec_attend<D, PW, NW, D == 64>(kc, vtc, a.max_seq, ctx, a.scale, qs, knew, vnew, red, kf, vf,
                              a.out + (size_t)row * a.H * D + kvh * DEC_G * D);
  TTS_STAMP(stp, 3);
  // the new position into the cache, after this workgroup's reads (no other workgroup reads
  // this (slot, kv head))
  if (tid < D) {
    a.kcache[kvbase + (size_t)pos * D + tid] = knew[tid];
    a.vtcache[kvbase + vt_off(a.max_seq, tid, pos)] = vnew[tid];
  }
}

void launch_attn_decode_step(const AttnArgs& a, hipStream_t s) {
  if (dry_record(a.D == 64 ? "attn_decode_kernel<64>" : "attn_decode_kernel<128>")) return;
  const dim3 grid(a.rows * a.KVH);
  if (a.D == 64) hipLaunchKernelGGL((attn_decode_kernel<64>), grid, dim3(dec_nw<64>() * 64), 0, s, a);
  else hipLaunchKernelGGL((attn_decode_kernel<128>), grid, dim3(dec_nw<128>() * 64), 0, s, a);
}

// ----------------------------------------------------------------------- prefill ------
// One workgroup = one block of up to 16 consecutive query rows of one sequence (a.blocks:
// {first row, rows, slot, first position}) x one kv head; wave w = q head kvh*4 + w.  The
// block's 16 queries are the 16 columns of S^T = K.Q^T; keys in steps of 32 with the same
// row permutation as the decode kernel, so P^T feeds O^T = V^T.P^T from the accumulators.
// Two passes over the keys: the causal maximum per query first, then p, l and P.V — the
// reference's global-max numerics.
template <int D>
__global__ __launch_bounds__(256) void attn_prefill_kernel(AttnArgs a) {
  using C = DecShape<D, 32>;  // 32 keys per step: 2 m-tiles of S^T, one k-step of P.V
  const int4 blk = a.blocks[blockIdx.x / a.KVH];
  const int kvh = blockIdx.x % a.KVH;
  const int row0 = blk.x, nrows = blk.y, slot = blk.z, pos0 = blk.w;
  const int tid = threadIdx.x, lane = tid & 63;
  const int h = kvh * DEC_G + __builtin_amdgcn_readfirstlane(tid >> 6);  // this wave's q head
  const int c = lane & 15, g = lane >> 4;
  const int qpos = pos0 + c;   // query column c (columns >= nrows: duplicates, never stored)
  const int qrow = row0 + min(c, nrows - 1);
  const size_t kvbase = ((size_t)slot * a.KVH + kvh) * a.max_seq * D;
  const bf16_t* kc = a.kcache + kvbase;
  const bf16_t* vtc = a.vtcache + kvbase;
  const int kend = pos0 + nrows;  // keys 0 .. kend-1 (causal per column below)
  const int nkb = (kend + 31) / 32;
  bf16x8_t qb[C::KS];
#pragma unroll
  for (int ks = 0; ks < C::KS; ++ks)
    qb[ks] = __builtin_bit_cast(bf16x8_t, *(const u32x4_t*)(a.q_rot + (size_t)qrow * a.H * D + h * D + 32 * ks + 8 * g));
  auto scores = [&](int kb, f32x4_t (&s)[2]) {
    u32x4_t kf[2][C::KS];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int p = min(dec_pos(kb * 32, mt, c), kend - 1);
#pragma unroll
      for (int ks = 0; ks < C::KS; ++ks) kf[mt][ks] = *(const u32x4_t*)(kc + (size_t)p * D + 32 * ks + 8 * g);
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < C::KS; ++ks)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, kf[mt][ks]), qb[ks], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] = (dec_pos(kb * 32, mt, 4 * g + r) <= qpos) ? acc[r] * a.scale : -INFINITY;
      s[mt] = acc;
    }
  };
  float mx = -INFINITY;
  for (int kb = 0; kb < nkb; ++kb) {
    f32x4_t s[2];
    scores(kb, s);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[mt][r]);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float lsum = 0.f;
  f32x4_t o[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt) o[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  for (int kb = 0; kb < nkb; ++kb) {
    u32x4_t vf[1][C::DT];
    const int p0 = kb * 32 + 8 * g;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) vf[0][dt] = *(const u32x4_t*)(vtc + vt_off(a.max_seq, 16 * dt + c, p0));
    f32x4_t s[2];
    scores(kb, s);
    // V elements past the block's last key: zeroed (never-written memory)
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (p0 + e >= kend) vf[0][dt][e >> 1] &= ~(0xffffu << ((e & 1) * 16));
    dec_pv<D, 32>(mx, lsum, s, vf, o);
  }
  lsum += __shfl_xor(lsum, 16, 64);
  lsum += __shfl_xor(lsum, 32, 64);
  if (c < nrows) {
    bf16_t* out = a.out + (size_t)(row0 + c) * a.H * D + h * D;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
      const uint32_t lo = pack_bf2(o[dt][0] / lsum, o[dt][1] / lsum), hi = pack_bf2(o[dt][2] / lsum, o[dt][3] / lsum);
      *(uint2*)(out + 16 * dt + 4 * g) = make_uint2(lo, hi);
    }
  }
}

void launch_rope_append(const AttnArgs& a, hipStream_t s) {
  if (a.KVH > 8) throw std::runtime_error("rope_append: at most 8 kv heads");
  if (a.D == 64) hipLaunchKernelGGL(rope_append_kernel<64>, dim3(a.rows + a.nblocks), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(rope_append_kernel<128>, dim3(a.rows + a.nblocks), dim3(256), 0, s, a);
}

void launch_attn_prefill(const AttnArgs& a, hipStream_t s) {
  const dim3 grid(a.nblocks * a.KVH);
  if (a.D == 64) hipLaunchKernelGGL((attn_prefill_kernel<64>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((attn_prefill_kernel<128>), grid, dim3(256), 0, s, a);
}

}  // namespace tts
