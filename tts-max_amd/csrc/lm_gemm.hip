// lm_gemm.hip — weight-streaming bf16 GEMM for the SpeechLM (decode GEMV, batched decode,
// chunked prefill) with fused prologue (RMSNorm) and epilogues (store / residual add /
// SwiGLU / lm_head+repetition-penalty+EOS-mask+argmax).
//
// Reference semantics (transformers LlamaForCausalLM, pinned 4.53.2 by uv.lock:4610):
//   nn.Linear in bf16 = fp32-accumulated dot product rounded once to bf16.
//   LlamaRMSNorm (modeling_llama.py:62-67): fp32 mean(x^2), rsqrt(var+eps), cast to bf16,
//     then weight * x in bf16.
//   LlamaMLP (modeling_llama.py:163-176): down(silu(gate(x)) * up(x)), each op rounded to bf16.
//   Decoder residual (modeling_llama.py:~310-322): residual + h rounded to bf16.
//   lm_head + GenerationMixin._sample (generation/utils.py:2894-2925): logits in bf16,
//     .float(), RepetitionPenaltyLogitsProcessor (logits_process.py:306-413),
//     MinNewTokensLengthLogitsProcessor (:164-236), argmax (first max on ties).
//
// MI355X design: weights are re-laid out at load time into 1 KiB MFMA B-fragment tiles so
// that every wave-instruction streams 1 KiB of contiguous HBM and feeds
// v_mfma_f32_16x16x32_bf16 with no shuffles.  Tile (nt, kt) holds
//   tile[lane*8 + j] = W[nt*16 + (lane & 15)][kt*32 + 8*(lane >> 4) + j]
// and tiles of one n-tile are consecutive along K.  Activations (M <= 64 rows) are the
// A operand; at M = 1 fifteen of the sixteen A rows are zero, which costs nothing because
// the kernel is HBM-bound on the weight stream.
#include <algorithm>
#include <cstdio>
#include <stdexcept>

#include "lm_gemm_kernel.h"

namespace tts {

std::vector<std::string>*& dry_launches() {
  static thread_local std::vector<std::string>* rec = nullptr;
  return rec;
}

// ---------------------------------------------------------------- weight re-layout ----
__global__ void retile_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ t, int N,
                              int K, int nt_mult, int nt_off, StreamPlan p, int units) {
  const int KT = K / 32;
  const long long nchunks = (long long)(N / 16) * KT * 64;
  const int ur = p.ur();
  for (long long c = blockIdx.x * (long long)blockDim.x + threadIdx.x; c < nchunks;
       c += (long long)gridDim.x * blockDim.x) {
    const int lane = (int)(c & 63);
    const long long tile = c >> 6;
    const int kt = (int)(tile % KT);
    const int nt = (int)(tile / KT);
    const int n = nt * 16 + (lane & 15);
    const int k = kt * 32 + 8 * (lane >> 4);
    const u32x4_t v = *(const u32x4_t*)(w + (size_t)n * K + k);
    const long long dtile = plan_tile(p.ng, p.ksplit, p.ku, ur, units, KT, p.kc, nt * nt_mult + nt_off, kt);
    *(u32x4_t*)(t + (size_t)(dtile * 64 + lane) * 8) = v;
  }
}

void launch_retile(const bf16_t* w, bf16_t* t, int N, int K, int N_total, int ng, int num_cu,
                   hipStream_t s, int nt_mult, int nt_off) {
  const StreamPlan p = stream_plan(N_total, K, ng, num_cu);
  const int units = (N_total / 16) / ng;
  long long nchunks = (long long)(N / 16) * (K / 32) * 64;
  int grid = (int)((nchunks + 255) / 256);
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(retile_kernel, dim3(grid), dim3(256), 0, s, w, t, N, K, nt_mult, nt_off, p, units);
}

static bool shape_fits(int c, int KT, int ng) {
  const Shape3& h = kShapes[c];
  return shape_ng2(c) == (ng == 2) && KT % (h.ksplit * h.ku) == 0 && h.waves % h.ksplit == 0;
}

// The stream plan of a matrix (its tile layout and its decode launch).  Chosen from the
// HBM streaming sweeps (scripts/hbm_floor.hip, scripts/wgemm_probe.cpp): one workgroup per
// CU where the units allow it, many waves each with a few KiB in flight, stage-interleaved.
StreamPlan stream_plan(int N, int K, int ng, int num_cu) {
  const int units = (N / 16) / ng;
  const int KT = K / 32;
  int c;
  if (ng == 2) c = 5;
  else if (units >= 4 * num_cu) c = 0;
  else if (K >= 4096) c = 3;
  else c = 2;
  // experiment hook (scripts/wgemm_probe.cpp): TTS_STREAM_PLAN=<shape index>[,grid]
  static const char* forced = getenv("TTS_STREAM_PLAN");
  int fgrid = 0;
  if (forced) {
    int fc = -1;
    sscanf(forced, "%d,%d", &fc, &fgrid);
    if (fc >= 0 && fc < kNumShapes && shape_fits(fc, KT, ng)) c = fc;
  }
  if (!shape_fits(c, KT, ng)) {  // small test shapes
    c = -1;
    for (int t = 0; t < kNumShapes && c < 0; ++t)
      if (shape_fits(t, KT, ng)) c = t;
    if (c < 0) throw std::runtime_error("no stream plan fits K");
  }
  StreamPlan p;
  p.ng = ng;
  p.waves = kShapes[c].waves;
  p.ku = kShapes[c].ku;
  p.ksplit = kShapes[c].ksplit;
  const int upw = p.waves / p.ksplit;
  int grid = (units + upw - 1) / upw;
  // one workgroup per CU (lm_head: rounds of 4 units per workgroup); the argmax partials of
  // EPI_LOGITS hold at most LOGITS_MAX_PARTS workgroups
  const int cap = (fgrid > 0) ? std::min(fgrid, LOGITS_MAX_PARTS) : num_cu;
  p.grid = std::min(grid, cap);
  // between one and two rounds of units per CU, a full grid leaves half the workgroups with
  // one round more than the rest (TTS-1-Max qkv: 384 units on 256 CUs): balance the rounds
  static const bool balance = !(getenv("TTS_BALANCE") && !atoi(getenv("TTS_BALANCE")));
  if (balance && fgrid <= 0 && grid > num_cu && grid < 2 * num_cu) p.grid = (grid + 1) / 2;
  // K chunks of 2048 columns (64 k-tiles) where the shape divides them: at batch 17..32 one
  // chunk of A (32 x 2048 bf16 = 128 KiB) fits LDS where the whole K (8192) does not
  if (K > 2048 && K % 2048 == 0 && (2048 / 32) % (p.ksplit * p.ku) == 0) p.kc = K / 2048;
  return p;
}

static int shape_index(const StreamPlan& p) {
  for (int c = 0; c < kNumShapes; ++c)
    if (kShapes[c].waves == p.waves && kShapes[c].ku == p.ku && kShapes[c].ksplit == p.ksplit &&
        shape_ng2(c) == (p.ng == 2))
      return c;
  return -1;
}

// LDS of one launch: A rows (+16 B per row), split-K partials of the waves with kpart > 0,
// the argmax / RMSNorm-segment scratch, and 64 floats of slack.  Must match the kernel's
// carve-up (wgemm_kernel: red_floats).
size_t wgemm_lds_bytes(int waves, int ksplit, int ng, int M, int Kl, bool a_in_lds) {
  const int mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  const size_t xs = a_in_lds ? (((size_t)M * (Kl + 8) * 2 + 15) & ~(size_t)15) : 0;
  return xs + (size_t)wgemm_red_floats(waves, ksplit, ng, mt, M, Kl) * sizeof(float);
}

static constexpr size_t kLdsBudget = 160 * 1024;

WgemmPlan plan_wgemm(int M, int N, int K, int epi, int num_cu) {
  WgemmPlan p;
  const int ng = (epi == EPI_SWIGLU) ? 2 : 1;
  p.sp = stream_plan(N, K, ng, num_cu);
  p.cfg = shape_index(p.sp);
  p.grid = p.sp.grid;
  const int w = p.sp.waves, ks = p.sp.ksplit;
  p.a_lds = wgemm_lds_bytes(w, ks, ng, M, K, true) <= kLdsBudget;
  // the LDS prologues stage rows in 512-column pieces (LDS-DMA) or registers (also K % 512 ==
  // 0); other widths (small test configs) take A fragments from global memory + a standalone
  // RMSNorm (same canonical sum order: same bits)
  if (K % 512 != 0) p.a_lds = false;
  // experiment hook: TTS_HEAD_GRID=<workgroups> for the lm_head launch (units are walked
  // grid-stride, so any grid covers them; at most LOGITS_MAX_PARTS argmax partials)
  static const int head_grid = getenv("TTS_HEAD_GRID") ? atoi(getenv("TTS_HEAD_GRID")) : 0;
  if (epi == EPI_LOGITS && head_grid > 0) p.grid = std::min(head_grid, LOGITS_MAX_PARTS);
  // Up to 16 rows, a residual projection whose rows do not fit the LDS prologue and whose
  // K-sliced form would run the grid in more than two rounds (TTS-1-Max down, K 14336: 7
  // chunks x 256 workgroups) streams its A fragments from L2 beside the weights (A_GLOBAL
  // ring) instead: at 8 rows 39 -> 23 us.  (TTS-1 down at 16 rows, 4 chunks x 128: the
  // sliced form is faster, 14.5 vs 15.5 us; at 17..32 rows the ring drops to one stage and
  // loses.)  Unsliced also keeps these rows' sums in the batch-1 order.  TTS_AGR=0: off.
  static const bool agr_on = !(getenv("TTS_AGR") && !atoi(getenv("TTS_AGR")));
  if (agr_on && M <= 16 && epi == EPI_RESID && !p.a_lds && p.sp.kc > 1 && p.grid * p.sp.kc > 2 * num_cu)
    return p;  // a_lds = false, unsliced
  // (17..32 rows with A fragments from L2 beside the weight tiles instead of the LDS rows,
  // the RMSNorm in the LDS prologue, and column halves at 17..32 rows were measured slower and
  // removed in round 6: profiles/r4c_ab_agr32.txt, r2_ab_norm32.txt)
  // Residual projections with K chunks run K-sliced from 8 rows on even where the rows fit the
  // LDS prologue (TTS-1's down at 8..9 rows), so the per-row combine normalises each row once
  // for the next QKV launch (lm_engine.cpp, TTS_NORM_ONCE): 8 rows 753 -> 748 us a step; at 2 and 4
  // rows it loses (671 -> 692, 706 -> 713 us; profiles/r6f_ab_slice_*.txt).  Only matrices of
  // four or more K chunks (a down projection): a 2-chunk o_proj (TTS-1-Max, K 4096) must keep the
  // unsliced sum order of the o_proj that rides the 2..16-row QKV launch, so the separate and
  // fused forms give the same bits.  TTS_SLICE_RESID_ROWS=<n> moves the threshold (0: only where
  // the rows do not fit)
  static const int slice_rows = getenv("TTS_SLICE_RESID_ROWS") ? atoi(getenv("TTS_SLICE_RESID_ROWS")) : 8;
  const bool force_slice = slice_rows > 0 && M >= slice_rows && epi == EPI_RESID && p.sp.kc >= 4;
  if ((!p.a_lds || force_slice) && p.sp.kc > 1 && (epi == EPI_STORE || epi == EPI_RESID) &&
      wgemm_lds_bytes(w, ks, ng, M, K / p.sp.kc, true) <= kLdsBudget) {
    p.a_lds = true;
    p.sliced = true;
    // one round of workgroups over all K chunks: each stages its A chunk (up to 128 KiB)
    // once and walks several units grid-stride (tiles are addressed by the layout's rounds,
    // so the launch grid is free).  TTS-1 down at 32 rows: 128 x 4 workgroups in two rounds,
    // each staging 128 KiB of A for 64 KiB of weights -> 64 x 4: 19.5 -> 15.6 us, step
    // 1,228 -> 1,179 us, same ids (profiles/r2_ab_sliced_grid.txt).  TTS_SLICED_GRID=0: off.
    static const bool one_round = !(getenv("TTS_SLICED_GRID") && !atoi(getenv("TTS_SLICED_GRID")));
    if (one_round) p.grid = std::max(1, std::min(p.grid, (num_cu + p.sp.kc - 1) / p.sp.kc));
  }
  // A matrix with at most half a unit per CU (TTS-1 o_proj and down at 1..16 rows: 128 units)
  // streams each unit as two 8-column halves on twice the workgroups: every CU pulls half
  // the bytes.  TTS_CSPLIT=0: off; =2: also at 17..64 rows.
  static const int csplit_mode = getenv("TTS_CSPLIT") ? atoi(getenv("TTS_CSPLIT")) : 1;
  const int units = (N / 16) / ng;
  const int upw = w / ks;
  if (csplit_mode > 0 && (M <= 16 || csplit_mode == 2) && !p.sliced && p.a_lds &&
      (epi == EPI_STORE || epi == EPI_RESID) && p.grid * upw >= units && 2 * units <= num_cu * upw) {
    p.csplit = 2;
    p.grid = (2 * units + upw - 1) / upw;
  }
  return p;
}

// The one-row QKV launch can carry the fused decode attention (fattn_consumer) when it takes
// the register-staged RMSNorm prologue (the EARLY instantiation, as launch_one decides).
bool wgemm_fattn_ok(int N, int K, int num_cu) {
  const WgemmPlan p = plan_wgemm(1, N, K, EPI_STORE, num_cu);
  if (!p.a_lds || p.sliced || K > 4096 || p.sp.waves != DEC_NW) return false;  // (16-wave workgroups)
  if (wgemm_fattn_d(p.sp.ku) != 64) return false;  // (the one-row form: head dim 64)
  const int kch = K / 8, NT = p.sp.waves * 64;
  const int ea = p.sp.waves >= 16 ? 1 : (p.sp.waves >= 8 ? 2 : 4);  // wgemm_ea
  return kch % 64 == 0 && (kch + NT - 1) / NT <= ea;
}

// 2..32 rows: the QKV launch of the batched step can carry the attention when it is one
// 16-wave, unsliced launch with the A rows in LDS (any prologue; 17..32 rows: two m-tiles)
bool wgemm_fattn_rows_ok(int M, int N, int K, int D, int num_cu) {
  const WgemmPlan p = plan_wgemm(M, N, K, EPI_STORE, num_cu);
  // (launch_wgemm runs the fused launch with whole units, csplit 1; the launch shape's ring
  // depth is 2 when the item's stage count is even, which the fused o_proj also requires)
  const int S = (K / 32) / (p.sp.ksplit * p.sp.ku);
  return M >= 2 && M <= 32 && p.a_lds && !p.sliced && p.sp.waves == DEC_NW && D == wgemm_fattn_d(p.sp.ku) &&
         K % 512 == 0 && S % 2 == 0;
}

bool wgemm_supported(int M, int N, int K, int epi) {
  const int NG = (epi == EPI_SWIGLU) ? 2 : 1;
  // (the weight stream addresses the tiled matrix through one buffer resource: 32-bit byte
  // offsets, and the out-of-range sentinel of the refills past a wave's last unit must stay
  // beyond the matrix, wgemm_kernel)
  return M >= 1 && M <= 64 && N > 0 && K > 0 && (N % (16 * NG)) == 0 && (K % 256) == 0 &&
         (unsigned long long)N * (unsigned long long)K * 2ull <= kWgemmMaxBytes;
}

void launch_wgemm(const WgemmArgs& a_in, const WgemmPlan& p_in, int epi, bool norm, hipStream_t s) {
  WgemmArgs a = a_in;
  WgemmPlan p = p_in;
  if (p.csplit == 2 && a.fattn_wgs) {  // the fused QKV + attention launch keeps whole units
    p.csplit = 1;
    p.grid = p.sp.grid;
  }
  a.ur = p.sp.ur();
  a.kc = p.sp.kc;
  a.sliced = p.sliced ? 1 : 0;
  a.csplit = p.csplit;
  if (a.csplit == 2 && epi != EPI_STORE && epi != EPI_RESID)
    throw std::runtime_error("wgemm: column split only for plain store / residual launches");
  static const int diag = getenv("TTS_WGEMM_DIAG") ? atoi(getenv("TTS_WGEMM_DIAG")) : 0;
  a.diag = diag;
  if (p.sliced) {
    // one K chunk per workgroup row of the grid: fp32 partials, then the epilogue in a
    // combine kernel (fixed chunk order: deterministic)
    if (norm || (epi != EPI_STORE && epi != EPI_RESID) || (a.part_out == nullptr && !dry_launches()))
      throw std::runtime_error("K-sliced wgemm: store/residual epilogues with a partial workspace only");
    const int Kfull = a.K;
    a.K = Kfull / p.sp.kc;  // the kernel's A chunk; ldx stays the full row
    launch_wgemm_store(a, p, false, s);
    if (epi == EPI_RESID && a.next_norm && !a.norm_out && !dry_launches())
      throw std::runtime_error("K-sliced wgemm: next_norm without norm_out");
    if (epi == EPI_RESID && a.next_norm)
      launch_splitk_combine_norm(a.part_out, p.sp.kc, a.M, a.N, a.ldo, a.resid, a.ldo, a.next_norm, a.eps,
                                 a.norm_out, a.ldo, s);
    else
      launch_splitk_combine(a.part_out, p.sp.kc, a.M, a.N, a.ldo, a.out, epi == EPI_RESID ? a.resid : nullptr,
                            a.ldo, s);
    return;
  }
  a.part_out = nullptr;
  switch (epi) {
    case EPI_STORE: launch_wgemm_store(a, p, norm, s); break;
    case EPI_RESID: launch_wgemm_resid(a, p, norm, s); break;
    case EPI_SWIGLU: launch_wgemm_swiglu(a, p, norm, s); break;
    case EPI_LOGITS: launch_wgemm_logits(a, p, norm, s); break;
  }
}

}  // namespace tts
