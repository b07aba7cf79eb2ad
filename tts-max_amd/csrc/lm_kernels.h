// lm_kernels.h — host-side declarations of the SpeechLM kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace tts {

// Dry run (tts_debug_step_plan): while a recorder is set on this thread, the SpeechLM
// launchers append what they would launch — the wgemm_kernel template arguments, other
// kernels by name — and return without any HIP call, so a decode step's launch list can be
// read on a machine without a GPU (the spill gate, tests/test_kernel_resources.py).
std::vector<std::string>*& dry_launches();
inline bool dry_record(const std::string& what) {
  std::vector<std::string>* v = dry_launches();
  if (!v) return false;
  v->push_back(what);
  return true;
}

typedef uint16_t bf16_t;

enum { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2, EPI_LOGITS = 3 };

// Weight layout + decode launch decomposition of one tiled matrix ("stream plan").
// Work item = (unit of NG n-tiles, K part of KT/ksplit k-tiles); a wave streams its item
// in stages of ku k-tiles.  Units run in rounds of ur() = grid * waves/ksplit (one unit
// per wave group of every workgroup).  Tiles are stored round-major, then STAGE-major:
// at stage s every wave of the launch reads one contiguous block (ur*ksplit*NG*ku KiB),
// the access pattern that streams HBM fastest (scripts/hbm_floor.hip, pipe sweep).
// K is cut into kc chunks of KT/kc k-tiles (chunk-major): a wave's K part is split evenly
// over the chunks, so a launch may also run one chunk per workgroup (grid.y = chunk,
// "K-sliced": the A operand of one chunk fits LDS at batch 17..32; fp32 partials combined
// by a second kernel).
struct StreamPlan {
  int ng = 1, ksplit = 1, ku = 8, waves = 4, grid = 1, kc = 1;
  __host__ __device__ int ur() const { return grid * (waves / ksplit); }
};
// Tile index (1 KiB units) of n-tile nt (unit nt/ng, member nt%ng), k-tile kt.
__host__ __device__ inline long long plan_tile(int ng, int ksplit, int ku, int ur, int units, int KT,
                                               int kc, int nt, int kt) {
  const int u = nt / ng, g = nt - u * ng;
  const int KTc = KT / kc, kt_pc = KTc / ksplit;
  const int c = kt / KTc, rr = kt - c * KTc;
  const int kp = rr / kt_pc, ki = rr - kp * kt_pc;
  const int st = c * (kt_pc / ku) + ki / ku, kk = ki % ku;
  const int r = u / ur, ui = u - r * ur;
  const int nr = (units - r * ur) < ur ? (units - r * ur) : ur;
  return (long long)r * ur * KT * ng +
         (((long long)st * nr * ksplit + (long long)ui * ksplit + kp) * ng + g) * ku + kk;
}
StreamPlan stream_plan(int N, int K, int ng, int num_cu);
constexpr int LOGITS_MAX_PARTS = 1024;  // lm_head workgroups = argmax partials per row

struct AttnArgs {
  const bf16_t* qkv = nullptr;  // [rows][ld_qkv]: q (H*D) | k (KVH*D) | v (KVH*D)
  int ld_qkv = 0;
  int rows = 0;
  const int* row_slot = nullptr;  // KV slot (sequence) of each query row
  const int* row_pos = nullptr;   // absolute position of each query row
  bf16_t* kcache = nullptr;       // this layer's K rows: [slots][KVH][max_seq][D]
  bf16_t* vtcache = nullptr;      // this layer's V^T: [slots][KVH] blocks of D x max_seq in 16 x 32 tiles (vt_off)
  int max_seq = 0;                // position stride of the cache (a multiple of 64)
  const bf16_t* rope_cos = nullptr;  // [max_seq][D]
  const bf16_t* rope_sin = nullptr;
  int H = 0, KVH = 0, D = 0;
  float scale = 0.f;
  bf16_t* q_rot = nullptr;  // prefill: roped q [rows][H*D]
  bf16_t* out = nullptr;    // [rows][H*D] bf16 attention output
  const int4* blocks = nullptr;  // prefill: query blocks {first row, rows (<= 16), slot, first position}
  int nblocks = 0;
  unsigned long long* stamps = nullptr;  // diagnostic build only (TTS_STAMPS)
  // decode: q | k | v as fp32 partials of a K-sliced QKV launch ([qkv_nsl][rows][ld_qkv], summed
  // in slice order and rounded to bf16 here, as splitk_combine_kernel would) instead of qkv
  const float* qkv_part = nullptr;
  int qkv_nsl = 0;
};

// ---- sampling / bookkeeping state of a decode step (lm_ops.hip, lm_finalize.h)
struct StepState {
  int* tokens;        // [B] token fed to the next step
  int* pos;           // [B] position of the next token (= current length)
  int* gen_count;     // [B] tokens generated so far
  int* limit;         // [B] max new tokens
  int* done;          // [B]
  int* eos_mask;      // [B] eos id while gen_count < min_new, else -1
  uint32_t* seen;     // [B][seen_stride]
  int seen_stride;
  int* out_ids;       // [B][out_stride]
  int out_stride;
  int* n_active;      // [1]
  uint16_t* counts;   // [B][V] new-token counts (frequency penalty) or nullptr
  unsigned long long* row_seed;  // [B] sampling key of each row
  uint32_t* epoch;    // [1] step counter (+1 by the finalize of every step: the norm-once hand-off's tags)
  int eos_id;
  int min_new;
};

// Largest tiled weight matrix a wgemm launch streams: one buffer resource with 32-bit byte
// offsets, and the past-the-last-unit sentinel offsets (wgemm_kernel: kWgemmSentinel - the
// stage's tile offsets, at most 15 KiB below it) must stay beyond the matrix
constexpr unsigned long long kWgemmMaxBytes = 0xFFFF0000ull;
constexpr uint32_t kWgemmSentinel = 0xFFFFFFF0u;

struct WgemmArgs {
  const bf16_t* x = nullptr;  // A: [M][ldx] bf16 activations
  int M = 0, K = 0, ldx = 0;
  const bf16_t* w = nullptr;  // B: tiled weights (see lm_gemm.hip)
  int N = 0;
  const bf16_t* normw = nullptr;  // RMSNorm weight [K] (NORM prologue)
  float eps = 0.f;
  bf16_t* out = nullptr;  // [M][ldo]
  int ldo = 0;
  bf16_t* resid = nullptr;  // EPI_RESID: residual stream, updated in place
  // EPI_LOGITS
  const uint32_t* seen = nullptr;  // [M][seen_stride] bitmap of ids present in the sequence
  int seen_stride = 0;
  float penalty = 1.f;
  const int* eos_mask = nullptr;  // [M] token id forced to -inf (or -1)
  float* part_val = nullptr;      // [M][part_stride]
  int* part_idx = nullptr;
  int part_stride = 0;
  float* logits_out = nullptr;  // EPI_LOGITS: also store the processed fp32 logits [M][ldl] (sampling)
  const uint16_t* counts = nullptr;  // EPI_LOGITS: new-token counts [M][seen_stride*32] (frequency penalty)
  float freq_penalty = 0.f;
  int ldl = 0;
  int ur = 0;         // layout: units per round (StreamPlan::ur, filled in by launch_wgemm)
  int kc = 1;         // layout: K chunks (StreamPlan::kc, filled in by launch_wgemm)
  int sliced = 0;     // 1: grid.y = K chunk, K = one chunk, ldx = full K (filled in by launch_wgemm)
  float* part_out = nullptr;  // K-sliced launches: fp32 partials [kc][M][ldo] (caller's workspace)
  const bf16_t* next_norm = nullptr;  // K-sliced residual launches: RMSNorm the updated rows
  bf16_t* norm_out = nullptr;         //   with next_norm (eps) into norm_out [M][ldo]
  // QKV launch with the decode attention fused in (decode, one row): the projection's
  // workgroups publish q/k/v as data-tagged 8-byte granules {bf16 pair, tag} with
  // agent-scope stores; fattn_wgs extra workgroups (blockIdx.x >= the GEMM grid), one per kv
  // head, load their K / V^T fragments, wait for their q (and the new k/v) granules and
  // attend exactly as attn_decode_kernel does.  tag = (pos << 6) | layer differs between any
  // two consecutive launches, so a granule left by the previous launch never matches.
  uint64_t* gran = nullptr;   // [M][N / 2] q|k|v granules, then (fo_units) [M][H*D / 2] attention rows
  AttnArgs fa;                // the attention of this layer (its output row: fa.out)
  int fattn_wgs = 0;          // attention workgroups appended to the grid (0: not fused)
  int fattn_layer = 0;
  // grid order.  0 (default): the projection workgroups, then the attention workgroups, then
  // (fo_units > 0) one o_proj workgroup per o_proj unit: every workgroup waits only on blocks
  // of lower index, and blocks are dispatched in index order, so the launch completes whatever
  // else occupies the GPU (no co-residency needed).  1 (round-3 order, TTS_FATTN_FIRST=1): the
  // attention workgroups first and o_proj on the projection workgroups after their QKV unit —
  // circular waits, so it needs the whole grid resident (grid <= CUs, checked at launch).
  int fattn_first = 0;
  int* fattn_err = nullptr;   // set to 1 if a granule wait timed out; later waits then give up at once
  int fattn_spins = 1 << 16;  // polls (s_sleep 1 each, ~0.1 s in all) before a wait gives up
  // o_proj fused behind the attention (fo_units > 0): the attention workgroups also publish
  // the bf16 attention row as granules (gran + N/2, same tag); o_proj unit b (tiled weights
  // fo_w, layout rounds fo_ur, one round) runs on the grid's b-th o_proj workgroup (order 0)
  // or on projection workgroup b after its QKV unit (order 1), with the residual epilogue on
  // fo_resid (the hidden row), its o_proj weights loaded while the attention runs
  // (2..16 rows, order 0: the attention rows' granules at gran + M*N/2, row m's H*D/2 at
  // m*H*D/2; o_proj's layout K chunks fo_kc; fo_resid holds the M hidden rows)
  const bf16_t* fo_w = nullptr;
  int fo_units = 0, fo_ur = 0, fo_kc = 1;
  bf16_t* fo_resid = nullptr;
  // RMSNorm once per row, by the producer launch (2..32 decode rows; round 6): the launch's
  // residual epilogue (fused o_proj of the QKV launch, or the down projection's own) also
  // publishes every pair of the updated hidden row as a granule {bf16 pair, tag = (step << 6) |
  // layer} in nw_gran [M][hid / 2], and nrm_wgs = M workgroups appended last in the grid (each
  // waits only on lower blocks) gather one row each and write RMSNorm(row, nw_w) to nw_out
  // [M][hid] in the canonical order (chunk_sumsq per 16 B, the wave DPP tree per 512 values,
  // segments in order): the same bits as every other RMSNorm path.  The consumer launch then
  // stages normalised rows instead of every workgroup normalising every row.  The step counter
  // (*nw_epoch, one scalar load: no registers held through the weight stream) advances at every
  // decode step, so two launches that write one granule region never share a tag.
  int nrm_wgs = 0;
  const bf16_t* nw_w = nullptr;
  bf16_t* nw_out = nullptr;
  uint64_t* nw_gran = nullptr;
  const uint32_t* nw_epoch = nullptr;
  int nw_layer = 0, nw_hid = 0;
  unsigned long long* stamps = nullptr;  // diagnostic build only (TTS_STAMPS): [block][8]
  int csplit = 1;     // 2: each 16-column unit runs as two 8-column halves (twice the workgroups; filled in by launch_wgemm)
  int diag = 0;       // timing diagnostics only (TTS_WGEMM_DIAG): 1 no prologue, 2 no epilogue, 8 barrier before the stream, 64 per-wave norm-end stamps
};

struct WgemmPlan {
  StreamPlan sp;  // the matrix's layout + launch shape (waves, stage depth, split-K)
  int cfg = 0;    // kernel instantiation of that shape (lm_gemm.hip)
  int grid = 1;
  bool a_lds = true;
  bool sliced = false;  // one K chunk per workgroup (grid.y = sp.kc) + combine kernel
  int csplit = 1;       // 2: units split into 8-column halves over twice the workgroups
};

// Row-major W [N][K] -> tiles of the matrix's stream plan.  The destination matrix has
// N_total rows; source n-tile nt lands at n-tile nt * nt_mult + nt_off (nt_mult = 2
// interleaves gate/up n-tiles: unit u = (gate tile u, up tile u), ng = 2).
void launch_retile(const bf16_t* w, bf16_t* t, int N, int K, int N_total, int ng, int num_cu,
                   hipStream_t s, int nt_mult = 1, int nt_off = 0);
WgemmPlan plan_wgemm(int M, int N, int K, int epi, int num_cu);
// LDS bytes of a wgemm launch whose A operand (M rows x Kl columns) is staged in LDS
size_t wgemm_lds_bytes(int waves, int ksplit, int ng, int M, int Kl, bool a_in_lds);
// fp32 partial workspace a K-sliced launch of this plan needs (elements)
inline size_t wgemm_part_elems(const WgemmPlan& p, int M, int ldo) {
  return p.sliced ? (size_t)p.sp.kc * M * ldo : 0;
}
bool wgemm_supported(int M, int N, int K, int epi);
bool wgemm_fattn_ok(int N, int K, int num_cu);
bool wgemm_fattn_rows_ok(int M, int N, int K, int D, int num_cu);
void launch_wgemm(const WgemmArgs& a, const WgemmPlan& p, int epi, bool norm, hipStream_t s);
// 17..32 rows of a kc = 1 qkv / o_proj layout (16-wave KSPLIT 16, KU 2), K split over 4
// workgroups (grid.y): fp32 partials [4][M][ldo] to a.part_out; a.K = K / 4 (lm_gemm_store.hip)
void launch_wgemm_kslice(const WgemmArgs& a, int units, hipStream_t s);

// ---- greedy lm_head as an exact two-pass argmax (lm_head_screen.hip): an int8 screen that
// bounds every column's processed score, then (in the same launch) the units that can hold the
// argmax recomputed exactly as the bf16 lm_head computes them
struct HeadScreenArgs {
  const bf16_t* x = nullptr;      // [M][ldx] rows (RMSNorm'ed here when normw)
  int M = 0, K = 0, ldx = 0, V = 0;
  const bf16_t* normw = nullptr;  // final RMSNorm weight, or nullptr (rows already normalised)
  float eps = 0.f;
  const int8_t* xq = nullptr;     // (17..32 rows) the rows pre-quantised [2M][K] (launch_head_rowquant)
  const float* xstat = nullptr;   //   and their {sx, |x|, |x - sx X|, 0} [M][4]
  const int8_t* q = nullptr;      // int8 lm_head in the screen's block layout (launch_head_quant)
  const float4* cst = nullptr;    // [V] {scale, |W - Wh|, |W|, |Wh|}
  int ur = 0;                     // layout units per round = screen grid * head_screen_waves()
  const bf16_t* w = nullptr;      // the tiled bf16 lm_head and its stream plan (ng 1, ksplit 1)
  int hku = 8, hur = 0, hKT = 0, hkc = 1;
  const uint32_t* seen = nullptr;
  int seen_stride = 0;
  float penalty = 1.f;
  const int* eos_mask = nullptr;
  const uint16_t* counts = nullptr;
  float freq_penalty = 0.f;
  const uint32_t* epoch = nullptr;      // the decode-step counter (finalize_greedy_kernel advances it)
  unsigned long long* lbg = nullptr;    // [M][8 shards] maximum lower bound: (step << 32) | order key
  uint32_t* arrive = nullptr;           // [8 shards, 64 B apart] workgroups that added their bounds (only grows)
  int spins = 1 << 14;                  // polls (s_sleep 1 each) before the wait for them gives up (0: no wait)
  float* part_val = nullptr;      // [M][part_stride] argmax partials, one per workgroup
  int* part_idx = nullptr;
  int part_stride = 0;
  int check = 0;                  // 1: recompute every unit, check each score against its bound
  float* ub = nullptr;            // check mode: [M][ldu] upper bound of every processed score
  int ldu = 0;
  int* err = nullptr;             // check mode: set to 1 when a score exceeds its bound
  int diag = 0;                   // probes only (TTS_HEAD_SCREEN_DIAG): 1 skip the recompute (wrong ids), 2 count flagged units
};
bool head_screen_supported(int M, int K, int V);
bool head_screen_prequant(int M);  // rows quantised by launch_head_rowquant first (17..32 rows, K 2048)
int head_screen_waves();
void launch_head_rowquant(const bf16_t* x, int ldx, int M, int K, int8_t* xq, float* xstat, hipStream_t s);
void launch_head_quant(const bf16_t* w, int V, int K, int ur, int8_t* q, float* cst, hipStream_t s);
void launch_head_screen(const HeadScreenArgs& a, int grid, hipStream_t s);

// ---- prefill GEMM (lm_pgemm.hip): many rows against the same tiled weights, LDS-staged
// MFMA blocks; epilogues EPI_STORE / EPI_RESID / EPI_SWIGLU; no fused RMSNorm
struct PgemmArgs {
  const bf16_t* x = nullptr;  // [M][ldx]
  int M = 0, K = 0, ldx = 0;
  const bf16_t* w = nullptr;  // tiled weights (the matrix's stream plan, filled in by launch_pgemm)
  int N = 0;
  int ng = 1, ksplit = 1, ku = 1, ur = 1, units = 1, kc = 1;
  bf16_t* out = nullptr;  // [M][ldo]
  int ldo = 0;
  bf16_t* resid = nullptr;  // EPI_RESID: updated in place
  int xcd_order = 0;        // set by launch_pgemm: the XCD-grouped tile order (lm_pgemm.hip)
  float* part = nullptr;    // fp32 partials of the one-chunk-per-workgroup form (null: never used)
  size_t part_bytes = 0;
  // optional (EPI_RESID): the next RMSNorm of the updated rows, written to xn [M][N] by the
  // one-chunk form's combine (launch_pgemm then returns true)
  const bf16_t* next_norm = nullptr;
  float eps = 0.f;
  bf16_t* xn = nullptr;
};
bool pgemm_supported(int M, int N, int K, int epi);
size_t pgemm_part_bytes(int M, int N, int K);  // the one-chunk form's partials of an M x N x K GEMM
bool launch_pgemm(const PgemmArgs& a, int epi, int num_cu, hipStream_t s);  // true: xn written

// ---- elementwise / small kernels (lm_ops.hip)
void launch_rmsnorm(const bf16_t* x, int ldx, const bf16_t* w, float eps, bf16_t* y, int ldy,
                    int M, int K, hipStream_t s);
void launch_embed(const int* tokens, const bf16_t* table, bf16_t* x, int M, int hidden,
                  hipStream_t s);
void launch_gather_rows(const bf16_t* x, int ld, const int* rows, bf16_t* y, int M, int hidden,
                        hipStream_t s);
void launch_synth_fill(void* dst, int dtype, long long n, unsigned long long seed, float scale,
                       hipStream_t s);
void launch_f32_to_bf16(const float* x, bf16_t* y, long long n, hipStream_t s);
void launch_f16_to_bf16(const void* x, bf16_t* y, long long n, hipStream_t s);  // x: _Float16
// K-sliced GEMM combine: v = bf16(sum_c part[c][m][n]);  resid ? resid += v : out = v
void launch_splitk_combine(const float* part, int kc, int M, int N, int ldp, bf16_t* out,
                           bf16_t* resid, int ldo, hipStream_t s);
// residual combine + the next RMSNorm of the updated rows into xn (N % 8 == 0, N <= 8192)
void launch_splitk_combine_norm(const float* part, int kc, int M, int N, int ldp, bf16_t* resid, int ldo,
                                const bf16_t* normw, float eps, bf16_t* xn, int ldn, hipStream_t s);

// ---- attention (lm_attn.hip)
void launch_rope_append(const AttnArgs& a, hipStream_t s);  // prefill: rope q, k; K rows, V columns
void launch_attn_prefill(const AttnArgs& a, hipStream_t s);  // prefill: causal attention per query block
// decode step: one workgroup per (row, kv head): RoPE, attention over pos + 1 positions,
// bf16 output, KV append
void launch_attn_decode_step(const AttnArgs& a, hipStream_t s);

// ---- sampling head (lm_sample.hip): temperature, top-k, top-p, multinomial draw
struct SampleArgs {
  const float* logits = nullptr;  // processed logits [B][ldl]
  int ldl = 0, V = 0;
  float temperature = 1.f;
  int top_k = 50;                 // 1 .. 1024
  float top_p = 1.f;
  unsigned long long seed = 0;
  const unsigned long long* row_seed = nullptr;  // per-row keys (seed, row ignored) or nullptr
  const int* step = nullptr;      // per-row draw counter (generated count), or step0
  int step0 = 0;
  const int* done = nullptr;      // rows already stopped (skipped)
  const float* part_val = nullptr;  // lm_head workgroup maxima [B][part_stride] (top-k bound)
  int nparts = 0, part_stride = 0;
  float* out_part_val = nullptr;  // chosen token as the single "partial" finalize reads
  int* out_part_idx = nullptr;
  float* probs = nullptr;         // optional: final distribution [B][ldl] (kept ids only)
  int* tokens = nullptr;          // optional: chosen token [B]
};
constexpr int SAMPLE_MAX_TOP_K = 1024;
void launch_sample(const SampleArgs& a, int B, hipStream_t s);

void launch_bump_epoch(uint32_t* epoch, hipStream_t s);  // *epoch += 1 (a decode step without finalize)
void launch_finalize_greedy(const float* part_val, const int* part_idx, int part_stride,
                            int nparts, StepState st, int B, const bf16_t* embed, bf16_t* x,
                            int hidden, hipStream_t s);

}  // namespace tts
