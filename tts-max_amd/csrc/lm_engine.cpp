// lm_engine.cpp — SpeechLM host runtime: weight loading/re-layout, workspaces, chunked
// prefill, hipGraph-captured decode step, device-side stop bookkeeping.
//
// Replaces the reference AR loop `_generate_speech_tokens` -> HF `model.generate`
// (tts/inference/inferencing.py:94-107; transformers generation/utils.py:2783-2950):
//   * prefill over the prompt, then one decode step per generated code;
//   * greedy: argmax over fp32(bf16 logits) after repetition penalty and min-new-tokens EOS
//     mask; stop at EOS (included in the output) or at max_length (total length);
//   * batch > 1 = independent sequences (each identical to its batch-1 generate).
// HF syncs the host every token (`unfinished_sequences.max() == 0`); here the step is one
// hipGraph replay and the host polls a device counter of active sequences every
// kPollEvery steps, one poll behind, so the GPU never waits for the host.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <cstdio>

#include "engine.h"

namespace tts {

static constexpr int kPollEvery = 8;
static constexpr int kPrefillChunk = 64;   // rows per GEMM launch (MFMA A-tiles of 16)
static constexpr int kMaxPrefillRows = 8192;

// The greedy lm_head as an exact two-pass argmax (lm_head_screen.hip): default on;
// TTS_HEAD_SCREEN=0 streams the full bf16 lm_head for greedy steps too (the same ids)
static bool head_screen_enabled() {
  static const bool v = !(getenv("TTS_HEAD_SCREEN") && !atoi(getenv("TTS_HEAD_SCREEN")));
  return v;
}
// ... whose workgroups wait for every workgroup's bounds before flagging their units (the
// exact candidate set; TTS_HEAD_SCREEN_WAIT=0: never, 1: always, n > 1 (default 2): from n rows —
// one row: 69 vs 73 us, 8 rows: 79 vs 96 us without, profiles/r6w_ab_head_wait_*).  Same bits
// either way: a lower LB only flags more units
static bool head_screen_wait(int rows) {
  static const int v = getenv("TTS_HEAD_SCREEN_WAIT") ? atoi(getenv("TTS_HEAD_SCREEN_WAIT")) : 2;
  return v == 1 || (v > 1 && rows >= v);
}
// TTS_HEAD_SCREEN_CHECK=1: every unit recomputed and each exact score checked against its bound
static bool head_screen_check() {
  static const bool v = getenv("TTS_HEAD_SCREEN_CHECK") && atoi(getenv("TTS_HEAD_SCREEN_CHECK"));
  return v;
}


int64_t numel(const tts_tensor_desc& d) {
  int64_t n = 1;
  for (int i = 0; i < d.ndim; ++i) n *= d.shape[i];
  return n;
}

void upload_bf16(const tts_tensor_desc& d, bf16_t* dst, hipStream_t s, DevBuf& staging) {
  const int64_t n = numel(d);
  if (d.dtype == TTS_DT_BF16) {
    HIP_CHECK(hipMemcpyAsync(dst, d.data, n * 2, d.on_device ? hipMemcpyDeviceToDevice
                                                             : hipMemcpyHostToDevice, s));
  } else if (d.dtype == TTS_DT_F32) {
    const float* src = (const float*)d.data;
    if (!d.on_device) {
      if (staging.bytes < (size_t)n * 4) staging.alloc((size_t)n * 4);
      HIP_CHECK(hipMemcpyAsync(staging.p, d.data, n * 4, hipMemcpyHostToDevice, s));
      src = staging.as<float>();
    }
    launch_f32_to_bf16(src, dst, n, s);
  } else if (d.dtype == TTS_DT_F16) {
    const void* src = d.data;
    if (!d.on_device) {
      if (staging.bytes < (size_t)n * 2) staging.alloc((size_t)n * 2);
      HIP_CHECK(hipMemcpyAsync(staging.p, d.data, n * 2, hipMemcpyHostToDevice, s));
      src = staging.p;
    }
    launch_f16_to_bf16(src, dst, n, s);
  } else {
    throw Error(TTS_E_UNSUPPORTED, std::string("tensor ") + d.name + ": dtype must be bf16, f16 or f32");
  }
}

void upload_f32(const tts_tensor_desc& d, float* dst, hipStream_t s, DevBuf&) {
  TTS_REQUIRE(d.dtype == TTS_DT_F32, std::string("tensor ") + d.name + " must be f32");
  HIP_CHECK(hipMemcpyAsync(dst, d.data, numel(d) * 4,
                           d.on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
}

// ------------------------------------------------------------------------ loading -----
namespace {
struct TensorMap {
  std::map<std::string, const tts_tensor_desc*> m;
  const tts_tensor_desc& get(const std::string& name, std::initializer_list<int64_t> shape) const {
    auto it = m.find(name);
    if (it == m.end()) throw Error(TTS_E_INVALID, "missing tensor: " + name);
    const tts_tensor_desc& d = *it->second;
    int i = 0;
    bool ok = (int)shape.size() == d.ndim;
    for (int64_t v : shape) { if (ok && d.shape[i] != v) ok = false; ++i; }
    if (!ok) throw Error(TTS_E_INVALID, "bad shape for tensor: " + name);
    return d;
  }
  bool has(const std::string& n) const { return m.count(n) != 0; }
};

// RoPE table as LlamaRotaryEmbedding computes it (modeling_llama.py:~100-128 and
// modeling_rope_utils.py:580-660 for llama3), evaluated in double then rounded; the Python
// host normally passes the torch-computed table instead ("rope.cos"/"rope.sin").
void compute_rope_table(const tts_lm_config& c, std::vector<bf16_t>& cs, std::vector<bf16_t>& sn) {
  const int D = c.head_dim, S = c.max_seq_len;
  std::vector<float> inv(D / 2);
  for (int i = 0; i < D / 2; ++i) {
    float e = (float)(2 * i) / (float)D;
    inv[i] = 1.0f / powf(c.rope_theta, e);
  }
  if (c.rope_llama3) {
    const double lo_wl = c.rope_original_max_position / c.rope_low_freq_factor;
    const double hi_wl = c.rope_original_max_position / c.rope_high_freq_factor;
    for (int i = 0; i < D / 2; ++i) {
      const float f = inv[i];
      const double wl = 2 * M_PI / f;
      float v = (wl > lo_wl) ? f / c.rope_factor : f;
      if (!(wl < hi_wl) && !(wl > lo_wl)) {
        const float sm = (float)((c.rope_original_max_position / wl - c.rope_low_freq_factor) /
                                 (c.rope_high_freq_factor - c.rope_low_freq_factor));
        v = (1 - sm) * v / c.rope_factor + sm * v;
      }
      inv[i] = v;
    }
  }
  auto to_bf = [](float f) -> bf16_t {
    uint32_t u;
    memcpy(&u, &f, 4);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (bf16_t)(u >> 16);
  };
  cs.resize((size_t)S * D);
  sn.resize((size_t)S * D);
  for (int p = 0; p < S; ++p)
    for (int i = 0; i < D; ++i) {
      const float fr = (float)p * inv[i % (D / 2)];
      cs[(size_t)p * D + i] = to_bf((float)cos((double)fr));
      sn[(size_t)p * D + i] = to_bf((float)sin((double)fr));
    }
}
}  // namespace

// K-sliced GEMMs (store / residual epilogues): fp32 partials of kc = K / 2048 chunks of <= 64 rows
static size_t kpart_bytes(const tts_lm_config& c) {
  const int kmax = std::max(c.hidden_size, std::max(c.intermediate_size, c.num_heads * c.head_dim));
  const int QKV = (c.num_heads + 2 * c.num_kv_heads) * c.head_dim;
  return (size_t)std::max(1, kmax / 2048) * kPrefillChunk * std::max(QKV, c.hidden_size) * 4;
}

// prefill GEMMs of <= kPgemmSplitRows rows may take one canonical K chunk per workgroup
// (lm_pgemm.hip): fp32 partials [chunks][rows][N] of the largest of the layer's four GEMMs
static constexpr int kPgemmSplitRows = 256;
static size_t ppart_bytes(const tts_lm_config& c) {
  const int H = c.hidden_size, HD = c.num_heads * c.head_dim, FF = c.intermediate_size;
  const int QKV = (c.num_heads + 2 * c.num_kv_heads) * c.head_dim;
  return std::max(std::max(pgemm_part_bytes(kPgemmSplitRows, QKV, H), pgemm_part_bytes(kPgemmSplitRows, H, HD)),
                  std::max(pgemm_part_bytes(kPgemmSplitRows, 2 * FF, H), pgemm_part_bytes(kPgemmSplitRows, H, FF)));
}

void lm_load(Engine* e, const tts_lm_config* cfgp, const tts_tensor_desc* t, int n) {
  TTS_REQUIRE(cfgp != nullptr, "null config");
  const tts_lm_config c = *cfgp;
  TTS_REQUIRE(c.head_dim == 64 || c.head_dim == 128, "head_dim must be 64 or 128");
  TTS_REQUIRE(c.num_heads == 4 * c.num_kv_heads, "GQA group must be 4 (num_heads == 4*num_kv_heads)");
  TTS_REQUIRE(c.hidden_size % 256 == 0 && c.intermediate_size % 256 == 0 &&
                  (c.num_heads * c.head_dim) % 256 == 0,
              "hidden/intermediate/attention widths must be multiples of 256");
  TTS_REQUIRE(c.vocab_size % 16 == 0, "vocab_size must be a multiple of 16");
  // (the GEMMs stream a matrix through one buffer resource: 32-bit byte offsets)
  TTS_REQUIRE((double)c.vocab_size * c.hidden_size * 2 < 4.0e9 &&
                  (double)2 * c.intermediate_size * c.hidden_size * 2 < 4.0e9,
              "a weight matrix of 4 GB or more is not supported");
  TTS_REQUIRE(c.max_batch >= 1 && c.max_batch <= 64, "max_batch must be in [1, 64]");
  TTS_REQUIRE(c.max_seq_len >= 16, "max_seq_len too small");
  TensorMap tm;
  for (int i = 0; i < n; ++i) tm.m[t[i].name] = &t[i];
  hipStream_t s = e->stream;
  LmModel& M = e->lm;
  M.loaded = false;
  M.cfg = c;
  const int H = c.num_heads, KVH = c.num_kv_heads, D = c.head_dim, HID = c.hidden_size;
  const int FF = c.intermediate_size, V = c.vocab_size, L = c.num_layers;
  const int QKV = M.qkv_n();

  // ---- one slab for everything
  const size_t per_layer = 2 * (size_t)HID + (size_t)QKV * HID + (size_t)HID * H * D +
                           2 * (size_t)FF * HID + (size_t)HID * FF;
  const size_t total = per_layer * L + HID + (size_t)V * HID;
  M.weights.alloc(total * 2);
  bf16_t* p = M.weights.as<bf16_t>();
  M.layers.resize(L);
  for (int l = 0; l < L; ++l) {
    LmLayer& ly = M.layers[l];
    ly.ln1 = p; p += HID;
    ly.ln2 = p; p += HID;
    ly.wqkv = p; p += (size_t)QKV * HID;
    ly.wo = p; p += (size_t)HID * H * D;
    ly.wgu = p; p += 2 * (size_t)FF * HID;
    ly.wd = p; p += (size_t)HID * FF;
  }
  M.final_norm = p; p += HID;
  M.lm_head = p; p += (size_t)V * HID;

  DevBuf staging, staging32;
  staging.alloc((size_t)std::max<size_t>((size_t)V * HID, (size_t)FF * HID) * 2);
  // matrix (N_total rows, ng) <- row block of N rows at n-tile offset `off` (or interleaved)
  const int ncu = e->num_cu;
  auto retiled = [&](const tts_tensor_desc& d, bf16_t* dst, int N, int K, int N_total, int ng,
                     int mult, int off) {
    upload_bf16(d, staging.as<bf16_t>(), s, staging32);
    launch_retile(staging.as<bf16_t>(), dst, N, K, N_total, ng, ncu, s, mult, off);
    HIP_CHECK(hipGetLastError());
  };
  for (int l = 0; l < L; ++l) {
    LmLayer& ly = M.layers[l];
    const std::string pre = "model.layers." + std::to_string(l) + ".";
    upload_bf16(tm.get(pre + "input_layernorm.weight", {HID}), ly.ln1, s, staging32);
    upload_bf16(tm.get(pre + "post_attention_layernorm.weight", {HID}), ly.ln2, s, staging32);
    retiled(tm.get(pre + "self_attn.q_proj.weight", {H * D, HID}), ly.wqkv, H * D, HID, QKV, 1, 1, 0);
    retiled(tm.get(pre + "self_attn.k_proj.weight", {KVH * D, HID}), ly.wqkv, KVH * D, HID, QKV, 1, 1,
            H * D / 16);
    retiled(tm.get(pre + "self_attn.v_proj.weight", {KVH * D, HID}), ly.wqkv, KVH * D, HID, QKV, 1, 1,
            (H + KVH) * D / 16);
    retiled(tm.get(pre + "self_attn.o_proj.weight", {HID, H * D}), ly.wo, HID, H * D, HID, 1, 1, 0);
    retiled(tm.get(pre + "mlp.gate_proj.weight", {FF, HID}), ly.wgu, FF, HID, 2 * FF, 2, 2, 0);
    retiled(tm.get(pre + "mlp.up_proj.weight", {FF, HID}), ly.wgu, FF, HID, 2 * FF, 2, 2, 1);
    retiled(tm.get(pre + "mlp.down_proj.weight", {HID, FF}), ly.wd, HID, FF, HID, 1, 1, 0);
  }
  upload_bf16(tm.get("model.norm.weight", {HID}), M.final_norm, s, staging32);
  const tts_tensor_desc& emb = tm.get("model.embed_tokens.weight", {V, HID});
  M.embed_rows.alloc((size_t)V * HID * 2);
  upload_bf16(emb, M.embed_rows.as<bf16_t>(), s, staging32);
  if (c.tie_word_embeddings) {
    launch_retile(M.embed_rows.as<bf16_t>(), M.lm_head, V, HID, V, 1, ncu, s, 1, 0);
  } else {
    retiled(tm.get("lm_head.weight", {V, HID}), M.lm_head, V, HID, V, 1, 1, 0);
  }
  // the greedy lm_head's int8 screen (lm_head_screen.hip; TTS_HEAD_SCREEN=0: none), made from
  // the row-major matrix (the embedding rows when tied, else the staged upload)
  M.head_grid = 0;
  M.head_q.release();
  M.head_c.release();
  {
    const StreamPlan hp = stream_plan(V, HID, 1, ncu);
    if (head_screen_enabled() && head_screen_supported(1, HID, V) && hp.ng == 1 && hp.ksplit == 1) {
      M.head_grid = ncu;
      M.head_q.alloc((size_t)V * HID);
      M.head_c.alloc((size_t)V * 16);
      launch_head_quant(c.tie_word_embeddings ? M.embed_rows.as<bf16_t>() : staging.as<bf16_t>(), V, HID,
                        M.head_grid * head_screen_waves(), M.head_q.as<int8_t>(), M.head_c.as<float>(), s);
      HIP_CHECK(hipGetLastError());
    }
  }

  // ---- RoPE table
  M.rope.alloc((size_t)2 * c.max_seq_len * D * 2);
  if (tm.has("rope.cos") && tm.has("rope.sin")) {
    upload_bf16(tm.get("rope.cos", {c.max_seq_len, D}), M.rope.as<bf16_t>(), s, staging32);
    upload_bf16(tm.get("rope.sin", {c.max_seq_len, D}),
                M.rope.as<bf16_t>() + (size_t)c.max_seq_len * D, s, staging32);
  } else {
    std::vector<bf16_t> cs, sn;
    compute_rope_table(c, cs, sn);
    HIP_CHECK(hipMemcpy(M.rope.as<bf16_t>(), cs.data(), cs.size() * 2, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(M.rope.as<bf16_t>() + cs.size(), sn.data(), sn.size() * 2,
                        hipMemcpyHostToDevice));
  }
  M.id_to_code.clear();
  if (tm.has("vocab.id_to_code")) {
    const tts_tensor_desc& d = tm.get("vocab.id_to_code", {V});
    TTS_REQUIRE(d.dtype == TTS_DT_I32 && !d.on_device, "vocab.id_to_code must be host int32");
    M.id_to_code.assign((const int*)d.data, (const int*)d.data + V);
  }
  HIP_CHECK(hipStreamSynchronize(s));

  // ---- workspaces
  LmWork& w = e->w;
  if (w.graph) { (void)hipGraphExecDestroy(w.graph); w.graph = nullptr; w.graph_batch = -1; }
  const int B = c.max_batch, S = c.max_seq_len;
  const int R = std::max(B, std::min(kMaxPrefillRows, B * S));
  w.cap_rows = R;
  w.cap_batch = B;
  w.cap_seq = S;
  w.kv_stride = (S + 63) / 64 * 64;  // (V^T fragments: 8 positions = 16 B, aligned)
  w.kv.alloc((size_t)L * 2 * B * KVH * w.kv_stride * D * 2);
  HIP_CHECK(hipMemsetAsync(w.kv.p, 0, w.kv.bytes, s));  // never-read garbage stays finite
  w.x.alloc((size_t)R * HID * 2);
  w.xn.alloc((size_t)R * HID * 2);
  w.qkv.alloc((size_t)R * QKV * 2);
  w.attn_out.alloc((size_t)R * H * D * 2);
  w.q_rot.alloc((size_t)R * H * D * 2);
  w.act.alloc((size_t)R * FF * 2);
  w.last_x.alloc((size_t)B * HID * 2);
  w.blocks.alloc(((size_t)R / 16 + B + 1) * 16);  // prefill query blocks: <= rows/16 + one per sequence
  // q|k|v granules of every decode row ([B][QKV/2]), and (one-row launches with o_proj fused)
  // the attention row's at row 1's place (a launch uses one form; every prefill resets them all)
  w.gran.alloc((size_t)std::max(B, 2) * (QKV + H * D) / 2 * 8);  // q|k|v, then attention rows
  HIP_CHECK(hipMemsetAsync(w.gran.p, 0xff, w.gran.bytes, s));  // tag 0xffffffff: never a launch's
  w.ferr.alloc(256);
  // norm-once hand-off granules: two regions of [B][hidden / 2]
  w.xgran.alloc((size_t)2 * B * (HID / 2) * 8);
  HIP_CHECK(hipMemsetAsync(w.xgran.p, 0xff, w.xgran.bytes, s));
  w.epoch.alloc(64);
  HIP_CHECK(hipMemsetAsync(w.epoch.p, 0, 64, s));
  HIP_CHECK(hipMemsetAsync(w.ferr.p, 0, 256, s));
  w.kpart.alloc(kpart_bytes(c));
  w.ppart.alloc(ppart_bytes(c));
  w.slogits.alloc((size_t)B * V * 4);
  w.counts.alloc((size_t)B * (V / 32 + 1) * 32 * 2);
  w.lpart_v.alloc((size_t)B * LOGITS_MAX_PARTS * 4);
  w.lpart_i.alloc((size_t)B * LOGITS_MAX_PARTS * 4);
  if (M.head_grid) {
    if (head_screen_check()) w.hub.alloc((size_t)std::min(B, 32) * V * 4);  // (check mode's bounds)
    else w.hub.release();
    w.hxq.alloc((size_t)2 * 32 * HID);
    w.hxs.alloc((size_t)32 * 16);
    w.hlb.alloc(32 * 8 * 8 + 8 * 64);  // 32 rows x 8 shards of bounds + 8 arrival counters (64 B apart)
    HIP_CHECK(hipMemsetAsync(w.hlb.p, 0, w.hlb.bytes, s));  // (below any step's key)
  } else {
    w.hub.release(); w.hlb.release(); w.hxq.release(); w.hxs.release();
  }
  w.row_slot.alloc((size_t)R * 4);
  w.row_pos.alloc((size_t)R * 4);
  w.row_idx.alloc((size_t)R * 4);
  w.st_int.alloc((size_t)B * 8 * 4 + 64);
  w.row_seed.alloc((size_t)B * 8);
  w.seen.alloc((size_t)B * (V / 32 + 1) * 4);
  w.out_cap = S;
  w.out_ids.alloc((size_t)B * S * 4);
  if (!w.h_active) HIP_CHECK(hipHostMalloc((void**)&w.h_active, 64, hipHostMallocDefault));
  M.loaded = true;
}

// ------------------------------------------------------------------------ compute -----
#ifdef TTS_STAMPS
// diagnostic build only: per-workgroup clock stamps of the last launches (scripts/stamp_probe.py)
static unsigned long long* g_stamps = nullptr;
constexpr int kStampSlots = 1 << 16;
static unsigned long long* stamp_buf() {
  if (!g_stamps) {
    HIP_CHECK(hipMalloc((void**)&g_stamps, kStampSlots * 8));
    HIP_CHECK(hipMemset(g_stamps, 0, kStampSlots * 8));
  }
  return g_stamps;
}
extern "C" int tts_debug_stamps(unsigned long long* host, int n) {
  if (!g_stamps || n > kStampSlots) return 1;
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  if (hipMemcpy(host, g_stamps, (size_t)n * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  return hipMemset(g_stamps, 0, kStampSlots * 8) == hipSuccess ? 0 : 1;
}
#else
static unsigned long long* stamp_buf() { return nullptr; }
#endif

namespace {

// Decode attention of a one-row step fused into the QKV launch (lm_gemm_kernel.h,
// fattn_consumer): default on; TTS_FUSED_ATTN=0 keeps the separate attention launch.
bool use_fused_attn() {
  static const bool v = !(getenv("TTS_FUSED_ATTN") && !atoi(getenv("TTS_FUSED_ATTN")));
  return v;
}
// ... and o_proj fused behind that attention (lm_gemm_kernel.h fused_oproj): default on;
// TTS_FUSED_OPROJ=0 keeps the separate o_proj launch.
bool use_fused_oproj() {
  static const bool v = !(getenv("TTS_FUSED_OPROJ") && !atoi(getenv("TTS_FUSED_OPROJ")));
  return v;
}

// 17..32 rows: the decode attention sums the K-sliced QKV partials (no combine launch);
// TTS_QKV_DEFER=0 keeps the combine launch (same sums in the same order: the same bits)
bool use_qkv_defer() {
  static const bool v = !(getenv("TTS_QKV_DEFER") && !atoi(getenv("TTS_QKV_DEFER")));
  return v;
}
bool use_kslice32() {
  static const bool v = !(getenv("TTS_KSLICE32") && !atoi(getenv("TTS_KSLICE32")));
  return v;
}
// ... and at 2..16 rows, o_proj fused behind the attention of the QKV launch (its own
// workgroups after the attention's): default on; TTS_FUSED_OPROJ_ROWS=0 keeps the launch
bool use_fused_oproj_rows() {
  static const bool v = !(getenv("TTS_FUSED_OPROJ_ROWS") && !atoi(getenv("TTS_FUSED_OPROJ_ROWS")));
  return v;
}

// 17..32 rows: the RMSNorm in the consuming GEMM's LDS prologue (every workgroup normalises
// the rows it stages) instead of a standalone pass — A/B switch TTS_NORM_PROLOGUE32=1 (the same
// canonical sum order: the same bits)
bool norm_prologue32() {
  static const bool v = getenv("TTS_NORM_PROLOGUE32") && atoi(getenv("TTS_NORM_PROLOGUE32"));
  return v;
}

struct Ctx {
  Engine* e;
  hipStream_t s;
  const tts_lm_config& c;
  LmModel& M;
  LmWork& w;
  Ctx(Engine* e_, hipStream_t s_) : e(e_), s(s_), c(e_->lm.cfg), M(e_->lm), w(e_->w) {}

  int QKV() const { return M.qkv_n(); }

  // out = epi(x . W^T) over M rows (chunked by 64), RMSNorm prologue if normw != nullptr.
  // w.xn holds RMSNorm(w.x, pending_norm) when a residual combine produced it (17..32-row
  // decode: the down projection's K-sliced combine normalises with the next norm weight)
  const bf16_t* pending_norm = nullptr;
  // a decode step's layers are being issued, and the current layer (the norm-once hand-off's
  // granule tags: (step << 6) | layer)
  bool decoding = false;
  int cur_layer = 0;
  int nrm_region = 1;  // (the residual launch being issued: 0 = o_proj, 1 = down)
  // RMSNorm once per row by the producing launch (2..32 decode rows), TTS_NORM_ONCE: 0 = every
  // consuming workgroup normalises in its prologue; 1 = norm workgroups appended to the fused
  // QKV + attention + o_proj launch and to the down projection (WgemmArgs::nrm_wgs), and the
  // K-sliced down projection's combine normalising; 2 = the same without the norm workgroups on
  // the down launch; 3 (default) = only the K-sliced down's combine (a per-row kernel already)
  // normalises.  The appended norm workgroups were measured slower (their gather after the last
  // producer costs more than the prologue norm they remove: TTS-1 8 rows 755 -> 835 / 801 us
  // with modes 1 / 2, TTS-1-Max 8 rows 3,096 -> 3,180 / 3,136 us; profiles/r6c_*, r6d_*)
  int norm_once_mode() const {
    static const int mode = getenv("TTS_NORM_ONCE") ? atoi(getenv("TTS_NORM_ONCE")) : 3;
    return mode;
  }
  bool norm_once_ok(int rows) const {
    return norm_once_mode() > 0 && rows >= 2 && rows <= 32 && c.hidden_size % 512 == 0 && c.hidden_size <= 8192;
  }
  // the two granule regions of w.xgran ([cap_batch][hidden / 2] each): 0 = the fused o_proj's
  // rows, 1 = the down projection's (consecutive writers of one region differ in (pos, layer))
  size_t xgran_region(int r) const { return (size_t)r * w.cap_batch * (c.hidden_size / 2); }
  void set_norm_wgs(WgemmArgs& a, int rows, const bf16_t* normw, uint64_t* gran, int hid) const {
    a.nrm_wgs = rows;
    a.nw_w = normw;
    a.nw_out = w.xn.as<bf16_t>();
    a.nw_gran = gran;
    a.nw_epoch = w.epoch.as<uint32_t>();
    a.nw_layer = cur_layer;
    a.nw_hid = hid;
    a.eps = c.rms_norm_eps;
  }
  // 17..32-row decode: the K-sliced QKV launch leaves fp32 partials in w.kpart and the decode
  // attention sums them (no combine launch); set by layers() around the QKV gemm
  bool defer_qkv_combine = false, qkv_part_pending = false;

  void gemm(const bf16_t* x, int rows, int K, const bf16_t* W, int N, const bf16_t* normw,
            bf16_t* out, int ldo, bf16_t* resid, int epi, const WgemmArgs* logit_extra = nullptr,
            const bf16_t* next_norm = nullptr) {
    const bf16_t* ready = pending_norm;
    if (resid) pending_norm = nullptr;  // the residual stream changes below
    if (rows > kPrefillChunk && x && pgemm_supported(rows, N, K, epi)) {
      // prefill: every prompt row of the batch in one LDS-staged MFMA launch
      const bf16_t* xin = x;
      if (normw) {
        // (rows a residual combine already normalised with this weight: none to redo)
        if (!(normw == ready && x == w.x.as<bf16_t>()))
          launch_rmsnorm(x, K, normw, c.rms_norm_eps, w.xn.as<bf16_t>(), K, rows, K, s);
        xin = w.xn.as<bf16_t>();
      }
      PgemmArgs a;
      a.x = xin; a.M = rows; a.K = K; a.ldx = K;
      a.w = W; a.N = N;
      a.out = out; a.ldo = ldo; a.resid = resid;
      a.part = w.ppart.as<float>(); a.part_bytes = w.ppart.bytes;
      if (resid == w.x.as<bf16_t>() && ldo == c.hidden_size && next_norm) {
        a.next_norm = next_norm; a.eps = c.rms_norm_eps; a.xn = w.xn.as<bf16_t>();
      }
      if (launch_pgemm(a, epi, e->num_cu, s)) pending_norm = next_norm;
      return;
    }
    // decode GEMV launches hold at most 32 rows (two m-tiles: the A rows fit LDS); 33..64
    // rows run as two launches (the weights stream twice, still far cheaper than A rows
    // read from global memory)
    const int chunk = rows > 32 ? 32 : kPrefillChunk;
    for (int r0 = 0; r0 < rows; r0 += chunk) {
      const int m = std::min(chunk, rows - r0);
      WgemmPlan p = plan_wgemm(m, N, K, epi, e->num_cu);
      if (p.sliced && wgemm_part_elems(p, m, ldo) * 4 > w.kpart.bytes) {
        p.sliced = false;  // wide outputs (teacher-forced scoring over the vocabulary):
        p.a_lds = false;   // A rows from global memory instead of fp32 chunk partials
      }
      const bf16_t* xin = x ? x + (size_t)r0 * K : nullptr;
      bool norm = normw != nullptr;
      // fused RMSNorm only where the rows sit in registers (<= 16 rows, the early prologue):
      // at 17..64 rows every workgroup would normalise every row again — one standalone
      // pass (same canonical order: identical bits) is cheaper, or none when the producer
      // already wrote the normalised rows
      // (by the batch's row count: every chunk of a 33..64-row batch takes the same path)
      if (norm && normw == ready && x == w.x.as<bf16_t>()) {
        xin = w.xn.as<bf16_t>() + (size_t)r0 * K;
        norm = false;
      } else if (norm && (!p.a_lds || p.sliced || K > 4096 || (rows > 16 && !norm_prologue32()))) {
        launch_rmsnorm(xin, K, normw, c.rms_norm_eps, w.xn.as<bf16_t>(), K, m, K, s);
        xin = w.xn.as<bf16_t>();
        norm = false;
      }
      // 17..32 rows of qkv / o_proj (kc = 1, K 2048): K split over 4 workgroups (each stages a
      // quarter of the A rows, 32 KiB instead of 128) + a combine: plain bf16 rows, or residual
      // add + the next RMSNorm (the gate/up prologue's norm) in one pass.  TTS_KSLICE32=0: off
      // (chosen by the batch's row count, not the chunk's: a 33..64-row batch runs two chunks,
      // and every row of a batch must take the same arithmetic)
      if (!norm && rows > 16 && m <= 32 && K == 2048 && !logit_extra &&
          (epi == EPI_STORE || epi == EPI_RESID) && use_kslice32() && p.sp.kc == 1 && p.sp.waves == 16 && p.sp.ksplit == 16 && p.sp.ku == 2 && p.sp.ng == 1 &&
          (size_t)4 * m * ldo * 4 <= w.kpart.bytes) {
        WgemmArgs a;
        a.x = xin; a.M = m; a.K = K / 4; a.ldx = K;
        a.w = W; a.N = N; a.ldo = ldo;
        a.ur = p.sp.ur(); a.kc = 1;
        a.part_out = w.kpart.as<float>();
        a.stamps = stamp_buf();
        launch_wgemm_kslice(a, N / 16, s);
        bf16_t* o = out ? out + (size_t)r0 * ldo : nullptr;
        bf16_t* rs = resid ? resid + (size_t)r0 * ldo : nullptr;
        if (epi == EPI_STORE && defer_qkv_combine) {  // the decode attention sums the partials
          qkv_part_pending = true;
        } else if (epi == EPI_RESID && next_norm && rows <= 32) {
          launch_splitk_combine_norm(w.kpart.as<float>(), 4, m, N, ldo, rs, ldo, next_norm, c.rms_norm_eps,
                                     w.xn.as<bf16_t>() + (size_t)r0 * ldo, ldo, s);
          pending_norm = next_norm;
        } else {
          launch_splitk_combine(w.kpart.as<float>(), 4, m, N, ldo, o, rs, ldo, s);
        }
        continue;
      }
      WgemmArgs a;
      if (logit_extra) {
        a = *logit_extra;
        if (r0 > 0) {  // per-row operands of the lm_head epilogue start at row r0
          if (a.seen) a.seen += (size_t)r0 * a.seen_stride;
          if (a.eos_mask) a.eos_mask += r0;
          if (a.part_val) a.part_val += (size_t)r0 * a.part_stride;
          if (a.part_idx) a.part_idx += (size_t)r0 * a.part_stride;
          if (a.logits_out) a.logits_out += (size_t)r0 * a.ldl;
          if (a.counts) a.counts += (size_t)r0 * a.seen_stride * 32;
        }
      }
      a.x = xin; a.M = m; a.K = K; a.ldx = K;
      a.w = W; a.N = N;
      a.stamps = stamp_buf();
      a.normw = normw; a.eps = c.rms_norm_eps;
      a.out = out ? out + (size_t)r0 * ldo : nullptr; a.ldo = ldo;
      a.resid = resid ? resid + (size_t)r0 * ldo : nullptr;
      if (p.sliced) a.part_out = w.kpart.as<float>();
      // the next RMSNorm once per row: in the K-sliced launch's combine (the combine is per row),
      // or (unsliced residual launches, 2..32 rows) by norm workgroups appended to the launch
      const bool fuse_norm = p.sliced && epi == EPI_RESID && next_norm && (m > 16 || norm_once_ok(rows)) &&
                             rows <= 32 && N <= 8192;
      if (fuse_norm) {
        a.next_norm = next_norm;
        a.norm_out = w.xn.as<bf16_t>() + (size_t)r0 * ldo;
      }
      const bool nrm = !p.sliced && epi == EPI_RESID && next_norm && norm_once_ok(rows) && decoding && rows == m &&
                       (norm_once_mode() == 1 || (norm_once_mode() == 2 && nrm_region == 0));
      if (nrm) set_norm_wgs(a, m, next_norm, w.xgran.as<uint64_t>() + xgran_region(nrm_region), N);
      launch_wgemm(a, p, epi, norm, s);
      if (fuse_norm || nrm) pending_norm = next_norm;
    }
  }

  AttnArgs attn_args(int layer, int rows, const int* slot, const int* pos, bool decode) {
    AttnArgs a;
    const int H = c.num_heads, KVH = c.num_kv_heads, D = c.head_dim;
    const size_t kv_layer = (size_t)c.max_batch * KVH * w.kv_stride * D;
    a.qkv = w.qkv.as<bf16_t>(); a.ld_qkv = QKV(); a.rows = rows;
    a.row_slot = slot; a.row_pos = pos;
    a.kcache = w.kv.as<bf16_t>() + (size_t)layer * 2 * kv_layer;
    a.vtcache = a.kcache + kv_layer;
    a.max_seq = w.kv_stride;
    a.rope_cos = M.rope.as<bf16_t>();
    a.rope_sin = a.rope_cos + (size_t)c.max_seq_len * D;
    a.H = H; a.KVH = KVH; a.D = D;
    a.scale = (float)(1.0 / sqrt((double)D));
    a.q_rot = w.q_rot.as<bf16_t>(); a.out = w.attn_out.as<bf16_t>();
    a.blocks = w.blocks.as<int4>(); a.nblocks = w.nblocks;
    a.stamps = stamp_buf();
    if (decode && qkv_part_pending) {
      a.qkv_part = w.kpart.as<float>();
      a.qkv_nsl = 4;
    }
    return a;
  }

  // The one-row decode step's QKV launch carries the attention (TTS-1 geometry: head dim 64);
  // consecutive fused launches differ in (pos, layer)
  bool fused_attn_ok(int rows, bool decode) const {
    if (!decode || !use_fused_attn() || c.num_layers < 2 || c.num_layers > 64) return false;
    if (rows == 1) return c.head_dim == 64 && wgemm_fattn_ok(QKV(), c.hidden_size, e->num_cu);
    // 2..16 rows by default (TTS_FATTN_ROWS = the largest batch that fuses; 0: none; up to 32:
    // at 17..32 rows two m-tiles, the rows staged pre-normalised by the previous down
    // projection's combine — measured slower than the K-sliced seven-launch layer, round 6:
    // 32 rows 978 -> 1,041 us, profiles/r6b_ab_frows32.txt): the attention workgroups after the
    // projection's (deadlock-free order)
    static const int max_rows = getenv("TTS_FATTN_ROWS") ? atoi(getenv("TTS_FATTN_ROWS")) : 16;
    static const bool first = getenv("TTS_FATTN_FIRST") && atoi(getenv("TTS_FATTN_FIRST"));
    return rows <= std::min(32, max_rows) && !first && wgemm_fattn_rows_ok(rows, QKV(), c.hidden_size, c.head_dim, e->num_cu);
  }
  WgemmArgs fused_attn_args(const AttnArgs& a, int layer, bool with_oproj = false) {
    WgemmArgs fx;
    fx.gran = w.gran.as<uint64_t>();
    fx.fa = a;
    fx.fattn_wgs = a.rows * a.KVH;
    fx.fattn_layer = layer;
    fx.fattn_err = w.ferr.as<int>();
    // TTS_FATTN_FIRST=1: round 3's order (attention workgroups first, o_proj on the projection
    // workgroups; needs the whole grid resident); default: the deadlock-free order
    static const bool first = getenv("TTS_FATTN_FIRST") && atoi(getenv("TTS_FATTN_FIRST"));
    fx.fattn_first = first ? 1 : 0;
    // TTS_FATTN_SPINS: polls before a granule wait gives up (tests drive the failure path with it)
    static const int spins = getenv("TTS_FATTN_SPINS") ? std::max(1, atoi(getenv("TTS_FATTN_SPINS"))) : (1 << 16);
    fx.fattn_spins = spins;
    if (with_oproj) {
      const LmLayer& ly = M.layers[layer];
      const WgemmPlan po = plan_wgemm(a.rows, c.hidden_size, c.num_heads * c.head_dim, EPI_RESID, e->num_cu);
      fx.fo_w = ly.wo;
      fx.fo_units = c.hidden_size / 16;
      fx.fo_ur = po.sp.ur();
      fx.fo_kc = po.sp.kc;
      fx.fo_resid = w.x.as<bf16_t>();
    }
    return fx;
  }
  // o_proj can ride the fused QKV + attention launch: its stream plan has the launch's shape
  // (16 waves, 2-tile stages, K split 16 ways, one K chunk, two stages = the ring), one round
  // of units, at most one unit per projection workgroup, 128 K values per wave
  bool fused_oproj_ok() const {
    if (!use_fused_oproj()) return false;
    const int HD = c.num_heads * c.head_dim, HID = c.hidden_size;
    const WgemmPlan pq = plan_wgemm(1, QKV(), HID, EPI_STORE, e->num_cu);
    const WgemmPlan po = plan_wgemm(1, HID, HD, EPI_RESID, e->num_cu);
    const StreamPlan& s = po.sp;
    return s.waves == 16 && s.ku == 2 && s.ksplit == 16 && s.kc == 1 && s.ng == 1 && HD == 16 * 128 &&
           (HD / 32) / (s.ksplit * s.ku) == 2 && HID / 16 <= s.ur() && HID / 16 <= pq.sp.grid &&
           pq.sp.waves == 16 && pq.sp.ku == 2 && pq.sp.ksplit == 16;
  }

  // 2..32 rows: o_proj can ride the fused QKV + attention launch when its stream plan has the
  // launch's shape (16 waves, the QKV plan's stage width, K split 16 ways, the item = the
  // two-stage ring) and o_proj's K is the hidden size (its A rows fit the launch's LDS rows)
  bool fused_oproj_rows_ok(int rows) const {
    if (!use_fused_oproj() || !use_fused_oproj_rows() || rows < 2 || rows > 32) return false;
    const int HD = c.num_heads * c.head_dim, HID = c.hidden_size;
    const WgemmPlan pq = plan_wgemm(rows, QKV(), HID, EPI_STORE, e->num_cu);
    const WgemmPlan po = plan_wgemm(rows, HID, HD, EPI_RESID, e->num_cu);
    const StreamPlan& s = po.sp;
    return HD == HID && s.waves == 16 && s.ksplit == 16 && s.ng == 1 && s.ku == pq.sp.ku && pq.sp.waves == 16 &&
           pq.sp.ksplit == 16 && (HD / 32) / (s.ksplit * s.ku) == 2 && (HD / 32) % (s.kc * s.ksplit * s.ku) == 0 &&
           HID / 16 <= s.ur() && (2 * s.ku) % 4 == 0;
  }

  // One transformer stack pass over `rows` rows held in w.x.
  void layers(int rows, const int* slot, const int* pos, bool decode) {
    pending_norm = nullptr;  // w.x was rewritten (embeddings) since any earlier combine
    const int HID = c.hidden_size, HD = c.num_heads * c.head_dim, FF = c.intermediate_size;
    const bool fattn = fused_attn_ok(rows, decode);
    const bool foproj = fattn && (rows == 1 ? fused_oproj_ok() : fused_oproj_rows_ok(rows));
    decoding = decode;
    for (int l = 0; l < c.num_layers; ++l) {
      const LmLayer& ly = M.layers[l];
      cur_layer = l;
      AttnArgs a = attn_args(l, rows, slot, pos, decode);
      if (fattn) {
        WgemmArgs fx = fused_attn_args(a, l, foproj);
        // (2..32 rows, o_proj fused: the ln2 RMSNorm once per row by appended workgroups)
        const bool nrm = foproj && rows > 1 && norm_once_ok(rows) && norm_once_mode() <= 2;
        if (nrm) set_norm_wgs(fx, rows, ly.ln2, w.xgran.as<uint64_t>() + xgran_region(0), HID);
        gemm(w.x.as<bf16_t>(), rows, HID, ly.wqkv, QKV(), ly.ln1, w.qkv.as<bf16_t>(), QKV(), nullptr,
             EPI_STORE, &fx);
        if (nrm) pending_norm = ly.ln2;
      } else {
        // (defer: TTS_QKV_DEFER=0 keeps the combine launch)
        defer_qkv_combine = decode && rows > 16 && rows <= 32 && use_qkv_defer();
        qkv_part_pending = false;
        gemm(w.x.as<bf16_t>(), rows, HID, ly.wqkv, QKV(), ly.ln1, w.qkv.as<bf16_t>(), QKV(), nullptr,
             EPI_STORE);
        defer_qkv_combine = false;
        if (qkv_part_pending) a = attn_args(l, rows, slot, pos, decode);
        qkv_part_pending = false;
      }
      // attention output (bf16 rows of w.attn_out): inside the QKV launch (one-row step), one
      // workgroup per (row, kv head) (decode), or per query block x kv head (prefill)
      if (fattn) {
      } else if (decode) {
        launch_attn_decode_step(a, s);
      } else {
        launch_rope_append(a, s);
        launch_attn_prefill(a, s);
      }
      nrm_region = 0;
      if (!foproj)  // (decode: o_proj's combine may normalise with ln2 for the gate/up launch)
        gemm(w.attn_out.as<bf16_t>(), rows, HD, ly.wo, HID, nullptr, nullptr, HID, w.x.as<bf16_t>(), EPI_RESID,
             nullptr, decode || rows > kPrefillChunk ? ly.ln2 : nullptr);
      gemm(w.x.as<bf16_t>(), rows, HID, ly.wgu, 2 * FF, ly.ln2, w.act.as<bf16_t>(), FF, nullptr,
           EPI_SWIGLU);
      const bf16_t* next_norm = (l + 1 < c.num_layers) ? M.layers[l + 1].ln1 : M.final_norm;
      nrm_region = 1;
      // (prefill GEMMs of > kPrefillChunk rows: the one-chunk form's combine may normalise too;
      // not after the last layer, whose rows only the gathered lm_head rows read)
      gemm(w.act.as<bf16_t>(), rows, FF, ly.wd, HID, nullptr, nullptr, HID, w.x.as<bf16_t>(), EPI_RESID, nullptr,
           decode ? next_norm : (rows > kPrefillChunk && l + 1 < c.num_layers ? next_norm : nullptr));
    }
  }

  StepState state(int B, int eos, int min_new) {
    StepState st;
    int* base = w.st_int.as<int>();
    st.tokens = base;
    st.pos = base + B;
    st.gen_count = base + 2 * B;
    st.limit = base + 3 * B;
    st.done = base + 4 * B;
    st.eos_mask = base + 5 * B;
    st.n_active = base + 6 * B;
    st.seen = w.seen.as<uint32_t>();
    st.seen_stride = c.vocab_size / 32 + 1;
    st.counts = nullptr;
    st.row_seed = w.row_seed.as<unsigned long long>();
    st.epoch = w.epoch.as<uint32_t>();
    st.out_ids = w.out_ids.as<int>();
    st.out_stride = w.out_cap;
    st.eos_id = eos;
    st.min_new = min_new;
    return st;
  }

  // lm_head over B rows of `xin` + the pick (greedy argmax, or the sampling head) + finalize
  // (state update, next embedding -> w.x)
  void head_and_pick(const bf16_t* xin, int B, const StepState& st, const tts_gen_params& gp) {
    if (!gp.do_sample && M.head_grid && head_screen_supported(B, c.hidden_size, c.vocab_size)) {
      screened_head(xin, B, st, gp);
      return;
    }
    WgemmArgs ex;
    ex.seen = st.seen; ex.seen_stride = st.seen_stride; ex.penalty = gp.repetition_penalty;
    ex.eos_mask = st.eos_mask;
    ex.part_val = w.lpart_v.as<float>(); ex.part_idx = w.lpart_i.as<int>();
    ex.part_stride = LOGITS_MAX_PARTS;
    if (gp.do_sample) { ex.logits_out = w.slogits.as<float>(); ex.ldl = c.vocab_size; }
    ex.counts = st.counts; ex.freq_penalty = gp.frequency_penalty;
    TTS_REQUIRE(B <= kPrefillChunk, "batch larger than one GEMM chunk");
    WgemmPlan p = plan_wgemm(B, c.vocab_size, c.hidden_size, EPI_LOGITS, e->num_cu);
    gemm(xin, B, c.hidden_size, M.lm_head, c.vocab_size, M.final_norm, nullptr, 0, nullptr,
         EPI_LOGITS, &ex);
    int nparts = p.grid;
    if (gp.do_sample) {
      SampleArgs sa;
      sa.logits = w.slogits.as<float>(); sa.ldl = c.vocab_size; sa.V = c.vocab_size;
      sa.temperature = gp.temperature; sa.top_k = gp.top_k; sa.top_p = gp.top_p;
      sa.seed = gp.seed; sa.row_seed = st.row_seed; sa.step = st.gen_count; sa.done = st.done;
      sa.part_val = ex.part_val; sa.nparts = p.grid; sa.part_stride = LOGITS_MAX_PARTS;
      sa.out_part_val = ex.part_val; sa.out_part_idx = ex.part_idx;
      launch_sample(sa, B, s);
      nparts = 1;
    }
    launch_finalize_greedy(ex.part_val, ex.part_idx, LOGITS_MAX_PARTS, nparts, st, B,
                           M.embed_rows.as<bf16_t>(), w.x.as<bf16_t>(), c.hidden_size, s);
  }

  // greedy pick through the int8 screen + exact recheck (lm_head_screen.hip): the same ids as
  // the full lm_head launch above
  void screened_head(const bf16_t* xin, int B, const StepState& st, const tts_gen_params& gp) {
    const int rg = screened_head_parts(xin, B, st, gp);
    launch_finalize_greedy(w.lpart_v.as<float>(), w.lpart_i.as<int>(), LOGITS_MAX_PARTS, rg, st, B,
                           M.embed_rows.as<bf16_t>(), w.x.as<bf16_t>(), c.hidden_size, s);
  }
  // the screened head's launch (int8 screen + exact recompute of the units that can hold the
  // argmax); returns the number of argmax partials per row
  int screened_head_parts(const bf16_t* xin, int B, const StepState& st, const tts_gen_params& gp) {
    const int HID = c.hidden_size, V = c.vocab_size;
    HeadScreenArgs a;
    a.M = B; a.K = HID; a.ldx = HID; a.V = V;
    const bool ready = pending_norm == M.final_norm && xin == w.x.as<bf16_t>();  // (a residual combine
    if (ready) {                                                                 //  wrote RMSNorm(x, final norm))
      a.x = w.xn.as<bf16_t>();
    } else if (head_screen_prequant(B)) {
      launch_rmsnorm(xin, HID, M.final_norm, c.rms_norm_eps, w.xn.as<bf16_t>(), HID, B, HID, s);
      a.x = w.xn.as<bf16_t>();
    } else {
      a.x = xin; a.normw = M.final_norm; a.eps = c.rms_norm_eps;
    }
    if (head_screen_prequant(B)) {  // (17..32 rows: quantised once, not by every workgroup)
      launch_head_rowquant(a.x, HID, B, HID, w.hxq.as<int8_t>(), w.hxs.as<float>(), s);
      a.xq = w.hxq.as<int8_t>(); a.xstat = w.hxs.as<float>();
    }
    a.q = M.head_q.as<int8_t>(); a.cst = M.head_c.as<float4>();
    a.ur = M.head_grid * head_screen_waves();
    a.w = M.lm_head;
    const StreamPlan sp = stream_plan(V, HID, 1, e->num_cu);
    a.hku = sp.ku; a.hur = sp.ur(); a.hKT = HID / 32; a.hkc = sp.kc;
    a.seen = st.seen; a.seen_stride = st.seen_stride; a.penalty = gp.repetition_penalty;
    a.eos_mask = st.eos_mask; a.counts = st.counts; a.freq_penalty = gp.frequency_penalty;
    a.epoch = st.epoch; a.lbg = w.hlb.as<unsigned long long>();
    a.arrive = (uint32_t*)(w.hlb.as<unsigned long long>() + 32 * 8);
    a.spins = head_screen_wait(B) ? (1 << 14) : 0;
    a.part_val = w.lpart_v.as<float>(); a.part_idx = w.lpart_i.as<int>(); a.part_stride = LOGITS_MAX_PARTS;
    if (head_screen_check()) {
      a.check = 1; a.ub = w.hub.as<float>(); a.ldu = V; a.err = w.ferr.as<int>() + 1;
    }
    static const int diag = getenv("TTS_HEAD_SCREEN_DIAG") ? atoi(getenv("TTS_HEAD_SCREEN_DIAG")) : 0;
    a.diag = diag;
    if (diag & 2) a.err = w.ferr.as<int>() + 1;  // (the count lands in ferr[3])
    launch_head_screen(a, M.head_grid, s);
    return M.head_grid;
  }
};

}  // namespace

static void check_launch() { HIP_CHECK(hipGetLastError()); }

// Prefill a group of sequences [b0, b0+nb): rows = sum of their prompt lengths.
static void prefill_rows_setup(Ctx& X, const int32_t* ids, const int32_t* lens, int B, int slot_base,
                               std::vector<int>& last_rows, int& rows) {
  std::vector<int> slot, pos, tok, blk;
  rows = 0;
  last_rows.resize(B);
  for (int b = 0; b < B; ++b) {
    for (int i = 0; i < lens[b]; ++i) {
      slot.push_back(slot_base + b);
      pos.push_back(i);
      tok.push_back(ids[rows + i]);
    }
    // attention query blocks: up to 16 consecutive rows of one sequence (lm_attn.hip)
    for (int t0 = 0; t0 < lens[b]; t0 += 16)
      blk.insert(blk.end(), {rows + t0, std::min(16, lens[b] - t0), slot_base + b, t0});
    rows += lens[b];
    last_rows[b] = rows - 1;
  }
  TTS_REQUIRE(rows <= X.w.cap_rows, "total prompt rows exceed the prefill workspace");
  X.w.nblocks = (int)blk.size() / 4;
  HIP_CHECK(hipMemcpyAsync(X.w.blocks.p, blk.data(), blk.size() * 4, hipMemcpyHostToDevice, X.s));
  HIP_CHECK(hipMemcpyAsync(X.w.row_slot.p, slot.data(), rows * 4, hipMemcpyHostToDevice, X.s));
  HIP_CHECK(hipMemcpyAsync(X.w.row_pos.p, pos.data(), rows * 4, hipMemcpyHostToDevice, X.s));
  HIP_CHECK(hipMemcpyAsync(X.w.row_idx.p, tok.data(), rows * 4, hipMemcpyHostToDevice, X.s));
  launch_embed(X.w.row_idx.as<int>(), X.M.embed_rows.as<bf16_t>(), X.w.x.as<bf16_t>(), rows,
               X.c.hidden_size, X.s);
  // the fused QKV + attention launch tags its granules (position, layer): a sequence starting
  // over at a position an earlier sequence reached must not find that sequence's granules
  // (with a matching tag the attention workgroups could read them before this step's QKV
  // workgroups overwrite them)
  HIP_CHECK(hipMemsetAsync(X.w.gran.p, 0xff, X.w.gran.bytes, X.s));
  HIP_CHECK(hipMemsetAsync(X.w.xgran.p, 0xff, X.w.xgran.bytes, X.s));
}

// The decode step (all layers + lm_head + pick + finalize over B rows) captured once into a
// hipGraph.  The graph bakes in B, the penalty, eos/min_new and the sampling parameters
// (kernel arguments): recaptured when any of them changes.  The sampling keys are per-row
// device values (w.row_seed), so a new seed needs no recapture.
static void ensure_step_graph(Engine* e, int B, const StepState& st, const tts_gen_params& gp) {
  LmWork& W = e->w;
  const tts_gen_params* p = &gp;
  const float pen = p->repetition_penalty;
  const bool smp_changed =
      W.graph_sample != p->do_sample ||
      (p->do_sample && (W.graph_temp != p->temperature || W.graph_top_k != p->top_k ||
                        W.graph_top_p != p->top_p)) ||
      W.graph_freq != p->frequency_penalty;
  if (W.graph && (W.graph_batch != B || W.graph_pen != pen || W.graph_eos != p->eos_token_id ||
                  W.graph_min_new != p->min_new_tokens || smp_changed)) {
    (void)hipGraphExecDestroy(W.graph);
    W.graph = nullptr;
  }
  if (W.graph) return;
  auto step = [&](hipStream_t ss) {
    Ctx Y(e, ss);
    Y.layers(B, W.row_slot.as<int>(), st.pos, true);
    Y.head_and_pick(W.x.as<bf16_t>(), B, st, gp);
  };
  hipStream_t cs;
  HIP_CHECK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  hipGraph_t g;
  HIP_CHECK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
  step(cs);
  HIP_CHECK(hipStreamEndCapture(cs, &g));
  HIP_CHECK(hipGraphInstantiate(&W.graph, g, nullptr, nullptr, 0));
  HIP_CHECK(hipGraphDestroy(g));
  HIP_CHECK(hipStreamDestroy(cs));
  W.graph_batch = B;
  W.graph_pen = pen;
  W.graph_eos = p->eos_token_id;
  W.graph_min_new = p->min_new_tokens;
  W.graph_sample = p->do_sample;
  W.graph_temp = p->temperature;
  W.graph_top_k = p->top_k;
  W.graph_top_p = p->top_p;
  W.graph_freq = p->frequency_penalty;
}

void lm_gen_begin(Engine* e, const tts_gen_params* p, const int32_t* ids, const int32_t* lens, int B,
                  hipStream_t s) {
  TTS_REQUIRE(e->lm.loaded, "tts_lm_load has not been called");
  e->slots.open = false;
  TTS_REQUIRE(p != nullptr && ids != nullptr && lens != nullptr, "null argument");
  TTS_REQUIRE(B >= 1 && B <= e->w.cap_batch, "batch out of range");
  if (p->do_sample) {  // HF: TemperatureLogitsWarper requires T > 0; top_k from GenerationConfig (50)
    TTS_REQUIRE(p->temperature > 0.f, "sampling needs temperature > 0 (temperature 0 = greedy)");
    TTS_REQUIRE(p->top_k >= 1 && p->top_k <= SAMPLE_MAX_TOP_K,
                "sampling supports top_k in [1, 1024] (HF default 50; full-vocabulary sampling is not built)");
    TTS_REQUIRE(p->top_p > 0.f && p->top_p <= 1.f, "top_p must be in (0, 1]");
  }
  Ctx X(e, s);
  const tts_lm_config& c = X.c;
  const int V = c.vocab_size;
  // ---- host-side state init
  std::vector<int> st_host(7 * B + 1, 0);
  std::vector<uint32_t> seen((size_t)B * (V / 32 + 1), 0u);
  int max_new = 0, off = 0;
  for (int b = 0; b < B; ++b) {
    const int P = lens[b];
    TTS_REQUIRE(P >= 1, "empty prompt");
    // HF: max_length counts the prompt; input length >= max_length is a ValueError
    // (generation/utils.py _validate_generated_length)
    TTS_REQUIRE(P < p->max_length, "input length >= max_length");
    const int limit = p->max_length - P;
    TTS_REQUIRE(P + limit <= c.max_seq_len, "prompt + max new tokens exceed max_seq_len");
    TTS_REQUIRE(limit <= e->w.out_cap, "max new tokens exceed the output capacity");
    for (int i = 0; i < P; ++i) {
      const int t = ids[off + i];
      TTS_REQUIRE(t >= 0 && t < V, "token id out of range");
      seen[(size_t)b * (V / 32 + 1) + (t >> 5)] |= 1u << (t & 31);
    }
    off += P;
    st_host[1 * B + b] = P - 1;  // pos: finalize advances it to P for the first new token
    st_host[3 * B + b] = limit;
    st_host[5 * B + b] = (p->min_new_tokens > 0) ? p->eos_token_id : -1;
    max_new = std::max(max_new, limit);
  }
  st_host[6 * B] = B;
  StepState st = X.state(B, p->eos_token_id, p->min_new_tokens);
  TTS_REQUIRE(std::isfinite(p->frequency_penalty), "frequency_penalty must be finite");
  if (p->frequency_penalty != 0.f) {  // vLLM form: counts of the new tokens only
    st.counts = e->w.counts.as<uint16_t>();
    HIP_CHECK(hipMemsetAsync(st.counts, 0, (size_t)B * st.seen_stride * 32 * 2, s));
  }
  HIP_CHECK(hipMemcpyAsync(e->w.st_int.p, st_host.data(), st_host.size() * 4,
                           hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(e->w.seen.p, seen.data(), seen.size() * 4, hipMemcpyHostToDevice, s));
  {  // row b draws with key seed + GOLD * (b << 32)  (rng_uniform(key, 0, step))
    std::vector<unsigned long long> rs(B);
    for (int b = 0; b < B; ++b) rs[b] = p->seed + 0x9E3779B97F4A7C15ull * ((unsigned long long)b << 32);
    HIP_CHECK(hipMemcpyAsync(e->w.row_seed.p, rs.data(), B * 8, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));  // (rs is a stack buffer)
  }
  // rows' slots are 0..B-1 in the decode phase: prepare a persistent identity map
  HIP_CHECK(hipEventRecord(e->ev[2], s));

  // ---- prefill
  // groups of whole prompts that fit the prefill workspace, each in one pass
  {
    std::vector<int> last_rows;
    int b0 = 0;
    size_t id_off = 0;
    while (b0 < B) {
      int b1 = b0, grp_rows = 0;
      while (b1 < B && grp_rows + lens[b1] <= e->w.cap_rows) grp_rows += lens[b1++];
      TTS_REQUIRE(b1 > b0, "a prompt is longer than the prefill workspace");
      int rows = 0;
      prefill_rows_setup(X, ids + id_off, lens + b0, b1 - b0, b0, last_rows, rows);
      X.layers(rows, e->w.row_slot.as<int>(), e->w.row_pos.as<int>(), false);
      HIP_CHECK(hipMemcpyAsync(e->w.row_idx.p, last_rows.data(), (b1 - b0) * 4, hipMemcpyHostToDevice, s));
      launch_gather_rows(e->w.x.as<bf16_t>(), c.hidden_size, e->w.row_idx.as<int>(),
                         e->w.last_x.as<bf16_t>() + (size_t)b0 * c.hidden_size, b1 - b0, c.hidden_size, s);
      id_off += grp_rows;
      b0 = b1;
    }
  }
  X.head_and_pick(e->w.last_x.as<bf16_t>(), B, st, *p);
  check_launch();
  HIP_CHECK(hipEventRecord(e->ev[3], s));

  // ---- decode: identity slot map; positions live in the step state
  std::vector<int> ident(B);
  for (int b = 0; b < B; ++b) ident[b] = b;
  HIP_CHECK(hipMemcpyAsync(e->w.row_slot.p, ident.data(), B * 4, hipMemcpyHostToDevice, s));
  // (the embedding of each sequence's next token is already in w.x rows 0..B-1)
  ensure_step_graph(e, B, st, *p);
  Engine::Gen& G = e->gen;
  G.open = true;
  G.B = B;
  G.max_new = max_new;
  G.launched = 1;  // the prefill's head produced the first token
  G.polls = 0;
  G.finished = max_new <= 1;
  G.s = s;
  e->decode_steps = 0;
}

// Up to n_steps decode-step graph replays.  The host polls the device's active-row counter
// every kPollEvery steps, one poll behind (no per-step D->H sync; HF syncs every step,
// generation/utils.py:2936-2937): a stopped row runs idle (its kernels skip it) until the
// poll sees every row done.
int lm_gen_continue(Engine* e, int n_steps) {
  Engine::Gen& G = e->gen;
  TTS_REQUIRE(G.open, "no generation in progress (tts_generate_begin)");
  const hipStream_t s = G.s;
  const StepState st = Ctx(e, s).state(G.B, e->w.graph_eos, e->w.graph_min_new);
  for (int n = 0; n < n_steps && !G.finished; ++n) {
    if (G.launched >= G.max_new) { G.finished = true; break; }
    HIP_CHECK(hipGraphLaunch(e->w.graph, s));
    ++G.launched;
    ++e->decode_steps;
    if (G.launched % kPollEvery == 0) {
      const int slot = G.polls & 1;
      HIP_CHECK(hipMemcpyAsync(&e->w.h_active[slot], st.n_active, 4, hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipEventRecord(e->ev[slot], s));
      if (G.polls > 0) {
        HIP_CHECK(hipEventSynchronize(e->ev[slot ^ 1]));
        if (e->w.h_active[slot ^ 1] == 0) G.finished = true;
      }
      ++G.polls;
    }
  }
  if (G.launched >= G.max_new) G.finished = true;
  if (!G.finished) {  // exact answer for a streaming caller: sync once per chunk
    int act = 0;
    HIP_CHECK(hipMemcpyAsync(&act, st.n_active, 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (act == 0) G.finished = true;
  }
  return G.finished ? 1 : 0;
}

// A fused QKV+attention launch whose granule wait timed out leaves garbage: fail loudly at
// the next read (the flag is cleared for the next generation).
static void check_fattn(Engine* e, hipStream_t s) {
  if (!e->w.ferr.p) return;
  int err[4] = {0, 0, 0, 0};
  HIP_CHECK(hipMemcpyAsync(err, e->w.ferr.p, 16, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (err[3]) {  // (TTS_HEAD_SCREEN_DIAG=2: units the screen recomputed since the last read)
    fprintf(stderr, "head screen: %d units recomputed\n", err[3]);
    HIP_CHECK(hipMemsetAsync((int*)e->w.ferr.p + 3, 0, 4, s));
  }
  if (err[0] || err[1]) {
    HIP_CHECK(hipMemsetAsync(e->w.ferr.p, 0, 8, s));
    HIP_CHECK(hipStreamSynchronize(s));
    TTS_REQUIRE(!err[0], "fused QKV+attention: a granule wait timed out (results invalid)");
    TTS_REQUIRE(false, "screened lm_head: an exact score above its int8 bound (TTS_HEAD_SCREEN_CHECK)");
  }
}

void lm_gen_read(Engine* e, int32_t* out_ids, int out_stride, int32_t* out_lens) {
  Engine::Gen& G = e->gen;
  TTS_REQUIRE(G.open, "no generation in progress (tts_generate_begin)");
  const hipStream_t s = G.s;
  const StepState st = Ctx(e, s).state(G.B, e->w.graph_eos, e->w.graph_min_new);
  std::vector<int> gc(G.B);
  HIP_CHECK(hipMemcpyAsync(gc.data(), st.gen_count, G.B * 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  check_fattn(e, s);
  for (int b = 0; b < G.B; ++b) {
    TTS_REQUIRE(gc[b] <= out_stride, "out_stride too small");
    out_lens[b] = gc[b];
    HIP_CHECK(hipMemcpy(out_ids + (size_t)b * out_stride, st.out_ids + (size_t)b * st.out_stride,
                        (size_t)gc[b] * 4, hipMemcpyDeviceToHost));
  }
}

void lm_generate(Engine* e, const tts_gen_params* p, const int32_t* ids, const int32_t* lens,
                 int B, int32_t* out_ids, int out_stride, int32_t* out_lens, hipStream_t s) {
  for (int b = 0; b < B; ++b)
    TTS_REQUIRE(p->max_length - lens[b] <= out_stride, "out_stride too small");
  lm_gen_begin(e, p, ids, lens, B, s);
  const int max_new = e->gen.max_new;
  lm_gen_continue(e, max_new);
  HIP_CHECK(hipEventRecord(e->ev[1], s));
  lm_gen_read(e, out_ids, out_stride, out_lens);
  float t0 = 0.f, t1 = 0.f;
  HIP_CHECK(hipEventElapsedTime(&t0, e->ev[2], e->ev[3]));
  HIP_CHECK(hipEventElapsedTime(&t1, e->ev[3], e->ev[1]));
  e->t_prefill_ms = t0;
  e->t_decode_ms = t1;
  e->gen.open = false;
}

// ---------------------------------------------------------------- continuous batching --
// S persistent rows (slots) share one captured decode step; a sequence is admitted into a
// free slot between chunks (its prompt prefilled into that slot's KV strip, its first token
// picked, its step-state row initialised) and retired when it stops.  Rows never mix, so
// every sequence's tokens equal a batch-1 generate of its prompt with the shared settings.
static void validate_gen_params(const tts_gen_params* p) {
  TTS_REQUIRE(p != nullptr, "null argument");
  if (p->do_sample) {
    TTS_REQUIRE(p->temperature > 0.f, "sampling needs temperature > 0 (temperature 0 = greedy)");
    TTS_REQUIRE(p->top_k >= 1 && p->top_k <= SAMPLE_MAX_TOP_K,
                "sampling supports top_k in [1, 1024] (HF default 50; full-vocabulary sampling is not built)");
    TTS_REQUIRE(p->top_p > 0.f && p->top_p <= 1.f, "top_p must be in (0, 1]");
  }
  TTS_REQUIRE(std::isfinite(p->frequency_penalty), "frequency_penalty must be finite");
}

static StepState slots_state(Engine* e, hipStream_t s) {
  Engine::Slots& Z = e->slots;
  StepState st = Ctx(e, s).state(Z.S, Z.gp.eos_token_id, Z.gp.min_new_tokens);
  if (Z.gp.frequency_penalty != 0.f) st.counts = e->w.counts.as<uint16_t>();
  return st;
}

void lm_slots_open(Engine* e, const tts_gen_params* p, int S, hipStream_t s) {
  TTS_REQUIRE(e->lm.loaded, "tts_lm_load has not been called");
  validate_gen_params(p);
  TTS_REQUIRE(S >= 1 && S <= e->w.cap_batch, "slot count out of range (max_batch)");
  e->gen.open = false;
  Engine::Slots& Z = e->slots;
  Z.open = true;
  Z.S = S;
  Z.gp = *p;
  Z.busy.assign(S, 0);
  Z.next_req = 0;
  Z.s = s;
  const int V = e->lm.cfg.vocab_size;
  // every row idle: done = 1, n_active = 0, no EOS mask
  std::vector<int> st_host(7 * S + 1, 0);
  for (int b = 0; b < S; ++b) { st_host[4 * S + b] = 1; st_host[5 * S + b] = -1; }
  HIP_CHECK(hipMemcpyAsync(e->w.st_int.p, st_host.data(), st_host.size() * 4, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemsetAsync(e->w.seen.p, 0, (size_t)S * (V / 32 + 1) * 4, s));
  std::vector<int> ident(S);
  for (int b = 0; b < S; ++b) ident[b] = b;
  HIP_CHECK(hipMemcpyAsync(e->w.row_slot.p, ident.data(), S * 4, hipMemcpyHostToDevice, s));
  const StepState st = slots_state(e, s);
  ensure_step_graph(e, S, st, Z.gp);
  HIP_CHECK(hipStreamSynchronize(s));
}

// seed: the request's sampling key (vLLM SamplingParams.seed); nullptr = the batch seed
// mixed with a request counter, so every request draws its own stream
void lm_slots_add(Engine* e, int slot, const int32_t* prompt, int len, int max_new, const uint64_t* seed) {
  Engine::Slots& Z = e->slots;
  TTS_REQUIRE(Z.open, "no slot batch open (tts_slots_open)");
  TTS_REQUIRE(slot >= 0 && slot < Z.S && !Z.busy[slot], "slot out of range or busy");
  TTS_REQUIRE(prompt != nullptr && len >= 1, "empty prompt");
  const tts_lm_config& c = e->lm.cfg;
  const int V = c.vocab_size;
  TTS_REQUIRE(max_new >= 1 && len + max_new <= c.max_seq_len && max_new <= e->w.out_cap,
              "prompt + max new tokens exceed max_seq_len");
  TTS_REQUIRE(len <= e->w.cap_rows, "prompt longer than the prefill workspace");
  const hipStream_t s = Z.s;
  Ctx X(e, s);
  StepState st = slots_state(e, s);
  const int S = Z.S, stride = st.seen_stride;
  // ---- the slot's step-state row (and its penalty set) on the device
  std::vector<uint32_t> seen((size_t)stride, 0u);
  for (int i = 0; i < len; ++i) {
    TTS_REQUIRE(prompt[i] >= 0 && prompt[i] < V, "token id out of range");
    seen[prompt[i] >> 5] |= 1u << (prompt[i] & 31);
  }
  HIP_CHECK(hipMemcpyAsync(st.seen + (size_t)slot * stride, seen.data(), (size_t)stride * 4,
                           hipMemcpyHostToDevice, s));
  if (st.counts) HIP_CHECK(hipMemsetAsync(st.counts + (size_t)slot * stride * 32, 0, (size_t)stride * 32 * 2, s));
  const int row[6] = {0, len - 1, 0, max_new, 0, (Z.gp.min_new_tokens > 0) ? Z.gp.eos_token_id : -1};
  int* base = e->w.st_int.as<int>();
  for (int k = 0; k < 6; ++k)  // tokens, pos, gen_count, limit, done, eos_mask
    HIP_CHECK(hipMemcpyAsync(base + k * S + slot, &row[k], 4, hipMemcpyHostToDevice, s));
  // the row's sampling key: the same for its first token (drawn below as a batch of 1) and
  // for every decode step (row = slot)
  const unsigned long long key =
      seed ? (unsigned long long)*seed : Z.gp.seed + 0x9E3779B97F4A7C15ull * ((++Z.next_req) << 32);
  HIP_CHECK(hipMemcpyAsync(st.row_seed + slot, &key, 8, hipMemcpyHostToDevice, s));
  int act = 0;
  HIP_CHECK(hipMemcpyAsync(&act, st.n_active, 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  ++act;
  HIP_CHECK(hipMemcpyAsync(st.n_active, &act, 4, hipMemcpyHostToDevice, s));
  // ---- prefill the prompt into the slot's KV strip, pick its first token
  std::vector<int> last_rows;
  int rows = 0;
  prefill_rows_setup(X, prompt, &len, 1, slot, last_rows, rows);
  X.layers(rows, e->w.row_slot.as<int>(), e->w.row_pos.as<int>(), false);
  HIP_CHECK(hipMemcpyAsync(e->w.row_idx.p, last_rows.data(), 4, hipMemcpyHostToDevice, s));
  launch_gather_rows(e->w.x.as<bf16_t>(), c.hidden_size, e->w.row_idx.as<int>(), e->w.last_x.as<bf16_t>(), 1,
                     c.hidden_size, s);
  StepState one = st;  // the slot's row as a batch of 1
  one.tokens += slot; one.pos += slot; one.gen_count += slot; one.limit += slot;
  one.done += slot; one.eos_mask += slot; one.row_seed += slot;
  one.seen += (size_t)slot * stride;
  one.out_ids += (size_t)slot * one.out_stride;
  if (one.counts) one.counts += (size_t)slot * stride * 32;
  X.head_and_pick(e->w.last_x.as<bf16_t>(), 1, one, Z.gp);
  // the prefill overwrote the decode rows of w.x: re-embed every row's next token
  std::vector<int> ident(S);
  for (int b = 0; b < S; ++b) ident[b] = b;
  HIP_CHECK(hipMemcpyAsync(e->w.row_slot.p, ident.data(), S * 4, hipMemcpyHostToDevice, s));
  launch_embed(st.tokens, e->lm.embed_rows.as<bf16_t>(), e->w.x.as<bf16_t>(), S, c.hidden_size, s);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipStreamSynchronize(s));
  Z.busy[slot] = 1;
}

int lm_slots_step(Engine* e, int n_steps) {
  Engine::Slots& Z = e->slots;
  TTS_REQUIRE(Z.open, "no slot batch open (tts_slots_open)");
  const StepState st = slots_state(e, Z.s);
  for (int n = 0; n < n_steps; ++n) HIP_CHECK(hipGraphLaunch(e->w.graph, Z.s));
  check_fattn(e, Z.s);
  int act = 0;
  HIP_CHECK(hipMemcpyAsync(&act, st.n_active, 4, hipMemcpyDeviceToHost, Z.s));
  HIP_CHECK(hipStreamSynchronize(Z.s));
  return act;
}

void lm_slots_read(Engine* e, int slot, int32_t* out_ids, int cap, int32_t* n_out, int32_t* finished) {
  Engine::Slots& Z = e->slots;
  TTS_REQUIRE(Z.open, "no slot batch open (tts_slots_open)");
  TTS_REQUIRE(slot >= 0 && slot < Z.S, "slot out of range");
  const StepState st = slots_state(e, Z.s);
  int gc = 0, dn = 0;
  HIP_CHECK(hipMemcpyAsync(&gc, st.gen_count + slot, 4, hipMemcpyDeviceToHost, Z.s));
  HIP_CHECK(hipMemcpyAsync(&dn, st.done + slot, 4, hipMemcpyDeviceToHost, Z.s));
  HIP_CHECK(hipStreamSynchronize(Z.s));
  TTS_REQUIRE(gc <= cap, "output capacity too small");
  if (gc > 0)
    HIP_CHECK(hipMemcpy(out_ids, st.out_ids + (size_t)slot * st.out_stride, (size_t)gc * 4, hipMemcpyDeviceToHost));
  *n_out = gc;
  *finished = Z.busy[slot] ? dn : 1;
}

void lm_slots_release(Engine* e, int slot) {
  Engine::Slots& Z = e->slots;
  TTS_REQUIRE(Z.open, "no slot batch open (tts_slots_open)");
  TTS_REQUIRE(slot >= 0 && slot < Z.S, "slot out of range");
  if (!Z.busy[slot]) return;
  const StepState st = slots_state(e, Z.s);
  int dn = 0;
  HIP_CHECK(hipMemcpyAsync(&dn, st.done + slot, 4, hipMemcpyDeviceToHost, Z.s));
  HIP_CHECK(hipStreamSynchronize(Z.s));
  if (!dn) {  // aborted while running: stop the row and drop it from the active count
    int act = 0;
    const int one = 1;
    HIP_CHECK(hipMemcpy(st.done + slot, &one, 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(&act, st.n_active, 4, hipMemcpyDeviceToHost));
    --act;
    HIP_CHECK(hipMemcpy(st.n_active, &act, 4, hipMemcpyHostToDevice));
  }
  Z.busy[slot] = 0;
}

void lm_bench_kernel(Engine* e, int which, int rows, int ctx, int iters, float* avg_ms,
                     double* bytes) {
  TTS_REQUIRE(e->lm.loaded, "tts_lm_load has not been called");
  TTS_REQUIRE(rows >= 1 && rows <= e->w.cap_batch, "rows out of range");
  TTS_REQUIRE(ctx >= 1 && ctx <= e->lm.cfg.max_seq_len, "ctx out of range");
  TTS_REQUIRE(which >= 0 && which <= 9 && iters >= 1, "bad kernel selector");
  TTS_REQUIRE(which < 6 || which > 7 || Ctx(e, e->stream).fused_attn_ok(rows, true),
              "fused QKV+attention does not apply to this shape");
  TTS_REQUIRE(which < 8 || (e->lm.head_grid && rows <= 32 && head_screen_supported(rows, e->lm.cfg.hidden_size,
                                                                                      e->lm.cfg.vocab_size)),
              "the screened lm_head does not apply to this shape (or is off)");
  TTS_REQUIRE(which != 7 || (rows == 1 ? Ctx(e, e->stream).fused_oproj_ok() : Ctx(e, e->stream).fused_oproj_rows_ok(rows)),
              "fused o_proj does not apply to this shape (or is off)");
  hipStream_t s = e->stream;
  Ctx X(e, s);
  const tts_lm_config& c = X.c;
  const int HID = c.hidden_size, HD = c.num_heads * c.head_dim, FF = c.intermediate_size;
  const int V = c.vocab_size, QKV = X.QKV();
  std::vector<int> tok(rows), slot(rows), pos(rows, ctx - 1);
  for (int r = 0; r < rows; ++r) { tok[r] = (r * 7919 + 11) % V; slot[r] = r; }
  HIP_CHECK(hipMemcpyAsync(e->w.row_idx.p, tok.data(), rows * 4, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(e->w.row_slot.p, slot.data(), rows * 4, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(e->w.row_pos.p, pos.data(), rows * 4, hipMemcpyHostToDevice, s));
  launch_embed(e->w.row_idx.as<int>(), X.M.embed_rows.as<bf16_t>(), e->w.x.as<bf16_t>(), rows, HID, s);
  const LmLayer& ly = X.M.layers[0];
  StepState st = X.state(rows, -1, 0);
  std::vector<int> zeros(7 * rows + 1, 0);
  for (int r = 0; r < rows; ++r) zeros[5 * rows + r] = -1;  // no EOS mask
  HIP_CHECK(hipMemcpyAsync(e->w.st_int.p, zeros.data(), zeros.size() * 4, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemsetAsync(e->w.seen.p, 0, (size_t)rows * st.seen_stride * 4, s));
  // real activations for every stage
  X.gemm(e->w.x.as<bf16_t>(), rows, HID, ly.wqkv, QKV, ly.ln1, e->w.qkv.as<bf16_t>(), QKV, nullptr, EPI_STORE);
  HIP_CHECK(hipMemsetAsync(e->w.attn_out.p, 0, (size_t)rows * HD * 2, s));
  HIP_CHECK(hipMemsetAsync(e->w.act.p, 0, (size_t)rows * FF * 2, s));
  AttnArgs aa = X.attn_args(0, rows, e->w.row_slot.as<int>(), e->w.row_pos.as<int>(), true);
  WgemmArgs ex;
  ex.seen = st.seen; ex.seen_stride = st.seen_stride; ex.penalty = 1.1f; ex.eos_mask = st.eos_mask;
  ex.part_val = e->w.lpart_v.as<float>(); ex.part_idx = e->w.lpart_i.as<int>();
  ex.part_stride = LOGITS_MAX_PARTS;
  launch_attn_decode_step(aa, s);  // (a real attention row for o_proj)
  double b = 0;
  const double act_rw = 2.0 * rows;
  // launches rotate over the layers (as the decode step does), so a layer's weights are
  // not still cached from the previous launch: the timing reflects HBM streaming
  // (experiment hook TTS_BENCH_ONE_LAYER=1: every launch on layer 0, weights L2-warm when
  // they fit the XCDs' L2s — what a cross-kernel weight prefetch could at best buy)
  static const bool one_layer = getenv("TTS_BENCH_ONE_LAYER") && atoi(getenv("TTS_BENCH_ONE_LAYER"));
  // (the fused launches tag their granules with (pos, layer): on one layer every launch would
  // match the previous launch's granules and never wait — an optimistic, stale measurement)
  TTS_REQUIRE(!(one_layer && which >= 6), "TTS_BENCH_ONE_LAYER cannot time the fused launches (selectors 6, 7)");
  int it_layer = 0;
  auto launch = [&]() {
    const int li = one_layer ? 0 : it_layer++ % c.num_layers;
    const LmLayer& ly = X.M.layers[li];
    switch (which) {
      case 0:
        X.gemm(e->w.x.as<bf16_t>(), rows, HID, ly.wqkv, QKV, ly.ln1, e->w.qkv.as<bf16_t>(), QKV, nullptr, EPI_STORE);
        b = 2.0 * QKV * HID + act_rw * (HID + QKV) + 2.0 * HID;
        break;
      case 1:
        X.gemm(e->w.attn_out.as<bf16_t>(), rows, HD, ly.wo, HID, nullptr, nullptr, HID, e->w.x.as<bf16_t>(), EPI_RESID);
        b = 2.0 * HID * HD + act_rw * (HD + 2 * HID);
        break;
      case 2:
        X.gemm(e->w.x.as<bf16_t>(), rows, HID, ly.wgu, 2 * FF, ly.ln2, e->w.act.as<bf16_t>(), FF, nullptr, EPI_SWIGLU);
        b = 2.0 * 2 * FF * HID + act_rw * (HID + FF) + 2.0 * HID;
        break;
      case 3:
        X.gemm(e->w.act.as<bf16_t>(), rows, FF, ly.wd, HID, nullptr, nullptr, HID, e->w.x.as<bf16_t>(), EPI_RESID);
        b = 2.0 * HID * FF + act_rw * (FF + 2 * HID);
        break;
      case 4:
        X.gemm(e->w.x.as<bf16_t>(), rows, HID, X.M.lm_head, V, X.M.final_norm, nullptr, 0, nullptr, EPI_LOGITS, &ex);
        b = 2.0 * V * HID + act_rw * HID + 2.0 * HID + rows * (V / 8.0);
        break;
      case 5:
        launch_attn_decode_step(aa, s);
        b = (double)rows * c.num_kv_heads * ctx * c.head_dim * 2 * 2 + act_rw * QKV;
        break;
      case 6:
      case 7: {  // QKV with the decode attention fused in (the one-row decode step's form), + o_proj (7)
        const AttnArgs al = X.attn_args(li, rows, e->w.row_slot.as<int>(), e->w.row_pos.as<int>(), true);
        const WgemmArgs fx = X.fused_attn_args(al, li, which == 7);
        X.gemm(e->w.x.as<bf16_t>(), rows, HID, ly.wqkv, QKV, ly.ln1, e->w.qkv.as<bf16_t>(), QKV, nullptr,
               EPI_STORE, &fx);
        b = 2.0 * QKV * HID + act_rw * (HID + QKV) + 2.0 * HID +
            (double)rows * c.num_kv_heads * ctx * c.head_dim * 2 * 2;
        if (which == 7) b += 2.0 * HID * HD + act_rw * (HD + 2 * HID);
        break;
      }
      case 8:    // the greedy head's int8 screen + exact recheck (lm_head_screen.hip)
      case 9: {  // the screen alone
        tts_gen_params gp{};
        gp.repetition_penalty = 1.1f;
        X.pending_norm = nullptr;
        X.screened_head_parts(e->w.x.as<bf16_t>(), rows, st, gp);
        if (which == 8) launch_bump_epoch(st.epoch, s);  // (the step counter finalize advances)
        // int8 matrix + per-column constants + rows + penalty bits (+ the recomputed units' bf16 tiles,
        // a few dozen of 64 KiB, not counted)
        b = (double)V * HID + 16.0 * V + act_rw * HID + rows * (V / 8.0);
        break;
      }
    }
  };
  launch();
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipEventRecord(e->ev[2], s));
  for (int i = 0; i < iters; ++i) launch();
  HIP_CHECK(hipEventRecord(e->ev[3], s));
  HIP_CHECK(hipEventSynchronize(e->ev[3]));
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, e->ev[2], e->ev[3]));
  *avg_ms = ms / iters;
  *bytes = b;
  check_fattn(e, s);
}

void lm_score(Engine* e, const int32_t* ids, const int32_t* lens, int B, int n_last,
              float* logits, hipStream_t s) {
  TTS_REQUIRE(e->lm.loaded, "tts_lm_load has not been called");
  TTS_REQUIRE(B >= 1 && B <= e->w.cap_batch, "batch out of range");
  Ctx X(e, s);
  const tts_lm_config& c = X.c;
  for (int b = 0; b < B; ++b) {
    TTS_REQUIRE(lens[b] >= n_last && lens[b] <= c.max_seq_len, "bad sequence length");
  }
  std::vector<int> last_rows;
  int rows = 0;
  prefill_rows_setup(X, ids, lens, B, 0, last_rows, rows);
  X.layers(rows, e->w.row_slot.as<int>(), e->w.row_pos.as<int>(), false);
  // gather the last n_last rows of every sequence
  std::vector<int> sel;
  for (int b = 0; b < B; ++b)
    for (int i = n_last - 1; i >= 0; --i) sel.push_back(last_rows[b] - i);
  const int nsel = (int)sel.size();
  DevBuf sel_d, xs, lg;
  sel_d.alloc(nsel * 4);
  xs.alloc((size_t)nsel * c.hidden_size * 2);
  lg.alloc((size_t)nsel * c.vocab_size * 2);
  HIP_CHECK(hipMemcpyAsync(sel_d.p, sel.data(), nsel * 4, hipMemcpyHostToDevice, s));
  launch_gather_rows(e->w.x.as<bf16_t>(), c.hidden_size, sel_d.as<int>(), xs.as<bf16_t>(), nsel,
                     c.hidden_size, s);
  // the lm_head in launches of <= kPrefillChunk rows: the decode GEMM's K order, which the
  // step's first token (B <= 64 gathered rows) also takes, so a sequence's logits do not depend
  // on how many sequences are scored with it (the prefill GEMM sums K in 1024-chunks)
  for (int r0 = 0; r0 < nsel; r0 += kPrefillChunk)
    X.gemm(xs.as<bf16_t>() + (size_t)r0 * c.hidden_size, std::min(kPrefillChunk, nsel - r0), c.hidden_size,
           X.M.lm_head, c.vocab_size, X.M.final_norm, lg.as<bf16_t>() + (size_t)r0 * c.vocab_size, c.vocab_size,
           nullptr, EPI_STORE);
  check_launch();
  std::vector<uint16_t> h((size_t)nsel * c.vocab_size);
  HIP_CHECK(hipMemcpyAsync(h.data(), lg.p, h.size() * 2, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  for (size_t i = 0; i < h.size(); ++i) {
    uint32_t u = (uint32_t)h[i] << 16;
    memcpy(&logits[i], &u, 4);
  }
}

// Teacher forcing through the DECODE step's kernels (the path generate runs after prefill):
// prefill the first lens[b] - n_last tokens of every sequence, then feed the remaining
// n_last tokens one decode step at a time (all rows together, the step's launch sequence:
// fused QKV+attention(+o_proj) at one row, the batched GEMVs and the (row, kv head) decode
// attention otherwise) and keep each step's bf16 logits.  Same positions as lm_score, so
// the two differ only by prefill vs decode arithmetic.  gidx (optional, [B][n_last][k]):
// keep only those vocabulary entries; otherwise k = V.
void lm_score_decode(Engine* e, const int32_t* ids, const int32_t* lens, int B, int n_last,
                     const int32_t* gidx, int k, float* out, hipStream_t s) {
  TTS_REQUIRE(e->lm.loaded, "tts_lm_load has not been called");
  TTS_REQUIRE(B >= 1 && B <= e->w.cap_batch, "batch out of range");
  Ctx X(e, s);
  const tts_lm_config& c = X.c;
  const int V = c.vocab_size, HID = c.hidden_size;
  if (!gidx) k = V;
  TTS_REQUIRE(k >= 1 && k <= V, "bad gather width");
  std::vector<int> start(B), plen(B);
  for (int b = 0, off = 0; b < B; off += lens[b], ++b) {
    TTS_REQUIRE(lens[b] > n_last && lens[b] <= c.max_seq_len, "bad sequence length (needs lens > n_last)");
    start[b] = off;
    plen[b] = lens[b] - n_last;
  }
  if (gidx)
    for (size_t i = 0; i < (size_t)B * n_last * k; ++i) TTS_REQUIRE(gidx[i] >= 0 && gidx[i] < V, "gather index out of range");
  // ---- prefill the prefixes (groups of whole prefixes that fit the workspace)
  {
    std::vector<int> last_rows;
    int b0 = 0;
    while (b0 < B) {
      int b1 = b0, grp = 0;
      std::vector<int32_t> pid;
      while (b1 < B && grp + plen[b1] <= e->w.cap_rows) {
        pid.insert(pid.end(), ids + start[b1], ids + start[b1] + plen[b1]);
        grp += plen[b1++];
      }
      TTS_REQUIRE(b1 > b0, "a prefix is longer than the prefill workspace");
      int rows = 0;
      prefill_rows_setup(X, pid.data(), plen.data() + b0, b1 - b0, b0, last_rows, rows);
      X.layers(rows, e->w.row_slot.as<int>(), e->w.row_pos.as<int>(), false);
      b0 = b1;
    }
  }
  // ---- n_last decode steps with the given tokens
  std::vector<int> ident(B), tok(B), pos(B);
  for (int b = 0; b < B; ++b) ident[b] = b;
  DevBuf lg;
  lg.alloc((size_t)B * V * 2);
  std::vector<uint16_t> h((size_t)B * V);
  HIP_CHECK(hipMemcpyAsync(e->w.row_slot.p, ident.data(), B * 4, hipMemcpyHostToDevice, s));
  for (int i = 0; i < n_last; ++i) {
    for (int b = 0; b < B; ++b) {
      tok[b] = ids[start[b] + plen[b] + i];
      pos[b] = plen[b] + i;
    }
    HIP_CHECK(hipMemcpyAsync(e->w.row_idx.p, tok.data(), B * 4, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(e->w.row_pos.p, pos.data(), B * 4, hipMemcpyHostToDevice, s));
    launch_embed(e->w.row_idx.as<int>(), X.M.embed_rows.as<bf16_t>(), e->w.x.as<bf16_t>(), B, HID, s);
    X.layers(B, e->w.row_slot.as<int>(), e->w.row_pos.as<int>(), true);
    X.gemm(e->w.x.as<bf16_t>(), B, HID, X.M.lm_head, V, X.M.final_norm, lg.as<bf16_t>(), V, nullptr, EPI_STORE);
    launch_bump_epoch(e->w.epoch.as<uint32_t>(), s);  // (a decode step without the finalize kernel)
    check_launch();
    HIP_CHECK(hipMemcpyAsync(h.data(), lg.p, h.size() * 2, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));  // (h and the token/position vectors are reused)
    for (int b = 0; b < B; ++b) {
      float* o = out + ((size_t)b * n_last + i) * k;
      const uint16_t* hb = h.data() + (size_t)b * V;
      const int32_t* gi = gidx ? gidx + ((size_t)b * n_last + i) * k : nullptr;
      for (int j = 0; j < k; ++j) {
        const uint32_t u = (uint32_t)hb[gi ? gi[j] : j] << 16;
        memcpy(&o[j], &u, 4);
      }
    }
  }
  check_fattn(e, s);
}

// The launch list of one decode step over `rows` rows of a model of config c on num_cu CUs,
// without a GPU: the step's own code (Ctx::layers + head_and_pick) run with the launchers in
// dry-run mode (lm_kernels.h dry_launches), nothing allocated.  Unique launches in first-seen
// order, one per line (wgemm instantiations as wgemm_inst_name writes them).
std::string lm_step_plan(const tts_lm_config& c, int rows, int num_cu) {
  TTS_REQUIRE(c.head_dim == 64 || c.head_dim == 128, "head_dim must be 64 or 128");
  TTS_REQUIRE(c.num_heads == 4 * c.num_kv_heads && c.num_layers >= 1, "bad config");
  TTS_REQUIRE(rows >= 1 && rows <= 64 && num_cu >= 1, "rows in [1, 64], num_cu >= 1");
  Engine e;  // (no HIP call: no stream, no buffer)
  e.num_cu = num_cu;
  e.lm.cfg = c;
  e.lm.cfg.max_batch = std::max(c.max_batch, rows);
  // distinct placeholder addresses for the weights (the step code compares norm-weight pointers
  // to choose its RMSNorm form; nothing is dereferenced in a dry run)
  uintptr_t fake = 0x10000;
  auto next = [&] { fake += 0x100; return (bf16_t*)fake; };
  e.lm.layers.resize(c.num_layers);
  for (LmLayer& ly : e.lm.layers) {
    ly.ln1 = next(); ly.ln2 = next(); ly.wqkv = next(); ly.wo = next(); ly.wgu = next(); ly.wd = next();
  }
  e.lm.final_norm = next();
  e.lm.lm_head = next();
  {
    const StreamPlan hp = stream_plan(c.vocab_size, c.hidden_size, 1, num_cu);
    if (head_screen_enabled() && head_screen_supported(1, c.hidden_size, c.vocab_size) && hp.ng == 1 && hp.ksplit == 1)
      e.lm.head_grid = num_cu;
  }
  e.w.cap_batch = e.lm.cfg.max_batch;
  e.w.kpart.bytes = kpart_bytes(c);  // (the size the plan checks; never dereferenced)
  std::vector<std::string> rec;
  dry_launches() = &rec;
  try {
    Ctx X(&e, nullptr);
    X.layers(rows, nullptr, nullptr, true);
    const StepState st = X.state(rows, 0, 0);
    tts_gen_params gp{};
    gp.repetition_penalty = 1.1f;
    X.head_and_pick(nullptr, rows, st, gp);
  } catch (...) {
    dry_launches() = nullptr;
    e.w.kpart.bytes = 0;
    throw;
  }
  dry_launches() = nullptr;
  e.w.kpart.bytes = 0;
  std::string out;
  std::vector<std::string> seen;
  for (const std::string& r : rec)
    if (std::find(seen.begin(), seen.end(), r) == seen.end()) {
      seen.push_back(r);
      out += r + "\n";
    }
  return out;
}

}  // namespace tts
