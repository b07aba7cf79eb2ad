// engine.h — the engine object behind the C ABI (one GPU, one stream, owned buffers).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/tts_mi355x.h"
#include "lm_kernels.h"

namespace tts {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIP_CHECK(expr)                                                                    \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      throw ::tts::Error(TTS_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e) +    \
                                        " (" + __FILE__ + ":" + std::to_string(__LINE__) + ")"); \
  } while (0)
#define TTS_REQUIRE(cond, msg)                                    \
  do {                                                            \
    if (!(cond)) throw ::tts::Error(TTS_E_INVALID, std::string(msg)); \
  } while (0)

// Device allocation owned by the engine.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void alloc(size_t n) {
    release();
    if (n == 0) n = 16;
    if (hipMalloc(&p, n) != hipSuccess) {
      p = nullptr;
      throw Error(TTS_E_OOM, "hipMalloc failed for " + std::to_string(n) + " bytes");
    }
    bytes = n;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T> T* as() const { return (T*)p; }
  ~DevBuf() { release(); }
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
};

struct LmLayer {
  bf16_t* ln1;   // [hidden]
  bf16_t* ln2;
  bf16_t* wqkv;  // tiled [(H+2KVH)*D][hidden]
  bf16_t* wo;    // tiled [hidden][H*D]
  bf16_t* wgu;   // tiled, gate/up n-tiles interleaved [2*ffn][hidden]
  bf16_t* wd;    // tiled [hidden][ffn]
};

struct LmModel {
  tts_lm_config cfg{};
  bool loaded = false;
  DevBuf weights;       // one slab for every tiled matrix + norms
  DevBuf embed_rows;    // row-major embedding [V][hidden] (token gather)
  DevBuf rope;          // cos | sin  [max_seq][D] bf16 each
  std::vector<LmLayer> layers;
  bf16_t* final_norm = nullptr;
  bf16_t* lm_head = nullptr;  // tiled [V][hidden]
  // the greedy lm_head's int8 screen (lm_head_screen.hip): codes in the screen's block layout,
  // per-column {scale, |W - Wh|, |W|, |Wh|}; head_grid = the screen's launch grid (0: none)
  DevBuf head_q, head_c;
  int head_grid = 0;
  std::vector<int> id_to_code;  // host LUT (optional)
  int qkv_n() const { return (cfg.num_heads + 2 * cfg.num_kv_heads) * cfg.head_dim; }
};

struct LmWork {
  int cap_rows = 0;    // activation rows (prefill rows and decode batch)
  int cap_batch = 0;
  int cap_seq = 0;
  DevBuf kv;           // per layer: K [slots][KVH][kv_stride][D], V^T [slots][KVH][D][kv_stride]
  int kv_stride = 0;   // positions per (slot, kv head) strip: max_seq_len rounded up to 64
  DevBuf x, xn, qkv, attn_out, act, q_rot, last_x;  // activations
  DevBuf blocks;                                    // prefill query blocks (int4, lm_attn.hip)
  int nblocks = 0;
  DevBuf gran, ferr;                                // fused QKV+attention: granules [QKV/2] u64, error flag
  DevBuf xgran;                                     // norm-once hand-off: hidden-row granules [2][B][hidden/2] u64
  DevBuf epoch;                                     // decode-step counter (u32; the hand-off's tags)
  DevBuf lpart_v, lpart_i;                          // lm_head argmax partials
  DevBuf hub, hlb;                                  // screened head: check-mode score bounds [B][V], per-row max lower bound (u64)
  DevBuf hxq, hxs;                                  // screened head at 17..32 rows: the rows quantised [2B][hidden] i8, their stats
  DevBuf kpart;                                     // K-sliced GEMM fp32 partials [kc][rows][N]
  DevBuf ppart;                                     // prefill GEMM fp32 partials [chunks][rows][N] (lm_pgemm.hip)
  DevBuf slogits;                                   // sampling: processed fp32 logits [B][V]
  DevBuf counts;                                    // vLLM frequency penalty: new-token counts [B][V] u16
  DevBuf logits;                                    // scoring output (bf16)
  DevBuf row_slot, row_pos, row_idx;                // prefill row descriptors
  DevBuf st_int;                                    // step-state ints
  DevBuf row_seed;                                  // [B] u64 sampling key of each row (graph-invariant)
  DevBuf seen;                                      // [B][V/32]
  DevBuf out_ids;                                   // [B][max_new]
  int out_cap = 0;
  hipGraphExec_t graph = nullptr;
  int graph_batch = -1;  // the captured step bakes in B, penalty, eos and min_new
  float graph_pen = -1.f;
  int graph_eos = -2, graph_min_new = -1;
  // sampling parameters baked into the captured step (kernel arguments)
  int graph_sample = -1, graph_top_k = -1;
  float graph_temp = -1.f, graph_top_p = -1.f;
  float graph_freq = 0.f;
  int* h_active = nullptr;  // pinned host copy of n_active (ring of 2)
};

struct Codec;         // codec_engine.cpp
struct AudioEncoder;  // codec_encoder.cpp

struct Engine {
  int device = 0;
  int num_cu = 256;
  hipStream_t stream = nullptr;
  hipEvent_t ev[4] = {};
  LmModel lm;
  LmWork w;
  Codec* codec = nullptr;
  AudioEncoder* encoder = nullptr;
  float t_prefill_ms = 0.f, t_decode_ms = 0.f;
  int decode_steps = 0;
  // an open generation (tts_generate_begin .. tts_generate_read): state lives on the device
  struct Gen {
    bool open = false;
    int B = 0, max_new = 0, launched = 0, polls = 0;
    bool finished = false;
    hipStream_t s = nullptr;
  } gen;
  // continuous batching (tts_slots_*): S persistent rows, sequences admitted / retired
  // between decode chunks
  struct Slots {
    bool open = false;
    int S = 0;
    tts_gen_params gp{};
    unsigned long long next_req = 0;  // default per-request sampling keys
    std::vector<int> busy;  // 1 while a sequence owns the slot (until released)
    hipStream_t s = nullptr;
  } slots;
  ~Engine();
};

hipStream_t pick_stream(Engine* e, void* s);
void lm_load(Engine* e, const tts_lm_config* cfg, const tts_tensor_desc* t, int n);
void lm_generate(Engine* e, const tts_gen_params* p, const int32_t* ids, const int32_t* lens,
                 int B, int32_t* out_ids, int out_stride, int32_t* out_lens, hipStream_t s);
// the same loop in pieces (streaming): begin = prefill + first token; continue = up to
// n_steps more decode steps (returns 1 when every row has stopped); read = ids so far
void lm_gen_begin(Engine* e, const tts_gen_params* p, const int32_t* ids, const int32_t* lens, int B,
                  hipStream_t s);
int lm_gen_continue(Engine* e, int n_steps);
void lm_gen_read(Engine* e, int32_t* out_ids, int out_stride, int32_t* out_lens);
void lm_slots_open(Engine* e, const tts_gen_params* p, int S, hipStream_t s);
void lm_slots_add(Engine* e, int slot, const int32_t* prompt, int len, int max_new, const uint64_t* seed);
int lm_slots_step(Engine* e, int n_steps);
void lm_slots_read(Engine* e, int slot, int32_t* out_ids, int cap, int32_t* n_out, int32_t* finished);
void lm_slots_release(Engine* e, int slot);
void lm_score(Engine* e, const int32_t* ids, const int32_t* lens, int B, int n_last,
              float* logits, hipStream_t s);
void lm_score_decode(Engine* e, const int32_t* ids, const int32_t* lens, int B, int n_last,
                     const int32_t* gidx, int k, float* out, hipStream_t s);
void lm_bench_kernel(Engine* e, int which, int rows, int ctx, int iters, float* avg_ms,
                     double* bytes);
std::string lm_step_plan(const tts_lm_config& c, int rows, int num_cu);

// upload a named tensor to device memory as bf16 (convert from f32 if needed)
void upload_bf16(const tts_tensor_desc& d, bf16_t* dst, hipStream_t s, DevBuf& staging);
void upload_f32(const tts_tensor_desc& d, float* dst, hipStream_t s, DevBuf& staging);
int64_t numel(const tts_tensor_desc& d);

void codec_load(Engine* e, const tts_codec_config* cfg, const tts_tensor_desc* t, int n);
void codec_decode(Engine* e, const int32_t* codes, const int32_t* lens, int B, float* wav,
                  int wav_is_device, int64_t* wav_lens, hipStream_t s);
int codec_samples_per_code(Engine* e);
// the prompt-audio encoder (codec_encoder.cpp)
void encoder_load(Engine* e, const tts_tensor_desc* t, int n);
int encoder_encode(Engine* e, const float* wav, int n, const float* w2v, int T_w2v, int32_t* codes, int cap,
                   float* pre, const float* feats = nullptr);
void encoder_destroy(AudioEncoder* a);
void codec_destroy(Codec* c);

}  // namespace tts
