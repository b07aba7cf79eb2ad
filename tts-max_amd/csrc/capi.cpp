// capi.cpp — the extern "C" boundary (include/tts_mi355x.h, include/tts_mi355x_ops.h).
// Every entry point catches everything: errors become a status code plus a thread-local
// message, never an exception across the ABI.
#include <stdlib.h>
#include <string.h>

#include <memory>
#include <string>

#include "../../include/tts_mi355x.h"
#include "../../include/tts_mi355x_ops.h"
#include "codec_kernels.h"
#include "engine.h"

namespace tts {

static thread_local std::string g_last_error;

template <class F>
static tts_status guarded(F&& f) {
  try {
    f();
    return TTS_OK;
  } catch (const Error& e) {
    g_last_error = e.what();
    return e.code;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return TTS_E_INVALID;
  } catch (...) {
    g_last_error = "unknown error";
    return TTS_E_INVALID;
  }
}

hipStream_t pick_stream(Engine* e, void* s) { return s ? (hipStream_t)s : e->stream; }

Engine::~Engine() {
  if (w.graph) (void)hipGraphExecDestroy(w.graph);
  if (w.h_active) (void)hipHostFree(w.h_active);
  if (codec) codec_destroy(codec);
  if (encoder) encoder_destroy(encoder);
  for (auto& v : ev)
    if (v) (void)hipEventDestroy(v);
  if (stream) (void)hipStreamDestroy(stream);
}

}  // namespace tts

using namespace tts;

extern "C" {

int32_t tts_abi_version(void) { return TTS_ABI_VERSION; }

const char* tts_last_error(void) { return g_last_error.c_str(); }

tts_status tts_engine_create(int32_t device, tts_engine** out) {
  return guarded([&] {
    TTS_REQUIRE(out != nullptr, "null output pointer");
    int n = 0;
    HIP_CHECK(hipGetDeviceCount(&n));
    TTS_REQUIRE(device >= 0 && device < n, "device index out of range");
    HIP_CHECK(hipSetDevice(device));
    std::unique_ptr<Engine> e(new Engine());  // freed if a HIP call below throws
    e->device = device;
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, device));
    e->num_cu = prop.multiProcessorCount;
    HIP_CHECK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    for (auto& v : e->ev) HIP_CHECK(hipEventCreate(&v));
    *out = reinterpret_cast<tts_engine*>(e.release());
  });
}

void tts_engine_destroy(tts_engine* e) {
  if (!e) return;
  Engine* E = reinterpret_cast<Engine*>(e);
  (void)hipSetDevice(E->device);
  (void)hipDeviceSynchronize();
  delete E;
}

tts_status tts_lm_load(tts_engine* e, const tts_lm_config* cfg, const tts_tensor_desc* t,
                       int32_t n) {
  return guarded([&] {
    TTS_REQUIRE(e && t && n > 0, "null argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    lm_load(E, cfg, t, n);
  });
}

tts_status tts_generate(tts_engine* e, const tts_gen_params* p, const int32_t* prompt_ids,
                        const int32_t* prompt_lens, int32_t batch, int32_t* out_ids,
                        int32_t out_stride, int32_t* out_lens, void* stream) {
  return guarded([&] {
    TTS_REQUIRE(e && p && prompt_ids && prompt_lens && out_ids && out_lens, "null argument");
    TTS_REQUIRE(batch >= 1, "batch must be >= 1");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    lm_generate(E, p, prompt_ids, prompt_lens, batch, out_ids, out_stride, out_lens,
                pick_stream(E, stream));
  });
}

tts_status tts_generate_begin(tts_engine* e, const tts_gen_params* p, const int32_t* prompt_ids,
                              const int32_t* prompt_lens, int32_t batch, void* stream) {
  return guarded([&] {
    TTS_REQUIRE(e && p && prompt_ids && prompt_lens, "null argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    lm_gen_begin(E, p, prompt_ids, prompt_lens, batch, pick_stream(E, stream));
  });
}

tts_status tts_generate_continue(tts_engine* e, int32_t n_steps, int32_t* all_done) {
  return guarded([&] {
    TTS_REQUIRE(e && all_done && n_steps >= 0, "bad argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    *all_done = lm_gen_continue(E, n_steps);
  });
}

tts_status tts_generate_read(tts_engine* e, int32_t* out_ids, int32_t out_stride, int32_t* out_lens) {
  return guarded([&] {
    TTS_REQUIRE(e && out_ids && out_lens, "null argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    lm_gen_read(E, out_ids, out_stride, out_lens);
  });
}

tts_status tts_slots_open(tts_engine* e, const tts_gen_params* p, int32_t n_slots, void* stream) {
  return guarded([&] {
    TTS_REQUIRE(e && p, "null argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    lm_slots_open(E, p, n_slots, pick_stream(E, stream));
  });
}

tts_status tts_slots_add(tts_engine* e, int32_t slot, const int32_t* prompt_ids, int32_t prompt_len,
                         int32_t max_new_tokens) {
  return guarded([&] {
    TTS_REQUIRE(e && prompt_ids, "null argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    lm_slots_add(E, slot, prompt_ids, prompt_len, max_new_tokens, nullptr);
  });
}

tts_status tts_slots_add_seeded(tts_engine* e, int32_t slot, const int32_t* prompt_ids, int32_t prompt_len,
                         int32_t max_new_tokens, uint64_t seed) {
  return guarded([&] {
    TTS_REQUIRE(e && prompt_ids, "null argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    lm_slots_add(E, slot, prompt_ids, prompt_len, max_new_tokens, &seed);
  });
}

tts_status tts_slots_step(tts_engine* e, int32_t n_steps, int32_t* n_active) {
  return guarded([&] {
    TTS_REQUIRE(e && n_active && n_steps >= 0, "bad argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    *n_active = lm_slots_step(E, n_steps);
  });
}

tts_status tts_slots_read(tts_engine* e, int32_t slot, int32_t* out_ids, int32_t capacity, int32_t* n_out,
                          int32_t* finished) {
  return guarded([&] {
    TTS_REQUIRE(e && out_ids && n_out && finished, "null argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    lm_slots_read(E, slot, out_ids, capacity, n_out, finished);
  });
}

tts_status tts_slots_release(tts_engine* e, int32_t slot) {
  return guarded([&] {
    TTS_REQUIRE(e, "null argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    lm_slots_release(E, slot);
  });
}

tts_status tts_lm_score(tts_engine* e, const int32_t* ids, const int32_t* lens, int32_t batch,
                        int32_t n_last, float* logits, void* stream) {
  return guarded([&] {
    TTS_REQUIRE(e && ids && lens && logits && n_last >= 1, "bad argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    lm_score(E, ids, lens, batch, n_last, logits, pick_stream(E, stream));
  });
}

tts_status tts_lm_score_decode(tts_engine* e, const int32_t* ids, const int32_t* lens, int32_t batch,
                               int32_t n_last, const int32_t* gather_idx, int32_t k, float* logits,
                               void* stream) {
  return guarded([&] {
    TTS_REQUIRE(e && ids && lens && logits && n_last >= 1, "bad argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    lm_score_decode(E, ids, lens, batch, n_last, gather_idx, k, logits, pick_stream(E, stream));
  });
}

tts_status tts_lm_id_to_code(tts_engine* e, const int32_t* ids, int32_t n, int32_t* codes) {
  return guarded([&] {
    TTS_REQUIRE(e && ids && codes && n >= 0, "bad argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    TTS_REQUIRE(!E->lm.id_to_code.empty(), "no vocab.id_to_code LUT was loaded");
    const int V = (int)E->lm.id_to_code.size();
    for (int i = 0; i < n; ++i) codes[i] = (ids[i] >= 0 && ids[i] < V) ? E->lm.id_to_code[ids[i]] : -1;
  });
}

tts_status tts_lm_last_timing(tts_engine* e, float* prefill_ms, float* decode_ms,
                              int32_t* decode_steps) {
  return guarded([&] {
    TTS_REQUIRE(e, "null engine");
    Engine* E = reinterpret_cast<Engine*>(e);
    if (prefill_ms) *prefill_ms = E->t_prefill_ms;
    if (decode_ms) *decode_ms = E->t_decode_ms;
    if (decode_steps) *decode_steps = E->decode_steps;
  });
}

tts_status tts_lm_bench_kernel(tts_engine* e, int32_t which, int32_t rows, int32_t ctx,
                               int32_t iters, float* avg_ms, double* bytes) {
  return guarded([&] {
    TTS_REQUIRE(e && avg_ms && bytes, "null argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    lm_bench_kernel(E, which, rows, ctx, iters, avg_ms, bytes);
  });
}

tts_status tts_debug_step_plan(const tts_lm_config* cfg, int32_t rows, int32_t num_cu, char* out, int32_t cap) {
  return guarded([&] {
    TTS_REQUIRE(cfg && out && cap > 0, "null argument");
    const std::string p = lm_step_plan(*cfg, rows, num_cu);
    TTS_REQUIRE((int64_t)p.size() < cap, "output buffer too small");
    memcpy(out, p.c_str(), p.size() + 1);
  });
}

tts_status tts_codec_load(tts_engine* e, const tts_codec_config* cfg, const tts_tensor_desc* t,
                          int32_t n) {
  return guarded([&] {
    TTS_REQUIRE(e && cfg && t && n > 0, "null argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    codec_load(E, cfg, t, n);
  });
}

tts_status tts_codec_decode(tts_engine* e, const int32_t* codes, const int32_t* lens,
                            int32_t batch, float* wav, int32_t wav_is_device, int64_t* wav_lens,
                            void* stream) {
  return guarded([&] {
    TTS_REQUIRE(e && codes && lens && wav && wav_lens && batch >= 1, "bad argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    codec_decode(E, codes, lens, batch, wav, wav_is_device, wav_lens, pick_stream(E, stream));
  });
}

tts_status tts_encoder_load(tts_engine* e, const tts_tensor_desc* t, int32_t n) {
  return guarded([&] {
    TTS_REQUIRE(e && t && n > 0, "null argument");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    encoder_load(E, t, n);
  });
}

tts_status tts_encoder_encode(tts_engine* e, const float* wav, int64_t n_samples, const float* w2v_features,
                              int32_t n_frames, int32_t* codes, int32_t codes_cap, int32_t* n_codes,
                              float* pre_round) {
  return guarded([&] {
    TTS_REQUIRE(e && wav && w2v_features && codes && n_codes, "null argument");
    TTS_REQUIRE(n_samples >= 1 && n_samples < (1ll << 31) - 640, "bad waveform length");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    *n_codes = encoder_encode(E, wav, (int)n_samples, w2v_features, n_frames, codes, codes_cap, pre_round);
  });
}

tts_status tts_encoder_encode_features(tts_engine* e, const float* wav, int64_t n_samples, const float* features,
                                       int32_t n_frames, int32_t* codes, int32_t codes_cap, int32_t* n_codes,
                                       float* pre_round) {
  return guarded([&] {
    TTS_REQUIRE(e && wav && features && codes && n_codes, "null argument");
    TTS_REQUIRE(n_samples >= 1 && n_samples < (1ll << 31) - 640, "bad waveform length");
    Engine* E = reinterpret_cast<Engine*>(e);
    HIP_CHECK(hipSetDevice(E->device));
    *n_codes = encoder_encode(E, wav, (int)n_samples, nullptr, n_frames, codes, codes_cap, pre_round, features);
  });
}

tts_status tts_codec_samples_per_code(tts_engine* e, int32_t* out) {
  return guarded([&] {
    TTS_REQUIRE(e && out, "null argument");
    *out = codec_samples_per_code(reinterpret_cast<Engine*>(e));
  });
}

// ------------------------------------------------------------------------ op level ----

tts_status tts_synth_fill(void* dst, int32_t dtype, int64_t n, uint64_t seed, float scale,
                          void* stream) {
  return guarded([&] {
    TTS_REQUIRE(dst && n >= 0 && (dtype == TTS_DT_F32 || dtype == TTS_DT_BF16), "bad argument");
    launch_synth_fill(dst, dtype == TTS_DT_F32 ? 0 : 1, n, seed, scale, (hipStream_t)stream);
    HIP_CHECK(hipGetLastError());
  });
}

static int device_cu_count() {  // (single-device process: cached, no per-call query)
  static int num_cu = 0;
  if (!num_cu) {
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&num_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  return num_cu;
}

tts_status tts_op_retile(const void* w, void* w_tiled, int32_t N, int32_t K, int32_t epi, void* stream) {
  return guarded([&] {
    TTS_REQUIRE(w && w_tiled && N % (epi == EPI_SWIGLU ? 32 : 16) == 0 && K % 256 == 0, "bad argument");
    const int ncu = device_cu_count();
    if (epi == EPI_SWIGLU) {  // rows [0, N/2) = gate, [N/2, N) = up: n-tiles interleaved
      const bf16_t* wg = (const bf16_t*)w;
      launch_retile(wg, (bf16_t*)w_tiled, N / 2, K, N, 2, ncu, (hipStream_t)stream, 2, 0);
      launch_retile(wg + (size_t)(N / 2) * K, (bf16_t*)w_tiled, N / 2, K, N, 2, ncu, (hipStream_t)stream, 2, 1);
    } else {
      launch_retile((const bf16_t*)w, (bf16_t*)w_tiled, N, K, N, 1, ncu, (hipStream_t)stream, 1, 0);
    }
    HIP_CHECK(hipGetLastError());
  });
}

tts_status tts_op_wgemm(const void* x, int32_t M, int32_t K, int32_t ldx, const void* w_tiled,
                        int32_t N, const void* normw, float eps, void* out, int32_t ldo,
                        void* resid, int32_t epi, void* stream) {
  return guarded([&] {
    TTS_REQUIRE(epi == EPI_STORE || epi == EPI_RESID || epi == EPI_SWIGLU, "bad epilogue");
    TTS_REQUIRE(wgemm_supported(M, N, K, epi), "unsupported GEMM shape");
    TTS_REQUIRE(ldx == K, "ldx must equal K");
    WgemmPlan p = plan_wgemm(M, N, K, epi, device_cu_count());
    hipStream_t st = (hipStream_t)stream;
    WgemmArgs a;
    a.x = (const bf16_t*)x; a.M = M; a.K = K; a.ldx = ldx;
    a.w = (const bf16_t*)w_tiled; a.N = N;
    a.normw = (const bf16_t*)normw; a.eps = eps;
    a.out = (bf16_t*)out; a.ldo = ldo; a.resid = (bf16_t*)resid;
    // RMSNorm in the GEMM's prologue where the rows fit it (LDS rows, K <= 4096, the LDS-DMA
    // pieces of 512 columns); otherwise a standalone pass first — the same canonical sum order
    // (chunk_sumsq), so the same bits either way, as the engine does (lm_engine.cpp gemm)
    bf16_t* xn = nullptr;
    if (normw && !(p.a_lds && !p.sliced && K <= 4096 && K % 512 == 0)) {
      HIP_CHECK(hipMallocAsync((void**)&xn, (size_t)M * K * 2, st));
      launch_rmsnorm(a.x, ldx, a.normw, eps, xn, K, M, K, st);
      a.x = xn;
      a.normw = nullptr;
    }
    float* part = nullptr;
    if (p.sliced) {
      HIP_CHECK(hipMallocAsync((void**)&part, wgemm_part_elems(p, M, ldo) * 4, st));
      a.part_out = part;
    }
    launch_wgemm(a, p, epi, a.normw != nullptr, st);
    HIP_CHECK(hipGetLastError());
    if (part) HIP_CHECK(hipFreeAsync(part, st));
    if (xn) HIP_CHECK(hipFreeAsync(xn, st));
  });
}

tts_status tts_op_pgemm(const void* x, int32_t M, int32_t K, const void* w_tiled, int32_t N, void* out,
                        int32_t ldo, void* resid, int32_t epi, void* stream) {
  return guarded([&] {
    TTS_REQUIRE(pgemm_supported(M, N, K, epi), "unsupported prefill GEMM shape / epilogue");
    TTS_REQUIRE(epi == EPI_RESID ? resid != nullptr : out != nullptr, "missing output");
    PgemmArgs a;
    a.x = (const bf16_t*)x; a.M = M; a.K = K; a.ldx = K;
    a.w = (const bf16_t*)w_tiled; a.N = N;
    a.out = (bf16_t*)out; a.ldo = ldo; a.resid = (bf16_t*)resid;
    // the engine's scratch for the one-chunk-per-workgroup form (prompts of <= 256 rows,
    // lm_engine.cpp kPgemmSplitRows): a stream-ordered allocation of this call's size
    hipStream_t s = (hipStream_t)stream;
    if (M <= 256) {
      a.part_bytes = pgemm_part_bytes(M, N, K);
      HIP_CHECK(hipMallocAsync((void**)&a.part, a.part_bytes, s));
    }
    launch_pgemm(a, epi, device_cu_count(), s);
    HIP_CHECK(hipGetLastError());
    if (a.part) HIP_CHECK(hipFreeAsync(a.part, s));
  });
}

tts_status tts_op_sample(const float* logits, int32_t B, int32_t V, float temperature, int32_t top_k,
                         float top_p, uint64_t seed, int32_t step, const float* part_max, int32_t nparts,
                         float* probs, int32_t* tokens, void* stream) {
  return guarded([&] {
    TTS_REQUIRE(logits && tokens && B >= 1 && V >= 1, "bad arguments");
    TTS_REQUIRE(temperature > 0.f && top_k >= 1 && top_k <= SAMPLE_MAX_TOP_K && top_p > 0.f && top_p <= 1.f,
                "temperature > 0, top_k in [1, 1024], top_p in (0, 1]");
    SampleArgs a;
    a.logits = logits; a.ldl = V; a.V = V;
    a.temperature = temperature; a.top_k = top_k; a.top_p = top_p; a.seed = seed; a.step0 = step;
    a.part_val = part_max; a.nparts = part_max ? nparts : 0; a.part_stride = nparts;
    a.probs = probs; a.tokens = tokens;
    launch_sample(a, B, (hipStream_t)stream);
    HIP_CHECK(hipGetLastError());
  });
}

tts_status tts_op_rmsnorm(const void* x, const void* w, float eps, void* y, int32_t M, int32_t K,
                          void* stream) {
  return guarded([&] {
    TTS_REQUIRE(x && w && y && K % 8 == 0, "bad argument");
    launch_rmsnorm((const bf16_t*)x, K, (const bf16_t*)w, eps, (bf16_t*)y, K, M, K,
                   (hipStream_t)stream);
    HIP_CHECK(hipGetLastError());
  });
}

tts_status tts_op_gemm_f32(const float* A, int32_t M, int32_t K, int32_t lda, const float* B,
                           int32_t N, const float* bias, float* C, int32_t ldc,
                           const float* resid, int32_t act, void* stream) {
  return guarded([&] {
    TTS_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0, "bad argument");
    GemmF32Args g;
    g.A = A; g.M = M; g.K = K; g.lda = lda; g.B = B; g.N = N; g.bias = bias;
    g.C = C; g.ldc = ldc; g.resid = resid; g.act = act;
    launch_gemm_f32(g, (hipStream_t)stream);
    HIP_CHECK(hipGetLastError());
  });
}

}  // extern "C"
