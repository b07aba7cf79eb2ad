/*
 * tts_mi355x.h — C ABI of the MI355X-native SpeechLM-TTS inference engine.
 *
 * This is the drop-in boundary for the `tts.inference` hot path of the reference
 * (ishine/tts-max).  The reference has no native code: its hot path is Python calling
 * third-party CUDA kernels.  Each entry point below replaces one reference interface:
 *
 *   tts_generate        replaces  model.generate(input_ids, max_length, min_new_tokens,
 *                                  eos_token_id, do_sample, repetition_penalty, top_p,
 *                                  temperature)     — tts/inference/inferencing.py:94-107
 *                                  (HF GenerationMixin._sample, transformers generation/utils.py)
 *   tts_lm_load         replaces  AutoModelForCausalLM.from_pretrained(dir, torch_dtype=...)
 *                                  — tools/serving/inference.py:103-107 (weights come in as
 *                                  host tensors named by their HF state-dict key)
 *   tts_codec_load      replaces  decoder.Decoder(...).load_from_checkpoint
 *                                  — tts/core/codec/decoder.py:17-67, 91-119
 *   tts_codec_decode    replaces  AudioDecoder.decode(speech_ids) -> Decoder.forward
 *                                  — tts/core/codec/decoding.py:84-89, decoder.py:69-89
 *
 * Conventions
 *   - Every function returns tts_status (0 = TTS_OK).  On error the message is available
 *     from tts_last_error() (thread-local).  No C++ exception crosses this boundary.
 *   - Plain pointers and sizes only.  `stream` is a hipStream_t passed as void* (NULL =
 *     the engine's own stream).  Pointers documented "device" must be device memory of the
 *     engine's GPU; "host" pointers are ordinary CPU memory.
 *   - One engine = one GPU.  An engine is not re-entrant: use one engine per thread/GPU.
 *   - The engine owns weights, KV cache, workspaces and captured hipGraphs; the caller owns
 *     every buffer it passes in.
 */
#ifndef TTS_MI355X_H
#define TTS_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TTS_ABI_VERSION 4

typedef int32_t tts_status;
enum {
  TTS_OK = 0,
  TTS_E_INVALID = 1,     /* bad argument / shape / missing tensor              */
  TTS_E_HIP = 2,         /* HIP runtime error                                  */
  TTS_E_OOM = 3,         /* device allocation failed                           */
  TTS_E_STATE = 4,       /* call order violated (e.g. generate before load)    */
  TTS_E_UNSUPPORTED = 5  /* configuration not implemented                      */
};

enum { TTS_DT_F32 = 0, TTS_DT_BF16 = 1, TTS_DT_F16 = 2, TTS_DT_I32 = 3, TTS_DT_I64 = 4 };

typedef struct tts_engine tts_engine;

/* One named host tensor (row-major, contiguous).  Names are the reference state-dict keys:
 * HF Llama keys for the SpeechLM ("model.layers.3.mlp.up_proj.weight", ...) and the codec
 * Decoder keys ("decoder.backbone.embed.weight", "fc_post_a.bias", ...). */
typedef struct {
  const char* name;
  const void* data;
  int32_t dtype;
  int32_t ndim;
  int64_t shape[4];
  int32_t on_device; /* 0: `data` is host memory; 1: device memory of the engine's GPU */
} tts_tensor_desc;

/* ---------------------------------------------------------------- engine lifecycle --- */

int32_t tts_abi_version(void);
const char* tts_last_error(void);
tts_status tts_engine_create(int32_t device, tts_engine** out);
void tts_engine_destroy(tts_engine* e);

/* ------------------------------------------------------------------------- SpeechLM --- */

/* LlamaForCausalLM architecture (transformers models/llama/configuration_llama.py). */
typedef struct {
  int32_t hidden_size;         /* 2048 (TTS-1) / 4096 (TTS-1-Max)                    */
  int32_t num_layers;          /* 16 / 32                                            */
  int32_t num_heads;           /* 32                                                 */
  int32_t num_kv_heads;        /* 8                                                  */
  int32_t head_dim;            /* 64 / 128                                           */
  int32_t intermediate_size;   /* 8192 / 14336                                       */
  int32_t vocab_size;          /* 193856                                             */
  int32_t tie_word_embeddings; /* 1 for TTS-1                                        */
  float rms_norm_eps;          /* 1e-5                                               */
  float rope_theta;            /* 500000                                             */
  int32_t rope_llama3;         /* 1: llama3 frequency smoothing                      */
  float rope_factor;           /* 32 (TTS-1) / 8 (TTS-1-Max)                         */
  float rope_low_freq_factor;  /* 1                                                  */
  float rope_high_freq_factor; /* 4                                                  */
  int32_t rope_original_max_position; /* 8192                                        */
  int32_t max_batch;           /* KV-cache slots (sequences resident at once)        */
  int32_t max_seq_len;         /* KV capacity per sequence (prompt + generated)      */
} tts_lm_config;

/* Loads the SpeechLM.  Weights are bf16, or f32 / f16 converted to bf16 on load (one RNE
 * rounding; exact for f16 values with at most 8 significant bits — the normal-range f16
 * images of bf16 checkpoint weights — and rounding for f16 subnormals below 6.1e-5 that
 * carry more, so such an f16 checkpoint does not load bit for bit).  The
 * engine always computes in bf16 with fp32 accumulation — the reference serving CLI's
 * fp16 arithmetic (tools/serving/inference.py:103-107) is not reproduced.
 * Optional tensors "rope.cos" / "rope.sin" ([max_seq_len, head_dim], bf16) override the
 * engine-computed RoPE table (the Python host passes the table computed exactly as
 * LlamaRotaryEmbedding.forward does).  Optional "vocab.id_to_code" (int32 [vocab]) is the
 * token-id -> speech-code LUT (-1 for non-speech ids), see tts_lm_id_to_code.
 * Greedy steps pick through an int8 copy of the lm_head made here (vocab x hidden bytes more
 * device memory) — the same ids as the bf16 lm_head; TTS_HEAD_SCREEN=0 at load
 * skips it. */
tts_status tts_lm_load(tts_engine* e, const tts_lm_config* cfg, const tts_tensor_desc* t,
                       int32_t n);

/* Generation parameters: the HF `generate` kwargs of inferencing.py:95-104. */
typedef struct {
  int32_t max_length;          /* TOTAL length incl. prompt (HF max_length)          */
  int32_t min_new_tokens;      /* EOS masked until this many new tokens exist        */
  int32_t eos_token_id;        /* <|speech_end|>; -1 = none                          */
  int32_t do_sample;           /* 0 = greedy (argmax, lowest index on ties)          */
  float repetition_penalty;    /* over the SET of ids in prompt+generated            */
  float temperature;           /* sampling only                                      */
  float top_p;                 /* sampling only                                      */
  int32_t top_k;               /* sampling only (HF default 50); 0 = off             */
  uint64_t seed;               /* sampling RNG seed                                  */
  float frequency_penalty;     /* vLLM form (inferencing.py:85): logit -= f * count of */
                               /* the id among the NEW tokens; 0 = off (HF form)       */
  int32_t reserved;
} tts_gen_params;

/* Runs prefill + the autoregressive decode loop for `batch` independent sequences.
 *   prompt_ids  host int32, the prompts concatenated            [sum(prompt_lens)]
 *   prompt_lens host int32                                      [batch]
 *   out_ids     host int32, NEW tokens per sequence, row stride `out_stride`
 *               (EOS included when produced, as HF returns it)  [batch][out_stride]
 *   out_lens    host int32, number of new tokens per sequence   [batch]
 * Each sequence is computed exactly as a batch-1 HF generate of that prompt would be
 * (ragged batching: no padding enters the arithmetic). */
tts_status tts_generate(tts_engine* e, const tts_gen_params* p, const int32_t* prompt_ids,
                        const int32_t* prompt_lens, int32_t batch, int32_t* out_ids,
                        int32_t out_stride, int32_t* out_lens, void* stream);

/* The same generation in pieces, for streaming callers (config 5: chunked AR decode with an
 * incremental codec).  tts_generate_begin validates, prefills and picks the first new
 * token of every sequence; tts_generate_continue runs up to `n_steps` further decode
 * steps (*all_done = 1 once every sequence has stopped: EOS or max_length);
 * tts_generate_read copies the new tokens produced so far (same layout as tts_generate's
 * outputs) and may be called after every continue.  Tokens are identical to one
 * tts_generate call with the same arguments.  One open generation per engine; a new
 * begin (or tts_generate) discards it. */
tts_status tts_generate_begin(tts_engine* e, const tts_gen_params* p, const int32_t* prompt_ids,
                              const int32_t* prompt_lens, int32_t batch, void* stream);
tts_status tts_generate_continue(tts_engine* e, int32_t n_steps, int32_t* all_done);
tts_status tts_generate_read(tts_engine* e, int32_t* out_ids, int32_t out_stride, int32_t* out_lens);

/* Continuous batching (serving): `n_slots` persistent decode rows share
 * one captured decode step and the settings `p` (max_length ignored).  A sequence is
 * admitted into a free slot between steps (tts_slots_add: prompt prefilled into that
 * slot, first token picked; max_new_tokens bounds it like HF max_length - prompt length),
 * tts_slots_step runs `n_steps` decode steps over all slots (*n_active = rows still
 * generating), tts_slots_read returns a slot's new tokens so far and whether it stopped,
 * tts_slots_release frees the slot (stopping it first if it is still running).  Each
 * sequence's tokens equal a batch-1 tts_generate of its prompt with the same settings
 * (rows never mix).  Opening slots discards an open tts_generate_begin generation. */
tts_status tts_slots_open(tts_engine* e, const tts_gen_params* p, int32_t n_slots, void* stream);
tts_status tts_slots_add(tts_engine* e, int32_t slot, const int32_t* prompt_ids, int32_t prompt_len,
                         int32_t max_new_tokens);
/* As tts_slots_add with the request's own sampling key (vLLM SamplingParams.seed): the
 * same key and prompt draw the same tokens whatever else the batch holds.  tts_slots_add
 * derives a distinct key per admitted request from the batch seed (p->seed). */
tts_status tts_slots_add_seeded(tts_engine* e, int32_t slot, const int32_t* prompt_ids, int32_t prompt_len,
                                int32_t max_new_tokens, uint64_t seed);
tts_status tts_slots_step(tts_engine* e, int32_t n_steps, int32_t* n_active);
tts_status tts_slots_read(tts_engine* e, int32_t slot, int32_t* out_ids, int32_t capacity, int32_t* n_out,
                          int32_t* finished);
tts_status tts_slots_release(tts_engine* e, int32_t slot);

/* Teacher-forced scoring (parity / debugging): runs the prefill over full sequences and
 * writes the bf16-rounded logits of the last `n_last` positions of each sequence, as
 * fp32, to host `logits` [batch][n_last][vocab]. */
tts_status tts_lm_score(tts_engine* e, const int32_t* ids, const int32_t* lens, int32_t batch,
                        int32_t n_last, float* logits, void* stream);

/* Teacher-forced scoring through the decode step: prefills the first lens[b] - n_last tokens
 * of each sequence, then feeds the last n_last tokens one decode step at a time (all
 * sequences as one batch: the kernels generate runs after its prefill) and writes each
 * step's bf16-rounded logits as fp32.  Same positions as tts_lm_score.  gather_idx
 * (optional, host [batch][n_last][k]) keeps only those vocabulary entries; with NULL,
 * k is ignored and the full [batch][n_last][vocab] is written.  Needs lens[b] > n_last. */
tts_status tts_lm_score_decode(tts_engine* e, const int32_t* ids, const int32_t* lens, int32_t batch,
                               int32_t n_last, const int32_t* gather_idx, int32_t k, float* logits,
                               void* stream);

/* Maps token ids to speech codes through the loaded LUT (-1 for non-speech ids). */
tts_status tts_lm_id_to_code(tts_engine* e, const int32_t* ids, int32_t n, int32_t* codes);

/* Device time of the last tts_generate, split in prefill / decode (milliseconds), and the
 * number of decode steps executed. */
tts_status tts_lm_last_timing(tts_engine* e, float* prefill_ms, float* decode_ms,
                              int32_t* decode_steps);

/* Times one decode-step kernel of the loaded model in isolation (HIP events on the engine
 * stream around `iters` back-to-back launches, after one warm-up launch) for roofline
 * accounting.  which: 0 qkv projection (+RMSNorm), 1 o_proj (+residual), 2 gate/up
 * (+RMSNorm, SwiGLU), 3 down_proj (+residual), 4 lm_head (+RMSNorm, penalty, argmax
 * partials), 5 decode attention (ctx = `ctx` positions), 6 qkv with the decode attention
 * fused in (1..16 rows where that form applies), 7 the same launch also carrying o_proj
 * (+residual; the 1..16-row step's default form where the shapes allow), 8 the greedy step's
 * screened lm_head (int8 screen + exact recheck of the tiles that can hold the argmax; <= 32
 * rows), 9 its int8 screen alone.  rows = batch rows.
 * Outputs: average ms per launch and the algorithmic HBM bytes one launch must move. */
tts_status tts_lm_bench_kernel(tts_engine* e, int32_t which, int32_t rows, int32_t ctx,
                               int32_t iters, float* avg_ms, double* bytes);

/* ---------------------------------------------------------------------- codec ------ */

/* xcodec2-compatible decoder (tts/core/codec/decoding.py:14-35 DecoderConfig). */
typedef struct {
  int32_t sample_rate;         /* 16000 / 24000 / 48000                               */
  int32_t token_rate;          /* 50                                                  */
  int32_t hop_length;          /* 320 / 160                                           */
  int32_t n_upsample;          /* len(upsample_factors), 0..4                         */
  int32_t upsample_factors[4];
  int32_t kernel_sizes[4];
  int32_t hidden_dim;          /* 1024                                                */
  int32_t depth;               /* 12 transformer blocks                               */
  int32_t heads;               /* 16                                                  */
  int32_t vq_dim;              /* 2048                                                */
  int32_t max_codes;           /* largest T of one utterance (tts_codec_decode rejects longer) */
} tts_codec_config;

tts_status tts_codec_load(tts_engine* e, const tts_codec_config* cfg, const tts_tensor_desc* t,
                          int32_t n);

/* Decodes `batch` code sequences (host int32, concatenated, lengths in `lens`) into
 * waveforms.  wav: float32 [sum(lens) * samples_per_code] concatenated in input order;
 * wav_is_device != 0 means `wav` is a device pointer.  wav_lens (host) receives each
 * utterance's sample count.  The batch runs as ragged passes of up to 32768 codes
 * (TTS_CODEC_PASS_CODES): every GEMM over all utterances of a pass, GroupNorm / attention /
 * overlap-add per utterance; an utterance's samples are bit-identical decoded alone or in
 * any batch.  Returns after the waveforms are written (the stream is synchronised). */
tts_status tts_codec_decode(tts_engine* e, const int32_t* codes, const int32_t* lens,
                            int32_t batch, float* wav, int32_t wav_is_device, int64_t* wav_lens,
                            void* stream);

tts_status tts_codec_samples_per_code(tts_engine* e, int32_t* out);

/* --------------------------------------------------------- prompt-audio encoder ---- */

/* Loads the codec ENCODER (the reference `Encoder` minus its w2v-bert feature model,
 * tts/core/codec/encoder.py:20-46): host f32 tensors by the reference state-dict names —
 * "semantic_encoder.*", "acoustic_encoder.*" (legacy weight_norm weight_g / weight_v; folded
 * here), "fusion_layer.*", "quantizer.project_in.*", and the anti-aliasing filter buffers
 * "acoustic_encoder.conv_final_block.0.upsample.filter" /
 * "...downsample.lowpass.filter" ([1, 1, 12]).  Replaces encoding.create / Encoder.__init__
 * + load_from_checkpoint (encoding.py:75-80, encoder.py:20-113). */
tts_status tts_encoder_load(tts_engine* e, const tts_tensor_desc* t, int32_t n);

/* Encodes one 16 kHz waveform to codec codes — Encoder.encode (encoder.py:115-128) from the
 * padding on, in fp32 on the device:
 *   wav           host f32 [n_samples]
 *   w2v_features  host f32 [n_frames][1024]: w2v-bert-2.0 hidden_states[16] of the padded
 *                 waveform's SeamlessM4T features (the reference's wav2vec_model call,
 *                 encoder.py:71; computed by the caller), n_frames = the 320-sample hops of
 *                 the waveform padded to a whole hop (plus one hop when already whole)
 *   codes         host int32 [codes_cap] <- n_codes = n_frames FSQ indices
 *   pre_round     optional host f32 [n_frames][8]: the values the FSQ rounded (diagnostics) */
tts_status tts_encoder_encode(tts_engine* e, const float* wav, int64_t n_samples, const float* w2v_features,
                              int32_t n_frames, int32_t* codes, int32_t codes_cap, int32_t* n_codes,
                              float* pre_round);

/* The same with w2v-bert-2.0 run here as well (its tensors given to tts_encoder_load under
 * the reference Encoder's "wav2vec_model." prefix: transformers Wav2Vec2BertModel names,
 * position_embeddings_type "relative_key", layers 0..15 used): features = the
 * SeamlessM4TFeatureExtractor input_features of the padded waveform, host f32
 * [n_frames][160] (the reference computes them on the CPU too, encoder.py:121-123). */
tts_status tts_encoder_encode_features(tts_engine* e, const float* wav, int64_t n_samples, const float* features,
                                       int32_t n_frames, int32_t* codes, int32_t codes_cap, int32_t* n_codes,
                                       float* pre_round);

#ifdef __cplusplus
}
#endif
#endif /* TTS_MI355X_H */
