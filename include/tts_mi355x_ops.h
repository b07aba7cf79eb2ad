/*
 * tts_mi355x_ops.h — op-level entry points of the same library, used by the parity tests
 * to check each kernel family in isolation against the CPU oracle.  All pointers are
 * device pointers of the current HIP device; `stream` is a hipStream_t (NULL = default).
 * These are not part of the drop-in surface (tts_mi355x.h) and may change between rounds.
 */
#ifndef TTS_MI355X_OPS_H
#define TTS_MI355X_OPS_H

#include <stdint.h>
#include "tts_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Deterministic synthetic weights: value_i = (2*u_i - 1) * scale, u_i = top 24 bits of
 * splitmix64(seed + (i+1)*golden) / 2^24.  dtype TTS_DT_F32 or TTS_DT_BF16 (RNE).  Bit-identical
 * to tts_amd.synth.synth_values (numpy). */
tts_status tts_synth_fill(void* dst, int32_t dtype, int64_t n, uint64_t seed, float scale,
                          void* stream);

/* W [N][K] bf16 row-major -> 1 KiB MFMA fragment tiles in the matrix's stream-plan order
 * (layout in lm_kernels.h / lm_gemm.hip).  epi = the epilogue the matrix will be used with:
 * 2 (SwiGLU) takes W = [gate; up] ([N/2][K] each) and interleaves their n-tiles. */
tts_status tts_op_retile(const void* w, void* w_tiled, int32_t N, int32_t K, int32_t epi, void* stream);

/* y[M][ldo] (bf16) = epilogue( A[M][K] . W^T ), A optionally RMSNorm'ed with normw.
 * epi: 0 store, 1 residual (resid += y, in place), 2 SwiGLU (W = interleaved gate/up tiles,
 * N = 2*intermediate, output [M][N/2]).  M <= 64. */
tts_status tts_op_wgemm(const void* x, int32_t M, int32_t K, int32_t ldx, const void* w_tiled,
                        int32_t N, const void* normw, float eps, void* out, int32_t ldo,
                        void* resid, int32_t epi, void* stream);

/* Prefill GEMM (many rows, one launch): same tiled weights and epilogues as tts_op_wgemm
 * (0 store, 1 residual, 2 SwiGLU), no fused RMSNorm, any M >= 1; N % 64 == 0, K % 128 == 0.
 * Every output sums its K in the canonical 1024-element chunks, in order, so a row's bits do
 * not depend on M or on the launch form (all of K per workgroup / one chunk per workgroup).
 * Replaces the per-token projections of transformers LlamaForCausalLM.forward over the
 * prompt (modeling_llama.py:163-176, 217-281) when the whole prompt batch is prefilled. */
tts_status tts_op_pgemm(const void* x, int32_t M, int32_t K, const void* w_tiled, int32_t N, void* out,
                        int32_t ldo, void* resid, int32_t epi, void* stream);

/* Sampling head (GenerationMixin._sample with TemperatureLogitsWarper, TopKLogitsWarper,
 * TopPLogitsWarper; transformers logits_process.py:238,473,542): rows of processed fp32
 * logits [B][V] -> one drawn token per row (tokens, device int32 [B]) and, when `probs` is
 * not NULL, the final distribution written into probs [B][V] at the kept ids (the caller
 * zero-fills it).  part_max (optional, [B][nparts]) = maxima of disjoint column blocks of
 * each row, used as the top-k lower bound the engine gets from its lm_head workgroups.
 * The draw is u = splitmix64(seed, row, step) in [0,1) walked over the kept ids in
 * descending-probability order (distribution-exact; not torch's RNG stream). */
tts_status tts_op_sample(const float* logits, int32_t B, int32_t V, float temperature, int32_t top_k,
                         float top_p, uint64_t seed, int32_t step, const float* part_max, int32_t nparts,
                         float* probs, int32_t* tokens, void* stream);

/* Diagnostics, no GPU needed: the kernels one decode step over `rows` rows of a model of
 * config `cfg` would launch on a GPU of `num_cu` CUs — the engine's own step code run with
 * its launchers in a dry-run mode (nothing allocated or launched).  Writes the unique launches
 * in first-seen order, one per line (the weight-streaming GEMMs as
 * "wgemm_kernel<template arguments>"), NUL-terminated, into out[cap].  The build's spill gate
 * (tests/test_kernel_resources.py) reads its hot instantiations from here. */
tts_status tts_debug_step_plan(const tts_lm_config* cfg, int32_t rows, int32_t num_cu, char* out, int32_t cap);

/* LlamaRMSNorm over rows of x (bf16). */
tts_status tts_op_rmsnorm(const void* x, const void* w, float eps, void* y, int32_t M, int32_t K,
                          void* stream);

/* fp32 GEMM on the codec path: C[M][N] = act(A[M][K] . B[N][K]^T + bias) (+ resid).
 * lda may be < K to express a sliding-window (im2col-free) conv operand.  act: 0 none,
 * 1 swish, 2 silu (same function), see codec_gemm.hip. */
tts_status tts_op_gemm_f32(const float* A, int32_t M, int32_t K, int32_t lda, const float* B,
                           int32_t N, const float* bias, float* C, int32_t ldc,
                           const float* resid, int32_t act, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TTS_MI355X_OPS_H */
