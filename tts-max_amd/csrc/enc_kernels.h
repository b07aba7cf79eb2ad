// enc_kernels.h — kernels of the prompt-audio encoder (enc_kernels.hip); its contractions run
// on the codec's fp32-exact GEMM (codec_kernels.h launch_gemm_f32).
#pragma once
#include <hip/hip_runtime.h>

namespace tts {

// conv windows of [T][C] for Conv1d(k, stride, dilation, pad) -> [To][k*C] (tap-major), rows
// lda apart
void launch_enc_im2col(const float* x, int T, int C, int k, int stride, int dil, int pad, int To, int lda,
                       float* a, hipStream_t s);
// Activation1d(SnakeBeta) on [T][C]: 2x up (fu, 12 taps), SnakeBeta(log-scale alpha, beta),
// 2x down (fd, 12 taps), replicate padding
void launch_enc_snake_aa(const float* x, int T, int C, const float* alpha, const float* beta, const float* fu,
                         const float* fd, float* y, hipStream_t s);
void launch_enc_relu(float* x, long long n, hipStream_t s);
// ResidualFSQ (one quantizer) on z [T][nl] -> codes [T]; pre (optional) = the rounded values
void launch_enc_fsq(const float* z, int T, int nl, const int* levels, int* codes, float* pre, hipStream_t s);

// w2v-bert conformer ops: GLU over channel halves of [T][2C]; causal depthwise conv (left
// pad k-1, w [C][k]); swish in place; relative-key self-attention (head dim 64, distance
// embedding E [L + R + 1][64]) on fused qkv rows [3 * H * 64] -> [T][H * 64]
void launch_enc_glu(const float* x, int T, int C, float* y, hipStream_t s);
void launch_enc_dwconv(const float* x, int T, int C, const float* w, int k, float* y, hipStream_t s);
void launch_enc_swish(float* x, long long n, hipStream_t s);
void launch_enc_relattn(const float* qkv, int T, int H, const float* E, int L, int R, float* out, hipStream_t s);

}  // namespace tts
