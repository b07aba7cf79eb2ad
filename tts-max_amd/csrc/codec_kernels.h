// codec_kernels.h — fp32 kernels of the xcodec2-compatible codec decoder (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tts {

// C[M][ldc] = act(A . B^T + bias) (+ resid), A row r at A + r*lda (lda may be < K: sliding
// window view of a time-major activation = Conv1d without im2col), B [N][K] row-major.
struct GemmF32Args {
  const float* A = nullptr;
  int M = 0, K = 0, lda = 0;
  const float* B = nullptr;
  int N = 0;
  const float* bias = nullptr;
  float* C = nullptr;
  int ldc = 0;
  const float* resid = nullptr;  // [M][ldc]
  int act = 0;                   // 0 none, 1 swish/silu
  // split-K over workgroups (short utterances / streaming windows: few output tiles, long
  // K): fp32 partials [ksplit][M][N] in `part`, summed in split order by a reduce kernel
  float* part = nullptr;
  size_t part_elems = 0;  // capacity of `part`
  int ksplit = 1, kchunk = 0;
};
void launch_gemm_f32(const GemmF32Args& g, hipStream_t s);

// FSQ index -> 8 base-4 digits -> (d-2)/2 -> project_out Linear(8 -> vq_dim)
void launch_fsq_project(const int* codes, int T, const float* w, const float* b, float* out,
                        int vq_dim, hipStream_t s);
// GroupNorm(32, eps) statistics over [T][C] time-major (per group: mean, rstd)
void launch_groupnorm_stats(const float* x, int T, int C, int groups, float eps, float* stats,
                            hipStream_t s);
// y = swish(GN(x)*gamma + beta)
void launch_groupnorm_swish(const float* x, int T, int C, int groups, const float* stats,
                            const float* gamma, const float* beta, float* y, hipStream_t s);
// codec RMSNorm (decoder_modules.py:226-236): x * rsqrt(mean(x^2) + eps) * w
void launch_rmsnorm_f32(const float* x, int T, int C, const float* w, float eps, float* y,
                        hipStream_t s);
// LayerNorm over channels with affine
void launch_layernorm_f32(const float* x, int T, int C, const float* w, const float* b, float eps,
                          float* y, hipStream_t s);
// torchtune RoPE applied with position = head index, interleaved pairs, in place on q and k
void launch_codec_rope(float* qkv, int T, int heads, int hd, hipStream_t s);
// non-causal full attention, fp32, qkv [T][3*heads*hd] -> out [T][heads*hd]
void launch_codec_attention(const float* qkv, int T, int heads, int hd, float* out,
                            hipStream_t s);
// ConvTranspose1d gather: y[t'][co] = b[co] + sum_j Z[(t'+pad-j)/u][j*Cout+co]
void launch_convt_gather(const float* Z, int T, int Cout, int k, int u, int pad,
                         const float* bias, float* y, hipStream_t s);
// ISTFT head: spec[f][c] from head[f][2*nb]: mag = min(exp(m), 100); re = mag cos p, im = mag sin p
void launch_istft_spec(const float* head, int F, int nb, int ld, float* spec, hipStream_t s);
// overlap-add of windowed frames [F][nfft] with hop, trim (nfft-hop)/2, divide by envelope
void launch_ola(const float* frames, int F, int nfft, int hop, const float* window, float* y,
                hipStream_t s);
void launch_zero(float* p, long long n, hipStream_t s);

}  // namespace tts
