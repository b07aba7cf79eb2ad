// codec_kernels.h — fp32 kernels of the xcodec2-compatible codec decoder (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>

namespace tts {

// A ragged batch of utterances in one time-major buffer: utterance b's frames are rows
// [row, row + T) of the buffer, with kCodecPad zero rows before the first utterance and after
// every utterance (a Conv1d window's padding).  One table per time resolution.
constexpr int kCodecPad = 3;
struct CodecSeg {
  int T, row;
};

// C[M][ldc] = act(A . B^T + bias) (+ resid), A row r at A + r*lda (lda may be < K: sliding
// window view of a time-major activation = Conv1d without im2col), B [N][K] row-major.
struct GemmF32Args {
  const float* A = nullptr;
  int M = 0, K = 0, lda = 0;
  const float* B = nullptr;
  const uint16_t* Bp = nullptr;  // optional: B split into bf16 planes [3][N][K] (launch_split_planes)
  // optional: A split into bf16 planes with A's addressing (element (m, k) of plane p at
  // Ap + p * ap_plane + m * lda + k; Ap stands for A's own base)
  const uint16_t* Ap = nullptr;
  long long ap_plane = 0;
  int N = 0;
  const float* bias = nullptr;
  float* C = nullptr;
  int ldc = 0;
  const float* resid = nullptr;  // [M][ldc]
  int act = 0;                   // 0 none, 1 swish/silu
  // optional output as bf16 planes for a consuming GEMM (gemm_x3p): element (m, n) of plane p
  // at Cp + p * cp_plane + m * ldc + n (C may then be null)
  uint16_t* Cp = nullptr;
  long long cp_plane = 0;
  // split-K over workgroups (fp32 partials [ksplit][M][N] in `part`, summed in split order by
  // a reduce kernel): kept by the kernels, never used by launch_gemm_f32 (M-independent sums)
  float* part = nullptr;
  size_t part_elems = 0;  // capacity of `part`
  int ksplit = 1, kchunk = 0;
};
void launch_gemm_f32(const GemmF32Args& g, hipStream_t s);
// the same contraction with A and B both given as planes (Ap, Bp; codec_gemm.hip)
bool gemm_x3p_supported(const GemmF32Args& g);
void launch_gemm_x3p(const GemmF32Args& g, hipStream_t s);
// diagnostic (stamps) build: print and reset the K-loop phase sums of gemm_x3p; no-op otherwise
void x3p_stamps_dump(FILE* f);
// planes[0..3n) = the (h, m, l) bf16 split of x[0..n) the GEMM applies to its operands
void launch_split_planes(const float* x, uint16_t* planes, long long n, hipStream_t s);

// FSQ index -> 8 base-4 digits -> (d-2)/2 -> project_out Linear(8 -> vq_dim); code i lands
// on buffer row code_row[i]
void launch_fsq_project(const int* codes, const int* code_row, int n, const float* w, const float* b,
                        float* out, int vq_dim, hipStream_t s);
// zero the kCodecPad rows before the first and after every utterance of a ragged buffer
void launch_zero_gaps(float* x, int C, const CodecSeg* seg, int B, hipStream_t s, uint16_t* xp = nullptr,
                      long long plane = 0);
// GroupNorm(32, eps) statistics of each utterance (stats [B][groups][mean, rstd])
void launch_groupnorm_stats(const float* x, const CodecSeg* seg, int B, int C, int groups, float eps,
                            float* stats, hipStream_t s);
// y = swish(GN(x)*gamma + beta) per utterance; y's gap rows are zeroed (a Conv1d input).
// With yp: y's bf16 planes (gemm_x3p's A operand, element offsets of y) instead of y
void launch_groupnorm_swish(const float* x, const CodecSeg* seg, int B, int max_T, int C, int groups,
                            const float* stats, const float* gamma, const float* beta, float* y, hipStream_t s,
                            uint16_t* yp = nullptr, long long plane = 0);
// codec RMSNorm (decoder_modules.py:226-236): x * rsqrt(mean(x^2) + eps) * w
void launch_rmsnorm_f32(const float* x, int T, int C, const float* w, float eps, float* y,
                        hipStream_t s, uint16_t* yp = nullptr, long long plane = 0);
// LayerNorm over channels with affine
void launch_layernorm_f32(const float* x, int T, int C, const float* w, const float* b, float eps,
                          float* y, hipStream_t s);
// non-causal full attention within each utterance, fp32, qkv rows [3*heads*hd] (q and k
// before RoPE: the torchtune rotation with position = head index is applied while staging)
// -> out rows [heads*hd]; qblk = (utterance, first query) of each 64-query block,
// codec_attn_qblocks(T) per utterance
int codec_attn_qblocks(int T);
int codec_attn_qrows();  // queries per block (first query of block q = q * codec_attn_qrows())
void launch_codec_attention(const float* qkv, const CodecSeg* seg, const int2* qblk, int nqblk, int heads,
                            int hd, const float* rope_cs, float* out, hipStream_t s, uint16_t* outp = nullptr,
                            long long plane = 0);
// rope_cs [heads][hd/2][cos, sin] of that rotation (once, at load)
void launch_codec_rope_table(float* rope_cs, int heads, hipStream_t s);
// ConvTranspose1d gather per utterance: y[t'][co] = b[co] + sum_j Z[(t'+pad-j)/u][j*Cout+co]
void launch_convt_gather(const float* Z, const CodecSeg* seg_in, const CodecSeg* seg_out, int B, int max_To, int Cout,
                         int k, int u, int pad, const float* bias, float* y, hipStream_t s);
// ISTFT head: spec[f][c] from head[f][2*nb]: mag = min(exp(m), 100); re = mag cos p, im = mag sin p
void launch_istft_spec(const float* head, int F, int nb, int ld, float* spec, hipStream_t s);
// overlap-add of each utterance's windowed frames [F][nfft] with hop, trim (nfft-hop)/2,
// divide by the envelope; utterance b's samples start at y + wav_off[b]
void launch_ola(const float* frames, const CodecSeg* seg, const long long* wav_off, int B, int max_F, int nfft,
                int hop, const float* window, float* y, hipStream_t s);
void launch_zero(float* p, long long n, hipStream_t s);

}  // namespace tts
