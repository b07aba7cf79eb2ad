// enc_kernels.hip — the prompt-audio encoder's non-GEMM kernels (gfx950, fp32 end to end as
// the reference): conv windows (im2col) for the dilated / strided convolutions, the
// anti-aliased SnakeBeta activation, ReLU, and the FSQ quantizer.  Every contraction goes
// through the codec's fp32-exact GEMM (codec_kernels.hip, launch_gemm_f32).
// Reference: tts/core/codec/encoder_modules.py, activations.py, filters.py, encoder.py.
#include "hip_common.h"
#include "enc_kernels.h"

namespace tts {

// A[t][j*C + c] = x[t*stride + j*dil - pad][c], zero outside [0, T): the window of output t
// of Conv1d(k, stride, dilation, padding) in the tap-major order of the re-laid-out weight
// [Cout][k*Cin]; rows lda apart (lda >= k*C: the GEMM's K padded to its step).
__global__ void enc_im2col_kernel(const float* __restrict__ x, int T, int C, int k, int stride, int dil, int pad,
                                  int To, int lda, float* __restrict__ a) {
  const long long total = (long long)To * k * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long r = i / C;
    const int j = (int)(r % k), t = (int)(r / k);
    const int src = t * stride + j * dil - pad;
    a[(size_t)t * lda + (size_t)j * C + c] = (src >= 0 && src < T) ? x[(size_t)src * C + c] : 0.f;
  }
}

void launch_enc_im2col(const float* x, int T, int C, int k, int stride, int dil, int pad, int To, int lda,
                       float* a, hipStream_t s) {
  const long long total = (long long)To * k * C;
  const long long g = (total + 255) / 256;
  hipLaunchKernelGGL(enc_im2col_kernel, dim3((unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g))), dim3(256), 0, s,
                     x, T, C, k, stride, dil, pad, To, lda, a);
}

// Activation1d(SnakeBeta(alpha_logscale=True)) on a time-major [T][C] signal (filters.py:
// UpSample1d(2, 12) then SnakeBeta then DownSample1d(2, 12)), one output sample per thread:
//   u[m] = 2 * sum_i xp[i] f[m + 15 - 2i],  xp[i] = x[clamp(i - 5)]     (m = 0 .. 2T-1)
//   z[m] = u + 1 / (exp(beta) + 1e-9) * sin(u * exp(alpha))^2
//   y[t] = sum_j g[j] z[clamp(2t + j - 5)]                              (t = 0 .. T-1)
// clamp = the replicate padding of both filters.
__global__ void enc_snake_aa_kernel(const float* __restrict__ x, int T, int C, const float* __restrict__ alpha,
                                    const float* __restrict__ beta, const float* __restrict__ fu,
                                    const float* __restrict__ fd, float* __restrict__ y) {
  __shared__ float sf[24];
  if (threadIdx.x < 12) sf[threadIdx.x] = fu[threadIdx.x];
  else if (threadIdx.x < 24) sf[threadIdx.x] = fd[threadIdx.x - 12];
  __syncthreads();
  const long long total = (long long)T * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C), t = (int)(i / C);
    const float a = expf(alpha[c]), ib = 1.0f / (expf(beta[c]) + 1e-9f);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      int m = 2 * t + j - 5;
      m = m < 0 ? 0 : (m > 2 * T - 1 ? 2 * T - 1 : m);
      // u[m]: taps i with 0 <= m + 15 - 2i < 12
      const int ilo = (m + 15 - 11 + 1) / 2, ihi = (m + 15) / 2;
      float u = 0.f;
      for (int ii = ilo; ii <= ihi; ++ii) {
        int src = ii - 5;
        src = src < 0 ? 0 : (src > T - 1 ? T - 1 : src);
        u += x[(size_t)src * C + c] * sf[m + 15 - 2 * ii];
      }
      u *= 2.f;
      const float sn = sinf(u * a);
      const float z = u + ib * (sn * sn);
      acc += sf[12 + j] * z;
    }
    y[i] = acc;
  }
}

void launch_enc_snake_aa(const float* x, int T, int C, const float* alpha, const float* beta, const float* fu,
                         const float* fd, float* y, hipStream_t s) {
  const long long total = (long long)T * C;
  const long long g = (total + 255) / 256;
  hipLaunchKernelGGL(enc_snake_aa_kernel, dim3((unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g))), dim3(256), 0, s,
                     x, T, C, alpha, beta, fu, fd, y);
}

__global__ void enc_relu_kernel(float* __restrict__ x, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    x[i] = fmaxf(x[i], 0.f);
}

void launch_enc_relu(float* x, long long n, hipStream_t s) {
  const long long g = (n + 255) / 256;
  hipLaunchKernelGGL(enc_relu_kernel, dim3((unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g))), dim3(256), 0, s, x, n);
}

// ResidualFSQ(levels, one quantizer) on project_in's output z [T][nl]: the residual is
// bound(z) and the FSQ layer bounds it again (vector_quantize_pytorch 1.17.8; the HF Xcodec2
// port keeps the double bound too), rounds half to even (torch.round), and the index is
// sum_j (q_j + L_j/2) * prod_{i<j} L_i.  One thread per frame; pre (optional) = the values
// that were rounded.
__global__ void enc_fsq_kernel(const float* __restrict__ z, int T, int nl, const int* __restrict__ levels,
                               int* __restrict__ codes, float* __restrict__ pre) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  int idx = 0, basis = 1;
  for (int j = 0; j < nl; ++j) {
    const int L = levels[j];
    const float half_l = (float)(L - 1) * (1.0f + 1e-3f) / 2.0f;
    const float offset = (L % 2 == 0) ? 0.5f : 0.0f;
    const float shift = atanhf(offset / half_l);
    float v = z[(size_t)t * nl + j];
    v = tanhf(v + shift) * half_l - offset;
    v = tanhf(v + shift) * half_l - offset;
    if (pre) pre[(size_t)t * nl + j] = v;
    const int q = (int)rintf(v);
    idx += (q + L / 2) * basis;
    basis *= L;
  }
  codes[t] = idx;
}

void launch_enc_fsq(const float* z, int T, int nl, const int* levels, int* codes, float* pre, hipStream_t s) {
  hipLaunchKernelGGL(enc_fsq_kernel, dim3((T + 127) / 128), dim3(128), 0, s, z, T, nl, levels, codes, pre);
}

}  // namespace tts
