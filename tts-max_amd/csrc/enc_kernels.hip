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

namespace tts {

// ------------------------------------------------------------ w2v-bert conformer ops ----
// (transformers models/wav2vec2_bert/modeling_wav2vec2_bert.py: Wav2Vec2BertConvolutionModule
// 157-226, Wav2Vec2BertSelfAttention 229-330 with position_embeddings_type "relative_key")

// GLU(dim=channels) on [T][2C]: a * sigmoid(b), a = the first C channels
__global__ void enc_glu_kernel(const float* __restrict__ x, int T, int C, float* __restrict__ y) {
  const long long total = (long long)T * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C), t = (int)(i / C);
    const float a = x[(size_t)t * 2 * C + c], b = x[(size_t)t * 2 * C + C + c];
    y[i] = a * (1.0f / (1.0f + expf(-b)));
  }
}

void launch_enc_glu(const float* x, int T, int C, float* y, hipStream_t s) {
  const long long g = ((long long)T * C + 255) / 256;
  hipLaunchKernelGGL(enc_glu_kernel, dim3((unsigned)(g > 65536 ? 65536 : g)), dim3(256), 0, s, x, T, C, y);
}

// causal depthwise Conv1d(k, groups = C, no bias): the sequence padded by k-1 zeros on the
// left only: y[t][c] = sum_j w[c][j] x[t - (k-1) + j][c]
__global__ void enc_dwconv_kernel(const float* __restrict__ x, int T, int C, const float* __restrict__ w, int k,
                                  float* __restrict__ y) {
  const long long total = (long long)T * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C), t = (int)(i / C);
    float acc = 0.f;
    for (int j = 0; j < k; ++j) {
      const int src = t - (k - 1) + j;
      if (src >= 0) acc += w[(size_t)c * k + j] * x[(size_t)src * C + c];
    }
    y[i] = acc;
  }
}

void launch_enc_dwconv(const float* x, int T, int C, const float* w, int k, float* y, hipStream_t s) {
  const long long g = ((long long)T * C + 255) / 256;
  hipLaunchKernelGGL(enc_dwconv_kernel, dim3((unsigned)(g > 65536 ? 65536 : g)), dim3(256), 0, s, x, T, C, w, k, y);
}

__global__ void enc_swish_kernel(float* __restrict__ x, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float v = x[i];
    x[i] = v * (1.0f / (1.0f + expf(-v)));
  }
}

void launch_enc_swish(float* x, long long n, hipStream_t s) {
  const long long g = (n + 255) / 256;
  hipLaunchKernelGGL(enc_swish_kernel, dim3((unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g))), dim3(256), 0, s, x, n);
}

// Self-attention with relative-key position scores, head dim 64, fp32:
//   s[i][j] = q_i.k_j / 8 + q_i.E[clamp(j - i, -L, R) + L] / 8,  softmax over j,  o_i = sum p v
// One workgroup = (head, 32 queries); thread (query tid / 8, part tid % 8) walks keys
// part, part + 8, ... of each 64-key tile (K and V staged in LDS, rows padded to 68 floats:
// conflict-free 16-B reads) with an online softmax, then the 8 parts of a query (adjacent
// lanes) merge their (max, sum, o) in a fixed order.  qkv rows [3 * H * 64] (q | k | v, head
// h at h * 64), out rows [H * 64].
constexpr int RA_Q = 32, RA_KT = 64, RA_LD = 68, RA_NR = 73;
__global__ __launch_bounds__(256) void enc_relattn_kernel(const float* __restrict__ qkv, int T, int H,
                                                          const float* __restrict__ E, int L, int R,
                                                          float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float Ks[RA_KT * RA_LD], Vs[RA_KT * RA_LD];
  __shared__ float QE[RA_Q * RA_NR];
  const int h = blockIdx.y, q0 = blockIdx.x * RA_Q;
  const int tid = threadIdx.x, qi = tid >> 3, part = tid & 7;
  const int qrow = min(q0 + qi, T - 1);
  const int ld = 3 * H * 64;
  const float* qp = qkv + (size_t)qrow * ld + h * 64;
  float q[64];
#pragma unroll
  for (int d = 0; d < 64; d += 4) {
    const float4 v = *(const float4*)(qp + d);
    q[d] = v.x; q[d + 1] = v.y; q[d + 2] = v.z; q[d + 3] = v.w;
  }
  // q . E_r for the 73 distance rows: thread (qi, part) takes r = part, part + 8, ...
  for (int r = part; r < L + R + 1; r += 8) {
    const float* e = E + (size_t)r * 64;
    float acc = 0.f;
#pragma unroll
    for (int d = 0; d < 64; ++d) acc += q[d] * e[d];
    QE[qi * RA_NR + r] = acc;
  }
  float m = -INFINITY, l = 0.f, o[64];
#pragma unroll
  for (int d = 0; d < 64; ++d) o[d] = 0.f;
  const int i = q0 + qi;
  for (int k0 = 0; k0 < T; k0 += RA_KT) {
    __syncthreads();
    for (int e = tid; e < RA_KT * 16; e += 256) {  // 64 keys x 16 float4 each of K and V
      const int kr = e >> 4, c4 = (e & 15) * 4;
      const int src = min(k0 + kr, T - 1);
      *(float4*)(Ks + kr * RA_LD + c4) = *(const float4*)(qkv + (size_t)src * ld + H * 64 + h * 64 + c4);
      *(float4*)(Vs + kr * RA_LD + c4) = *(const float4*)(qkv + (size_t)src * ld + 2 * H * 64 + h * 64 + c4);
    }
    __syncthreads();
    for (int kk = part; kk < RA_KT; kk += 8) {
      const int j = k0 + kk;
      if (j >= T) break;
      const float* kr = Ks + kk * RA_LD;
      float dot = 0.f;
#pragma unroll
      for (int d = 0; d < 64; d += 4) {
        const float4 kv = *(const float4*)(kr + d);
        dot += q[d] * kv.x + q[d + 1] * kv.y + q[d + 2] * kv.z + q[d + 3] * kv.w;
      }
      int dist = j - i;
      dist = dist < -L ? -L : (dist > R ? R : dist);
      const float s = dot / 8.0f + QE[qi * RA_NR + dist + L] / 8.0f;
      if (s > m) {
        const float sc = expf(m - s);
        l *= sc;
#pragma unroll
        for (int d = 0; d < 64; ++d) o[d] *= sc;
        m = s;
      }
      const float p = expf(s - m);
      l += p;
      const float* vr = Vs + kk * RA_LD;
#pragma unroll
      for (int d = 0; d < 64; d += 4) {
        const float4 vv = *(const float4*)(vr + d);
        o[d] += p * vv.x; o[d + 1] += p * vv.y; o[d + 2] += p * vv.z; o[d + 3] += p * vv.w;
      }
    }
  }
  // merge the 8 parts of the query (lanes 8qi .. 8qi+7 of the wave), partner order fixed
#pragma unroll
  for (int off = 1; off < 8; off <<= 1) {
    const float m2 = __shfl_xor(m, off, 64), l2 = __shfl_xor(l, off, 64);
    const float mn = fmaxf(m, m2);
    const float a = (m == -INFINITY) ? 0.f : expf(m - mn), b = (m2 == -INFINITY) ? 0.f : expf(m2 - mn);
    l = l * a + l2 * b;
#pragma unroll
    for (int d = 0; d < 64; ++d) {
      const float o2 = __shfl_xor(o[d], off, 64);
      o[d] = o[d] * a + o2 * b;
    }
    m = mn;
  }
  if (q0 + qi < T) {
    float* op = out + (size_t)(q0 + qi) * H * 64 + h * 64 + part * 8;
#pragma unroll
    for (int d = 0; d < 8; ++d) {
      float v = 0.f;
#pragma unroll
      for (int e = 0; e < 64; ++e) v = (e == part * 8 + d) ? o[e] : v;  // (register-indexed select)
      op[d] = v / l;
    }
  }
}

void launch_enc_relattn(const float* qkv, int T, int H, const float* E, int L, int R, float* out, hipStream_t s) {
  hipLaunchKernelGGL(enc_relattn_kernel, dim3((T + RA_Q - 1) / RA_Q, H), dim3(256), 0, s, qkv, T, H, E, L, R, out);
}

}  // namespace tts
