// codec_engine.cpp — codec decoder host runtime: weight loading (weight-norm fold, conv
// re-layout, iDFT basis), workspaces, and the Decoder.forward launch sequence.
//
// Reference: tts/core/codec/decoder.py:69-89 (Decoder.forward), decoding.py:84-89
// (AudioDecoder.decode), decoder_modules.py (Generator / VocosBackbone / ISTFTHead),
// upsampler.py (UpSamplerBlock).  The reference decodes one utterance per call in fp32.
// A batch runs as ONE ragged pass: the utterances are stacked in each
// time-major buffer with kCodecPad zero rows between them, every GEMM covers all of them
// (M = sum T + gaps: one utterance alone is far too small to fill 256 CUs), and only the
// ops that span an utterance take its bounds — GroupNorm statistics per utterance,
// block-diagonal attention, ConvTranspose gather and overlap-add.  Every op computes a row
// with the same arithmetic whatever the batch (the GEMM sums K in canonical chunks), so an
// utterance's waveform is bit-identical decoded alone or in any batch.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <memory>

#include "codec_kernels.h"
#include "engine.h"

namespace tts {

static constexpr int kPad = kCodecPad;  // zero rows before / after every utterance

struct CodecResBlock {
  float *n1w, *n1b, *c1w, *c1b, *n2w, *n2b, *c2w, *c2b;  // conv weights re-laid [co][3*ci]
  int C;
};
struct CodecTfBlock {
  float *att_norm, *ffn_norm, *c_attn, *c_proj, *fc1, *fc2;
};
struct CodecUp {
  float* wz;    // [k*Cout][Cin]: Z = x . wz^T
  float* bias;  // [Cout]
  int Cin, Cout, k, u, pad;
  CodecResBlock rb;
};

struct Codec {
  tts_codec_config cfg{};
  DevBuf weights;
  float *po_w, *po_b, *fc_w, *fc_b, *emb_w, *emb_b;
  CodecResBlock prior[2], post[2];
  std::vector<CodecTfBlock> tf;
  float *ln_w, *ln_b;
  std::vector<CodecUp> ups;
  float *out_w = nullptr, *out_b = nullptr;  // upsampler out_proj
  float *head_w, *head_b;                    // [ldh][1024] zero-padded rows, [ldh]
  float* basis;                              // [nfft][ldh] windowed irfft basis
  float* window;                             // [nfft]
  int nfft = 0, nb = 0, ldh = 0;
  int cap_T = 0;
  // ragged-batch workspace, grown on demand (rows = padded rows of one pass)
  DevBuf b0, b1, b2, big, qkv, stats, head, spec, frames;
  DevBuf meta;   // segment tables, wave offsets, code rows, attention query blocks
  DevBuf planes;  // every GEMM weight (B operand) split once into its bf16 h / m / l planes
  // bf16 planes [3][rows * C] of the activations only GEMMs read (gemm_x3p's A operand, the
  // same element offsets as the fp32 buffer they replace): b2 (RMSNorm / attention / GroupNorm +
  // swish outputs) and the fc1 -> fc2 hidden (4 D wide)
  DevBuf b2p, bigpp;
  DevBuf rope_cs;  // [heads][32][cos, sin] of the attention's RoPE
  std::map<const float*, const uint16_t*> bplanes;
  DevBuf codes, wav;  // all utterances' codes; host-bound waveforms staged on the device
};

void codec_destroy(Codec* c) { delete c; }

int codec_samples_per_code(Engine* e) {
  TTS_REQUIRE(e->codec != nullptr, "tts_codec_load has not been called");
  const tts_codec_config& c = e->codec->cfg;
  int ups = 1;
  for (int i = 0; i < c.n_upsample; ++i) ups *= c.upsample_factors[i];
  return c.hop_length * ups;
}

namespace {

struct HostTensors {
  std::map<std::string, const tts_tensor_desc*> m;
  const tts_tensor_desc& get(const std::string& n, std::initializer_list<int64_t> shape) const {
    auto it = m.find(n);
    if (it == m.end()) throw Error(TTS_E_INVALID, "missing codec tensor: " + n);
    const tts_tensor_desc& d = *it->second;
    bool ok = (int)shape.size() == d.ndim;
    int i = 0;
    for (int64_t v : shape) { if (ok && d.shape[i] != v) ok = false; ++i; }
    if (!ok) throw Error(TTS_E_INVALID, "bad shape for codec tensor: " + n);
    TTS_REQUIRE(d.dtype == TTS_DT_F32, "codec tensor must be f32: " + n);
    TTS_REQUIRE(!d.on_device, "codec tensors must be host memory: " + n);
    return d;
  }
  bool has(const std::string& n) const { return m.count(n) != 0; }
};

struct Slab {
  std::vector<std::pair<size_t, std::vector<float>>> parts;  // (offset, data)
  size_t size = 0;
  size_t add(std::vector<float>&& v) {
    const size_t off = size;
    size += (v.size() + 63) & ~(size_t)63;  // 256-B aligned sub-buffers
    parts.emplace_back(off, std::move(v));
    return off;
  }
};

std::vector<float> copy_of(const tts_tensor_desc& d) {
  const float* p = (const float*)d.data;
  return std::vector<float>(p, p + numel(d));
}

// Conv1d weight [co][ci][k] -> [co][k*ci] (tap-major), matching the sliding-window A row.
std::vector<float> conv_relayout(const tts_tensor_desc& d) {
  const int co = (int)d.shape[0], ci = (int)d.shape[1], k = (int)d.shape[2];
  const float* p = (const float*)d.data;
  std::vector<float> o((size_t)co * ci * k);
  for (int a = 0; a < co; ++a)
    for (int b = 0; b < ci; ++b)
      for (int j = 0; j < k; ++j) o[(size_t)a * k * ci + (size_t)j * ci + b] = p[((size_t)a * ci + b) * k + j];
  return o;
}

}  // namespace

void codec_load(Engine* e, const tts_codec_config* cfgp, const tts_tensor_desc* t, int n) {
  const tts_codec_config c = *cfgp;
  TTS_REQUIRE(c.hidden_dim == 1024 && c.heads == 16 && c.vq_dim >= 8,
              "codec: hidden_dim 1024 / 16 heads of 64 expected");
  TTS_REQUIRE(c.n_upsample >= 0 && c.n_upsample <= 4, "codec: at most 4 upsample stages");
  int ups = 1;
  for (int i = 0; i < c.n_upsample; ++i) ups *= c.upsample_factors[i];
  // decoder.py:31-37 guard
  TTS_REQUIRE(c.sample_rate / c.hop_length / ups == 50,
              "hop length and upsample factors do not match the sample rate (50 Hz tokens)");
  TTS_REQUIRE(c.max_codes >= 1, "max_codes must be >= 1");
  HostTensors tm;
  for (int i = 0; i < n; ++i) tm.m[t[i].name] = &t[i];
  const int D = c.hidden_dim, VQ = c.vq_dim;
  std::unique_ptr<Codec> cd(new Codec());
  cd->cfg = c;
  Slab slab;
  struct Fix { float** dst; size_t off; };
  std::vector<Fix> fixes;
  auto put = [&](float** dst, std::vector<float>&& v) { fixes.push_back({dst, slab.add(std::move(v))}); };

  put(&cd->po_w, copy_of(tm.get("decoder.quantizer.project_out.weight", {VQ, 8})));
  put(&cd->po_b, copy_of(tm.get("decoder.quantizer.project_out.bias", {VQ})));
  put(&cd->fc_w, copy_of(tm.get("fc_post_a.weight", {D, VQ})));
  put(&cd->fc_b, copy_of(tm.get("fc_post_a.bias", {D})));
  put(&cd->emb_w, conv_relayout(tm.get("decoder.backbone.embed.weight", {D, D, 7})));
  put(&cd->emb_b, copy_of(tm.get("decoder.backbone.embed.bias", {D})));
  auto resblock = [&](CodecResBlock& rb, const std::string& pre, int C) {
    rb.C = C;
    put(&rb.n1w, copy_of(tm.get(pre + "norm1.weight", {C})));
    put(&rb.n1b, copy_of(tm.get(pre + "norm1.bias", {C})));
    put(&rb.c1w, conv_relayout(tm.get(pre + "conv1.weight", {C, C, 3})));
    put(&rb.c1b, copy_of(tm.get(pre + "conv1.bias", {C})));
    put(&rb.n2w, copy_of(tm.get(pre + "norm2.weight", {C})));
    put(&rb.n2b, copy_of(tm.get(pre + "norm2.bias", {C})));
    put(&rb.c2w, conv_relayout(tm.get(pre + "conv2.weight", {C, C, 3})));
    put(&rb.c2b, copy_of(tm.get(pre + "conv2.bias", {C})));
  };
  for (int i = 0; i < 2; ++i) {
    resblock(cd->prior[i], "decoder.backbone.prior_net." + std::to_string(i) + ".", D);
    resblock(cd->post[i], "decoder.backbone.post_net." + std::to_string(i) + ".", D);
  }
  cd->tf.resize(c.depth);
  for (int i = 0; i < c.depth; ++i) {
    const std::string pre = "decoder.backbone.transformers." + std::to_string(i) + ".";
    CodecTfBlock& b = cd->tf[i];
    put(&b.att_norm, copy_of(tm.get(pre + "att_norm.weight", {D})));
    put(&b.ffn_norm, copy_of(tm.get(pre + "ffn_norm.weight", {D})));
    put(&b.c_attn, copy_of(tm.get(pre + "att.c_attn.weight", {3 * D, D})));
    put(&b.c_proj, copy_of(tm.get(pre + "att.c_proj.weight", {D, D})));
    put(&b.fc1, copy_of(tm.get(pre + "mlp.fc1.weight", {4 * D, D})));
    put(&b.fc2, copy_of(tm.get(pre + "mlp.fc2.weight", {D, 4 * D})));
  }
  put(&cd->ln_w, copy_of(tm.get("decoder.backbone.final_layer_norm.weight", {D})));
  put(&cd->ln_b, copy_of(tm.get("decoder.backbone.final_layer_norm.bias", {D})));
  cd->ups.resize(c.n_upsample);
  int C = D;
  for (int i = 0; i < c.n_upsample; ++i) {
    CodecUp& u = cd->ups[i];
    u.Cin = C; u.Cout = C / 2; u.k = c.kernel_sizes[i]; u.u = c.upsample_factors[i];
    u.pad = (u.k - u.u) / 2;
    TTS_REQUIRE((u.k - u.u) % 2 == 0, "ConvTranspose1d: (k - u) must be even");
    const std::string pre = "upsampler.upsample_layers." + std::to_string(i) + ".";
    std::vector<float> w;  // [Cin][Cout][k]
    if (tm.has(pre + "weight_v")) {
      // legacy torch.nn.utils.weight_norm(dim=0): w = g * v / ||v|| per input channel
      const tts_tensor_desc& v = tm.get(pre + "weight_v", {u.Cin, u.Cout, u.k});
      const tts_tensor_desc& g = tm.get(pre + "weight_g", {u.Cin, 1, 1});
      const float* vp = (const float*)v.data;
      const float* gp = (const float*)g.data;
      w.resize((size_t)u.Cin * u.Cout * u.k);
      const size_t sl = (size_t)u.Cout * u.k;
      for (int a = 0; a < u.Cin; ++a) {
        double ss = 0;
        for (size_t j = 0; j < sl; ++j) ss += (double)vp[a * sl + j] * vp[a * sl + j];
        const float sc = gp[a] / (float)sqrt(ss);
        for (size_t j = 0; j < sl; ++j) w[a * sl + j] = vp[a * sl + j] * sc;
      }
    } else {
      w = copy_of(tm.get(pre + "weight", {u.Cin, u.Cout, u.k}));
    }
    std::vector<float> wz((size_t)u.k * u.Cout * u.Cin);  // [j*Cout + co][ci]
    for (int a = 0; a < u.Cin; ++a)
      for (int co = 0; co < u.Cout; ++co)
        for (int j = 0; j < u.k; ++j)
          wz[((size_t)j * u.Cout + co) * u.Cin + a] = w[((size_t)a * u.Cout + co) * u.k + j];
    put(&u.wz, std::move(wz));
    put(&u.bias, copy_of(tm.get(pre + "bias", {u.Cout})));
    resblock(u.rb, "upsampler.resnet_blocks." + std::to_string(i) + ".", u.Cout);
    C = u.Cout;
  }
  if (c.n_upsample > 0) {
    put(&cd->out_w, copy_of(tm.get("upsampler.out_proj.weight", {D, C})));
    put(&cd->out_b, copy_of(tm.get("upsampler.out_proj.bias", {D})));
  }
  // ---- ISTFT head and its irfft basis
  const int nfft = 4 * c.hop_length;  // Generator: n_fft = hop_length * 4
  const int nb = nfft / 2 + 1;
  const int ldh = (2 * nb + 63) & ~63;  // K of the basis GEMM: a multiple of its K step
  cd->nfft = nfft; cd->nb = nb; cd->ldh = ldh;
  {
    const tts_tensor_desc& hw = tm.get("decoder.head.out.weight", {nfft + 2, D});
    const tts_tensor_desc& hb = tm.get("decoder.head.out.bias", {nfft + 2});
    std::vector<float> w((size_t)ldh * D, 0.f), b(ldh, 0.f);
    memcpy(w.data(), hw.data, sizeof(float) * (nfft + 2) * D);
    memcpy(b.data(), hb.data, sizeof(float) * (nfft + 2));
    put(&cd->head_w, std::move(w));
    put(&cd->head_b, std::move(b));
  }
  std::vector<float> win(nfft);
  if (tm.has("decoder.head.istft.window")) {
    const tts_tensor_desc& wd = tm.get("decoder.head.istft.window", {nfft});
    memcpy(win.data(), wd.data, sizeof(float) * nfft);
  } else {  // torch.hann_window(n) (periodic)
    for (int i = 0; i < nfft; ++i) win[i] = (float)(0.5 - 0.5 * cos(2.0 * M_PI * i / nfft));
  }
  {
    // frames[f][n] = w[n]/N * (Re0 + (-1)^n Re_{N/2} + 2 sum_k Re_k cos - Im_k sin)
    // (torch.fft.irfft, norm="backward"; imaginary parts of DC and Nyquist are ignored)
    std::vector<float> bm((size_t)nfft * ldh, 0.f);
    for (int nn = 0; nn < nfft; ++nn)
      for (int k = 0; k < nb; ++k) {
        const double ang = 2.0 * M_PI * (double)k * nn / nfft;
        const double wgt = (k == 0 || k == nfft / 2) ? 1.0 : 2.0;
        bm[(size_t)nn * ldh + k] = (float)(win[nn] * wgt * cos(ang) / nfft);
        bm[(size_t)nn * ldh + nb + k] =
            (k == 0 || k == nfft / 2) ? 0.f : (float)(-win[nn] * 2.0 * sin(ang) / nfft);
      }
    put(&cd->basis, std::move(bm));
  }
  put(&cd->window, std::move(win));

  // ---- upload
  cd->weights.alloc(slab.size * sizeof(float));
  for (auto& p : slab.parts)
    HIP_CHECK(hipMemcpy(cd->weights.as<float>() + p.first, p.second.data(),
                        p.second.size() * sizeof(float), hipMemcpyHostToDevice));
  for (auto& f : fixes) *f.dst = cd->weights.as<float>() + f.off;

  // ---- the GEMM weights' bf16x3 planes (the kernel would otherwise split every weight
  // tile again in every workgroup of every launch)
  {
    std::vector<std::pair<const float*, size_t>> bw = {{cd->fc_w, (size_t)D * VQ}, {cd->emb_w, (size_t)D * 7 * D}};
    auto rbw = [&](const CodecResBlock& rb) {
      bw.push_back({rb.c1w, (size_t)rb.C * 3 * rb.C});
      bw.push_back({rb.c2w, (size_t)rb.C * 3 * rb.C});
    };
    for (int i = 0; i < 2; ++i) { rbw(cd->prior[i]); rbw(cd->post[i]); }
    for (auto& b : cd->tf) {
      bw.push_back({b.c_attn, (size_t)3 * D * D});
      bw.push_back({b.c_proj, (size_t)D * D});
      bw.push_back({b.fc1, (size_t)4 * D * D});
      bw.push_back({b.fc2, (size_t)4 * D * D});
    }
    for (auto& u : cd->ups) {
      bw.push_back({u.wz, (size_t)u.k * u.Cout * u.Cin});
      rbw(u.rb);
    }
    if (cd->out_w) bw.push_back({cd->out_w, (size_t)D * C});
    bw.push_back({cd->head_w, (size_t)cd->ldh * D});
    bw.push_back({cd->basis, (size_t)nfft * cd->ldh});
    size_t tot = 0;
    for (auto& w : bw) tot += (3 * w.second + 127) & ~(size_t)127;
    cd->planes.alloc(tot * 2);
    size_t off = 0;
    for (auto& w : bw) {
      uint16_t* p = cd->planes.as<uint16_t>() + off;
      launch_split_planes(w.first, p, (long long)w.second, nullptr);
      cd->bplanes[w.first] = p;
      off += (3 * w.second + 127) & ~(size_t)127;
    }
    cd->rope_cs.alloc((size_t)c.heads * (c.hidden_dim / c.heads / 2) * 2 * 4);
    launch_codec_rope_table(cd->rope_cs.as<float>(), c.heads, nullptr);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipDeviceSynchronize());
  }

  cd->cap_T = c.max_codes;
  if (e->codec) codec_destroy(e->codec);
  e->codec = cd.release();
}

namespace {

thread_local Codec* t_codec = nullptr;  // the codec whose pass is being enqueued

void gemm(const float* A, int M, int K, int lda, const float* B, int N, const float* bias,
          float* C, int ldc, const float* resid, int act, hipStream_t s) {
  GemmF32Args g;
  g.A = A; g.M = M; g.K = K; g.lda = lda; g.B = B; g.N = N; g.bias = bias;
  auto it = t_codec->bplanes.find(B);
  if (it != t_codec->bplanes.end()) g.Bp = it->second;
  g.C = C; g.ldc = ldc; g.resid = resid; g.act = act;
  launch_gemm_f32(g, s);
}

// The same GEMM with A given as bf16 planes written by its producer (Ap: the planes image of
// A's first element, plane stride ap_plane) and optionally the output as planes too (Cp):
// gemm_x3p, no split in the GEMM (codec_gemm.hip)
void gemm_p(const uint16_t* Ap, long long ap_plane, int M, int K, int lda, const float* B, int N, const float* bias,
            float* C, int ldc, const float* resid, int act, hipStream_t s, uint16_t* Cp = nullptr,
            long long cp_plane = 0) {
  GemmF32Args g;
  g.Ap = Ap; g.ap_plane = ap_plane;
  g.M = M; g.K = K; g.lda = lda; g.B = B; g.N = N; g.bias = bias;
  auto it = t_codec->bplanes.find(B);
  TTS_REQUIRE(it != t_codec->bplanes.end(), "codec: weight planes missing");
  g.Bp = it->second;
  g.C = C; g.ldc = ldc; g.resid = resid; g.act = act;
  g.Cp = Cp; g.cp_plane = cp_plane;
  launch_gemm_x3p(g, s);
}

// TTS_CODEC_X3P=0: the fp32-staging GEMM (gemm_bx3_kernel splits A while staging) everywhere.
// TTS_CODEC_BX3=0 (plain fp32 MFMA for every contraction, a debugging switch) turns the
// split-bf16 x3p path off as well
bool use_x3p() {
  static const bool v = !(getenv("TTS_CODEC_X3P") && !atoi(getenv("TTS_CODEC_X3P"))) &&
                        !(getenv("TTS_CODEC_BX3") && !atoi(getenv("TTS_CODEC_BX3")));
  return v;
}

// The utterances of one pass at one time resolution: segment table (device), padded rows.
struct Level {
  const CodecSeg* seg = nullptr;
  int rows = 0;   // padded rows of the buffer (kPad + sum (T + kPad))
  int M = 0;      // GEMM rows: rows - 2 kPad (every utterance and the gaps between them)
  int max_T = 0;
};

// ResnetBlock (decoder_modules.py:162-223) on ragged time-major buffers: x -> out, tmp is
// scratch (its gap rows are the convs' zero padding, written by groupnorm_swish).
void resnet(const CodecResBlock& rb, float* x, float* tmp, float* out, const Level& lv, int B,
            float* stats, hipStream_t s, uint16_t* tmpp = nullptr, long long tplane = 0) {
  const int C = rb.C;
  float* xr = x + (size_t)kPad * C;
  float* tr = tmp + (size_t)kPad * C;
  float* orow = out + (size_t)kPad * C;
  // (tmpp: GroupNorm + swish write tmp's planes, the convs read them with gemm_x3p)
  const bool xp = tmpp != nullptr && (3 * C) % 32 == 0 && C % 8 == 0;
  const uint16_t* tw = xp ? tmpp + (size_t)(kPad - 1) * C : nullptr;  // the window one row above
  launch_groupnorm_stats(x, lv.seg, B, C, 32, 1e-6f, stats, s);
  launch_groupnorm_swish(x, lv.seg, B, lv.max_T, C, 32, stats, rb.n1w, rb.n1b, tmp, s, xp ? tmpp : nullptr, tplane);
  // conv1 (k=3, pad=1): sliding window starting one row above
  if (xp) gemm_p(tw, tplane, lv.M, 3 * C, C, rb.c1w, C, rb.c1b, orow, C, nullptr, 0, s);
  else gemm(tr - C, lv.M, 3 * C, C, rb.c1w, C, rb.c1b, orow, C, nullptr, 0, s);
  launch_groupnorm_stats(out, lv.seg, B, C, 32, 1e-6f, stats, s);
  launch_groupnorm_swish(out, lv.seg, B, lv.max_T, C, 32, stats, rb.n2w, rb.n2b, tmp, s, xp ? tmpp : nullptr,
                         tplane);
  if (xp) gemm_p(tw, tplane, lv.M, 3 * C, C, rb.c2w, C, rb.c2b, orow, C, xr, 0, s);  // x + h
  else gemm(tr - C, lv.M, 3 * C, C, rb.c2w, C, rb.c2b, orow, C, xr, 0, s);
}

void grow(DevBuf& b, size_t bytes) {
  if (b.bytes < bytes) b.alloc(bytes);
}

}  // namespace

// Decoder.forward (decoder.py:69-89) of B utterances in one ragged pass: codes_dev = their
// codes back to back (device), lens[b] codes each -> their waveforms back to back at wav_dev.
static void decode_pass(Codec& cd, const int* codes_dev, const int32_t* lens, int B, float* wav_dev,
                        hipStream_t s) {
  const tts_codec_config& c = cd.cfg;
  const int D = c.hidden_dim, H = c.heads, VQ = c.vq_dim;
  const int NU = (int)cd.ups.size();
  // ---- segment tables of every time resolution, wave offsets, code rows, query blocks
  std::vector<std::vector<CodecSeg>> seg(NU + 1, std::vector<CodecSeg>(B));
  std::vector<Level> lv(NU + 1);
  for (int i = 0; i <= NU; ++i) {
    int row = kPad, mx = 0;
    for (int b = 0; b < B; ++b) {
      int T = lens[b];
      for (int j = 0; j < i; ++j) T *= cd.ups[j].u;
      seg[i][b] = {T, row};
      row += T + kPad;
      mx = std::max(mx, T);
    }
    lv[i].rows = row;
    lv[i].M = row - 2 * kPad;
    lv[i].max_T = mx;
  }
  std::vector<long long> wav_off(B);
  std::vector<int> code_row;
  std::vector<int2> qblk;
  long long w = 0;
  for (int b = 0; b < B; ++b) {
    wav_off[b] = w;
    w += (long long)seg[NU][b].T * c.hop_length;
    for (int t = 0; t < lens[b]; ++t) code_row.push_back(seg[0][b].row + t);
    for (int q = 0; q < codec_attn_qblocks(lens[b]); ++q) qblk.push_back(make_int2(b, q * codec_attn_qrows()));
  }
  std::vector<char> host;
  auto put = [&](const void* p, size_t n) {
    const size_t off = host.size();
    host.resize((off + n + 255) & ~(size_t)255);
    memcpy(host.data() + off, p, n);
    return off;
  };
  std::vector<size_t> seg_off(NU + 1);
  for (int i = 0; i <= NU; ++i) seg_off[i] = put(seg[i].data(), sizeof(CodecSeg) * B);
  const size_t wav_o = put(wav_off.data(), sizeof(long long) * B);
  const size_t row_o = put(code_row.data(), sizeof(int) * code_row.size());
  const size_t qb_o = put(qblk.data(), sizeof(int2) * qblk.size());
  grow(cd.meta, host.size());
  HIP_CHECK(hipMemcpyAsync(cd.meta.p, host.data(), host.size(), hipMemcpyHostToDevice, s));
  char* mb = cd.meta.as<char>();
  for (int i = 0; i <= NU; ++i) lv[i].seg = (const CodecSeg*)(mb + seg_off[i]);

  // ---- workspace of this pass
  int max_rows = 0;
  for (auto& l : lv) max_rows = std::max(max_rows, l.rows);
  const Level& L0 = lv[0];
  const Level& LF = lv[NU];
  size_t big = std::max((size_t)L0.rows * 4 * D, (size_t)L0.rows * VQ);
  for (int i = 0; i < NU; ++i) big = std::max(big, (size_t)lv[i].rows * cd.ups[i].k * cd.ups[i].Cout);
  grow(cd.b0, (size_t)max_rows * D * 4);
  grow(cd.b1, (size_t)max_rows * D * 4);
  grow(cd.b2, (size_t)max_rows * D * 4);
  grow(cd.big, big * 4);
  grow(cd.qkv, (size_t)L0.rows * 3 * D * 4);
  grow(cd.stats, (size_t)B * 32 * 2 * 4);
  grow(cd.head, (size_t)LF.rows * cd.ldh * 4);
  grow(cd.spec, (size_t)LF.rows * cd.ldh * 4);
  grow(cd.frames, (size_t)LF.rows * cd.nfft * 4);
  const bool xp = use_x3p();
  const long long p2 = (long long)max_rows * D, pbig = (long long)L0.rows * 4 * D;  // plane strides
  if (xp) {
    grow(cd.b2p, (size_t)p2 * 3 * 2);
    grow(cd.bigpp, (size_t)pbig * 3 * 2);
  }
  uint16_t* b2p = xp ? cd.b2p.as<uint16_t>() : nullptr;
  uint16_t* bigpp = xp ? cd.bigpp.as<uint16_t>() : nullptr;
  auto RP = [&](uint16_t* buf, int C) { return buf + (size_t)kPad * C; };

  t_codec = &cd;
  float* b0 = cd.b0.as<float>();
  float* b1 = cd.b1.as<float>();
  float* b2 = cd.b2.as<float>();
  float* bigp = cd.big.as<float>();
  float* stats = cd.stats.as<float>();
  auto R = [&](float* buf, int C) { return buf + (size_t)kPad * C; };
  // FSQ -> project_out -> fc_post_a; the embed conv reads zero gaps
  launch_fsq_project(codes_dev, (const int*)(mb + row_o), (int)code_row.size(), cd.po_w, cd.po_b, bigp, VQ, s);
  if (xp) {  // fc_post_a writes the embed conv's planes (b2p holds them until the first resnet)
    GemmF32Args g;
    g.A = R(bigp, VQ); g.M = L0.M; g.K = VQ; g.lda = VQ; g.B = cd.fc_w; g.N = D; g.bias = cd.fc_b;
    g.Bp = cd.bplanes.at(cd.fc_w);
    g.C = nullptr; g.ldc = D; g.Cp = RP(b2p, D); g.cp_plane = p2;
    launch_gemm_f32(g, s);
    launch_zero_gaps(nullptr, D, L0.seg, B, s, b2p, p2);
    gemm_p(RP(b2p, D) - 3 * D, p2, L0.M, 7 * D, D, cd.emb_w, D, cd.emb_b, R(b1, D), D, nullptr, 0, s);
  } else {
    gemm(R(bigp, VQ), L0.M, VQ, VQ, cd.fc_w, D, cd.fc_b, R(b0, D), D, nullptr, 0, s);
    launch_zero_gaps(b0, D, L0.seg, B, s);
    // embed Conv1d(k=7, pad=3): window starts 3 rows above
    gemm(R(b0, D) - 3 * D, L0.M, 7 * D, D, cd.emb_w, D, cd.emb_b, R(b1, D), D, nullptr, 0, s);
  }
  // prior_net: b1 -> b0 -> b1
  resnet(cd.prior[0], b1, b2, b0, L0, B, stats, s, b2p, p2);
  resnet(cd.prior[1], b0, b2, b1, L0, B, stats, s, b2p, p2);
  // transformers on x = b1 (in place residual stream), scratch b2 / big / qkv
  float* x = R(b1, D);
  float* qkv = cd.qkv.as<float>();
  for (int l = 0; l < c.depth && xp; ++l) {
    // the planes form: every GEMM input written as planes by its producer (gemm_x3p)
    const CodecTfBlock& tb = cd.tf[l];
    launch_rmsnorm_f32(x, L0.M, D, tb.att_norm, 1e-6f, nullptr, s, RP(b2p, D), p2);
    gemm_p(RP(b2p, D), p2, L0.M, D, D, tb.c_attn, 3 * D, nullptr, R(qkv, 3 * D), 3 * D, nullptr, 0, s);
    launch_codec_attention(qkv, L0.seg, (const int2*)(mb + qb_o), (int)qblk.size(), H, D / H, cd.rope_cs.as<float>(),
                           b2, s, b2p, p2);
    gemm_p(RP(b2p, D), p2, L0.M, D, D, tb.c_proj, D, nullptr, x, D, x, 0, s);
    launch_rmsnorm_f32(x, L0.M, D, tb.ffn_norm, 1e-6f, nullptr, s, RP(b2p, D), p2);
    gemm_p(RP(b2p, D), p2, L0.M, D, D, tb.fc1, 4 * D, nullptr, nullptr, 4 * D, nullptr, 1, s, RP(bigpp, 4 * D), pbig);
    gemm_p(RP(bigpp, 4 * D), pbig, L0.M, 4 * D, 4 * D, tb.fc2, D, nullptr, x, D, x, 0, s);
  }
  for (int l = 0; l < c.depth && !xp; ++l) {
    const CodecTfBlock& tb = cd.tf[l];
    launch_rmsnorm_f32(x, L0.M, D, tb.att_norm, 1e-6f, R(b2, D), s);
    gemm(R(b2, D), L0.M, D, D, tb.c_attn, 3 * D, nullptr, R(qkv, 3 * D), 3 * D, nullptr, 0, s);
    // (RoPE of q and k runs inside the attention kernel's staging)
    launch_codec_attention(qkv, L0.seg, (const int2*)(mb + qb_o), (int)qblk.size(), H, D / H, cd.rope_cs.as<float>(),
                           b2, s);
    gemm(R(b2, D), L0.M, D, D, tb.c_proj, D, nullptr, x, D, x, 0, s);
    launch_rmsnorm_f32(x, L0.M, D, tb.ffn_norm, 1e-6f, R(b2, D), s);
    gemm(R(b2, D), L0.M, D, D, tb.fc1, 4 * D, nullptr, R(bigp, 4 * D), 4 * D, nullptr, 1, s);
    gemm(R(bigp, 4 * D), L0.M, 4 * D, 4 * D, tb.fc2, D, nullptr, x, D, x, 0, s);
  }
  // post_net: b1 -> b0 -> b1
  resnet(cd.post[0], b1, b2, b0, L0, B, stats, s, b2p, p2);
  resnet(cd.post[1], b0, b2, b1, L0, B, stats, s, b2p, p2);
  launch_layernorm_f32(R(b1, D), L0.M, D, cd.ln_w, cd.ln_b, 1e-6f, R(b0, D), s);
  float* hid = R(b0, D);
  int C = D;
  float* cur = b0;
  for (int i = 0; i < NU; ++i) {
    const CodecUp& u = cd.ups[i];
    // ConvTranspose1d as Z = x . Wz^T (every tap of every input frame), then a gather
    gemm(R(cur, C), lv[i].M, u.Cin, u.Cin, u.wz, u.k * u.Cout, nullptr, R(bigp, u.k * u.Cout), u.k * u.Cout,
         nullptr, 0, s);
    float* nxt = (cur == b0) ? b1 : b0;
    launch_convt_gather(bigp, lv[i].seg, lv[i + 1].seg, B, lv[i + 1].max_T, u.Cout, u.k, u.u, u.pad, u.bias, nxt, s);
    C = u.Cout;
    float* res_out = (nxt == b0) ? b1 : b0;
    resnet(u.rb, nxt, b2, res_out, lv[i + 1], B, stats, s, b2p, p2);
    cur = res_out;
  }
  if (NU > 0) {
    float* dst = (cur == b0) ? b1 : b0;
    gemm(R(cur, C), LF.M, C, C, cd.out_w, D, cd.out_b, R(dst, D), D, nullptr, 1, s);
    hid = R(dst, D);
  }
  // ISTFT head
  float* head = cd.head.as<float>();
  float* spec = cd.spec.as<float>();
  float* frames = cd.frames.as<float>();
  gemm(hid, LF.M, D, D, cd.head_w, cd.ldh, cd.head_b, R(head, cd.ldh), cd.ldh, nullptr, 0, s);
  launch_istft_spec(R(head, cd.ldh), LF.M, cd.nb, cd.ldh, R(spec, cd.ldh), s);
  gemm(R(spec, cd.ldh), LF.M, cd.ldh, cd.ldh, cd.basis, cd.nfft, nullptr, R(frames, cd.nfft), cd.nfft, nullptr, 0,
       s);
  launch_ola(frames, LF.seg, (const long long*)(mb + wav_o), B, LF.max_T, cd.nfft, c.hop_length, cd.window, wav_dev,
             s);
  HIP_CHECK(hipGetLastError());
  // the host tables must outlive their upload
  HIP_CHECK(hipStreamSynchronize(s));
}

void codec_decode(Engine* e, const int32_t* codes, const int32_t* lens, int B, float* wav,
                  int wav_is_device, int64_t* wav_lens, hipStream_t s) {
  TTS_REQUIRE(e->codec != nullptr, "tts_codec_load has not been called");
  Codec& cd = *e->codec;
  const tts_codec_config& c = cd.cfg;
  int ups = 1;
  for (int i = 0; i < c.n_upsample; ++i) ups *= c.upsample_factors[i];
  // ---- validate everything before any launch; one upload of all codes
  size_t n_codes = 0, n_wav = 0;
  for (int b = 0; b < B; ++b) {
    const int T = lens[b];
    TTS_REQUIRE(T >= 1 && T <= cd.cap_T, "utterance length out of range (max_codes)");
    for (int i = 0; i < T; ++i)
      TTS_REQUIRE(codes[n_codes + i] >= 0 && codes[n_codes + i] < 65536, "code out of range");
    n_codes += T;
    n_wav += (size_t)T * ups * c.hop_length;
  }
  if (cd.codes.bytes < n_codes * 4) cd.codes.alloc(n_codes * 4);
  if (!wav_is_device && cd.wav.bytes < n_wav * 4) cd.wav.alloc(n_wav * 4);
  HIP_CHECK(hipMemcpyAsync(cd.codes.p, codes, n_codes * 4, hipMemcpyHostToDevice, s));
  float* wav_dev = wav_is_device ? wav : cd.wav.as<float>();
  // passes of at most kPassCodes codes (the workspace grows with a pass: ~90 KB per code
  // at 24 kHz); one utterance longer than that is a pass of its own
  static const long long kPassCodes =
      getenv("TTS_CODEC_PASS_CODES") ? atoll(getenv("TTS_CODEC_PASS_CODES")) : 32768;
  size_t off_codes = 0, off_wav = 0;
  for (int b0 = 0; b0 < B;) {
    int b1 = b0;
    long long n = 0;
    while (b1 < B && (b1 == b0 || n + lens[b1] <= kPassCodes)) n += lens[b1++];
    decode_pass(cd, cd.codes.as<int>() + off_codes, lens + b0, b1 - b0, wav_dev + off_wav, s);
    for (int b = b0; b < b1; ++b) {
      wav_lens[b] = (int64_t)lens[b] * ups * c.hop_length;
      off_wav += (size_t)wav_lens[b];
    }
    off_codes += (size_t)n;
    b0 = b1;
  }
  if (!wav_is_device) HIP_CHECK(hipMemcpyAsync(wav, wav_dev, n_wav * 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (getenv("TTS_CODEC_STAMPS")) x3p_stamps_dump(stderr);  // (stamps build only)
}

}  // namespace tts
