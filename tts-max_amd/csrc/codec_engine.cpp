// codec_engine.cpp — codec decoder host runtime: weight loading (weight-norm fold, conv
// re-layout, iDFT basis), workspaces, and the Decoder.forward launch sequence.
//
// Reference: tts/core/codec/decoder.py:69-89 (Decoder.forward), decoding.py:84-89
// (AudioDecoder.decode), decoder_modules.py (Generator / VocosBackbone / ISTFTHead),
// upsampler.py (UpSamplerBlock).  The reference decodes one utterance per call in fp32.
// GroupNorm statistics and the unmasked attention span a whole utterance, so utterances
// are never padded together: a batch is spread over kLanes streams,
// each with its own workspace, and the utterances of different lanes run concurrently
// (each one alone is far too small to fill 256 CUs).
#include <math.h>
#include <string.h>

#include <algorithm>
#include <memory>

#include "codec_kernels.h"
#include "engine.h"

namespace tts {

static constexpr int kPad = 3;  // zero rows before/after every time-major activation

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
  int cap_T = 0, cap_F = 0;
  // per-lane workspaces + streams
  struct Lane {
    DevBuf b0, b1, b2, big, qkv, stats, head, spec, frames;
    DevBuf gcodes, gwav;  // fixed input / output of the lane's captured graphs
    DevBuf kpart;         // split-K GEMM partials
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr;
    std::map<int, hipGraphExec_t> graphs;  // one captured decode per utterance length
    ~Lane() {
      for (auto& g : graphs) (void)hipGraphExecDestroy(g.second);
      if (done) (void)hipEventDestroy(done);
      if (st) (void)hipStreamDestroy(st);
    }
  };
  std::vector<std::unique_ptr<Lane>> lanes;
  hipEvent_t start = nullptr;
  DevBuf codes, wav;  // all utterances' codes; host-bound waveforms staged on the device
  ~Codec() {
    if (start) (void)hipEventDestroy(start);
  }
};

static constexpr int kLanes = 4;  // = the HIP hardware queues per process (GPU_MAX_HW_QUEUES)
static constexpr size_t kSplitElems = (size_t)4 << 20;  // split-K partial floats per lane
// workspace of the lane whose launch sequence is being enqueued (decode_one)
static thread_local float* t_split_ws = nullptr;

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

  // ---- workspaces
  const int Tm = c.max_codes;
  const int Fm = Tm * ups;
  cd->cap_T = Tm;
  cd->cap_F = Fm;
  const size_t rows = (size_t)Fm + 2 * kPad;
  size_t big = std::max((size_t)Tm * 4 * D, (size_t)Tm * VQ);
  {  // ConvTranspose GEMM output Z = [Tc][k*Cout] at each stage's input length
    int Tc = Tm;
    for (auto& u : cd->ups) {
      big = std::max(big, (size_t)Tc * u.k * u.Cout);
      Tc *= u.u;
    }
  }
  for (int l = 0; l < kLanes; ++l) {
    auto ln = std::make_unique<Codec::Lane>();
    ln->b0.alloc(rows * D * 4);
    ln->b1.alloc(rows * D * 4);
    ln->b2.alloc(rows * D * 4);
    ln->big.alloc(big * 4);
    ln->qkv.alloc((size_t)Tm * 3 * D * 4);
    ln->stats.alloc(64 * 2 * 4);
    ln->head.alloc((size_t)Fm * ldh * 4);
    ln->spec.alloc((size_t)Fm * ldh * 4);
    ln->frames.alloc((size_t)Fm * nfft * 4);
    ln->gcodes.alloc((size_t)Tm * 4);
    ln->kpart.alloc(kSplitElems * 4);
    ln->gwav.alloc((size_t)Fm * c.hop_length * 4);
    HIP_CHECK(hipStreamCreateWithFlags(&ln->st, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&ln->done, hipEventDisableTiming));
    cd->lanes.push_back(std::move(ln));
  }
  HIP_CHECK(hipEventCreateWithFlags(&cd->start, hipEventDisableTiming));
  if (e->codec) codec_destroy(e->codec);
  e->codec = cd.release();
}

namespace {

void gemm(const float* A, int M, int K, int lda, const float* B, int N, const float* bias,
          float* C, int ldc, const float* resid, int act, hipStream_t s) {
  GemmF32Args g;
  g.A = A; g.M = M; g.K = K; g.lda = lda; g.B = B; g.N = N; g.bias = bias;
  g.C = C; g.ldc = ldc; g.resid = resid; g.act = act;
  g.part = t_split_ws; g.part_elems = t_split_ws ? kSplitElems : 0;
  launch_gemm_f32(g, s);
}

// ResnetBlock (decoder_modules.py:162-223) on a padded time-major buffer x (T rows of C at
// row kPad); tmp is a padded scratch buffer; result written to out (padded, may alias none).
void resnet(const CodecResBlock& rb, float* x, float* tmp, float* out, int T, float* stats,
            hipStream_t s) {
  const int C = rb.C;
  float* xr = x + (size_t)kPad * C;
  float* tr = tmp + (size_t)kPad * C;
  float* orow = out + (size_t)kPad * C;
  launch_groupnorm_stats(xr, T, C, 32, 1e-6f, stats, s);
  launch_groupnorm_swish(xr, T, C, 32, stats, rb.n1w, rb.n1b, tr, s);
  // conv1 (k=3, pad=1): sliding window starting one row above
  gemm(tr - C, T, 3 * C, C, rb.c1w, C, rb.c1b, orow, C, nullptr, 0, s);
  launch_groupnorm_stats(orow, T, C, 32, 1e-6f, stats, s);
  launch_groupnorm_swish(orow, T, C, 32, stats, rb.n2w, rb.n2b, tr, s);
  gemm(tr - C, T, 3 * C, C, rb.c2w, C, rb.c2b, orow, C, xr, 0, s);  // x + h
}

}  // namespace

// The whole Decoder.forward launch sequence of one utterance of T codes on lane `ln`
// (stream `ls`): codes_in [T] int32 (device) -> wav_out [T * samples_per_code] f32 (device).
static void decode_one(Codec& cd, Codec::Lane& ln, int T, const int* codes_in, float* wav_out,
                       hipStream_t ls) {
  const tts_codec_config& c = cd.cfg;
  const int D = c.hidden_dim, H = c.heads, VQ = c.vq_dim;
  int ups = 1;
  for (int i = 0; i < c.n_upsample; ++i) ups *= c.upsample_factors[i];
  t_split_ws = ln.kpart.as<float>();
    const int F = T * ups;
    const size_t rows_cap = (size_t)cd.cap_F + 2 * kPad;
    // zero the padding rows (and everything else) of the three activation buffers
    launch_zero(ln.b0.as<float>(), (long long)rows_cap * D, ls);
    launch_zero(ln.b1.as<float>(), (long long)rows_cap * D, ls);
    launch_zero(ln.b2.as<float>(), (long long)rows_cap * D, ls);
    float* big = ln.big.as<float>();
    float* b0 = ln.b0.as<float>();
    float* b1 = ln.b1.as<float>();
    float* b2 = ln.b2.as<float>();
    float* stats = ln.stats.as<float>();
    auto R = [&](float* buf, int C) { return buf + (size_t)kPad * C; };
    // FSQ -> project_out -> fc_post_a
    launch_fsq_project(codes_in, T, cd.po_w, cd.po_b, big, VQ, ls);
    gemm(big, T, VQ, VQ, cd.fc_w, D, cd.fc_b, R(b0, D), D, nullptr, 0, ls);
    // embed Conv1d(k=7, pad=3): window starts 3 rows above
    gemm(R(b0, D) - 3 * D, T, 7 * D, D, cd.emb_w, D, cd.emb_b, R(b1, D), D, nullptr, 0, ls);
    // prior_net: b1 -> b0 -> b1
    resnet(cd.prior[0], b1, b2, b0, T, stats, ls);
    resnet(cd.prior[1], b0, b2, b1, T, stats, ls);
    // transformers on x = b1 (in place residual stream), scratch b2 / big / qkv
    float* x = R(b1, D);
    float* qkv = ln.qkv.as<float>();
    for (int l = 0; l < c.depth; ++l) {
      const CodecTfBlock& tb = cd.tf[l];
      launch_rmsnorm_f32(x, T, D, tb.att_norm, 1e-6f, R(b2, D), ls);
      gemm(R(b2, D), T, D, D, tb.c_attn, 3 * D, nullptr, qkv, 3 * D, nullptr, 0, ls);
      launch_codec_rope(qkv, T, H, D / H, ls);
      launch_codec_attention(qkv, T, H, D / H, R(b2, D), ls);
      gemm(R(b2, D), T, D, D, tb.c_proj, D, nullptr, x, D, x, 0, ls);
      launch_rmsnorm_f32(x, T, D, tb.ffn_norm, 1e-6f, R(b2, D), ls);
      gemm(R(b2, D), T, D, D, tb.fc1, 4 * D, nullptr, big, 4 * D, nullptr, 1, ls);
      gemm(big, T, 4 * D, 4 * D, tb.fc2, D, nullptr, x, D, x, 0, ls);
    }
    // post_net: b1 -> b0 -> b1
    resnet(cd.post[0], b1, b2, b0, T, stats, ls);
    resnet(cd.post[1], b0, b2, b1, T, stats, ls);
    launch_layernorm_f32(R(b1, D), T, D, cd.ln_w, cd.ln_b, 1e-6f, R(b0, D), ls);
    float* hid = R(b0, D);  // [T][D]
    int Tc = T, C = D;
    float* cur = b0;
    for (size_t i = 0; i < cd.ups.size(); ++i) {
      const CodecUp& u = cd.ups[i];
      gemm(R(cur, C), Tc, u.Cin, u.Cin, u.wz, u.k * u.Cout, nullptr, big, u.k * u.Cout, nullptr, 0, ls);
      float* nxt = (cur == b0) ? b1 : b0;
      // clear stale rows of the destination so the padding below is zero again
      launch_zero(nxt, (long long)rows_cap * D, ls);
      launch_convt_gather(big, Tc, u.Cout, u.k, u.u, u.pad, u.bias, R(nxt, u.Cout), ls);
      Tc *= u.u;
      C = u.Cout;
      launch_zero(b2, (long long)rows_cap * D, ls);
      float* res_out = (nxt == b0) ? b1 : b0;
      launch_zero(res_out, (long long)rows_cap * D, ls);
      resnet(u.rb, nxt, b2, res_out, Tc, stats, ls);
      cur = res_out;
    }
    if (!cd.ups.empty()) {
      float* dst = (cur == b0) ? b1 : b0;
      gemm(R(cur, C), Tc, C, C, cd.out_w, D, cd.out_b, R(dst, D), D, nullptr, 1, ls);
      hid = R(dst, D);
    }
    // ISTFT head
    gemm(hid, F, D, D, cd.head_w, cd.ldh, cd.head_b, ln.head.as<float>(), cd.ldh, nullptr, 0, ls);
    launch_istft_spec(ln.head.as<float>(), F, cd.nb, cd.ldh, ln.spec.as<float>(), ls);
    gemm(ln.spec.as<float>(), F, cd.ldh, cd.ldh, cd.basis, cd.nfft, nullptr, ln.frames.as<float>(),
         cd.nfft, nullptr, 0, ls);
    launch_ola(ln.frames.as<float>(), F, cd.nfft, c.hop_length, cd.window, wav_out, ls);
  HIP_CHECK(hipGetLastError());
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
  const int NL = std::min(B, kLanes);
  HIP_CHECK(hipEventRecord(cd.start, s));
  for (int l = 0; l < NL; ++l) HIP_CHECK(hipStreamWaitEvent(cd.lanes[l]->st, cd.start, 0));

  // Each utterance replays its lane's graph for that length (captured on first use): ~150
  // launches become one, which is what makes short streaming windows cheap.  The graph
  // reads / writes the lane's fixed buffers; two device copies move codes and samples.
  size_t off_codes = 0, off_wav = 0;
  for (int b = 0; b < B; ++b) {
    Codec::Lane& ln = *cd.lanes[b % NL];
    const int T = lens[b];
    const size_t L = (size_t)T * ups * c.hop_length;
    auto it = ln.graphs.find(T);
    if (it == ln.graphs.end()) {
      if (ln.graphs.size() >= 32) {  // bounded cache: drop the smallest length
        (void)hipGraphExecDestroy(ln.graphs.begin()->second);
        ln.graphs.erase(ln.graphs.begin());
      }
      hipStream_t cs;
      HIP_CHECK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
      hipGraph_t g;
      HIP_CHECK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
      decode_one(cd, ln, T, ln.gcodes.as<int>(), ln.gwav.as<float>(), cs);
      HIP_CHECK(hipStreamEndCapture(cs, &g));
      hipGraphExec_t ge;
      HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      HIP_CHECK(hipGraphDestroy(g));
      HIP_CHECK(hipStreamDestroy(cs));
      it = ln.graphs.emplace(T, ge).first;
    }
    HIP_CHECK(hipMemcpyAsync(ln.gcodes.p, cd.codes.as<int>() + off_codes, (size_t)T * 4,
                             hipMemcpyDeviceToDevice, ln.st));
    HIP_CHECK(hipGraphLaunch(it->second, ln.st));
    HIP_CHECK(hipMemcpyAsync(wav_dev + off_wav, ln.gwav.p, L * 4, hipMemcpyDeviceToDevice, ln.st));
    wav_lens[b] = (int64_t)L;
    off_codes += T;
    off_wav += L;
  }
  // join the lanes back into the caller's stream
  for (int l = 0; l < NL; ++l) {
    HIP_CHECK(hipEventRecord(cd.lanes[l]->done, cd.lanes[l]->st));
    HIP_CHECK(hipStreamWaitEvent(s, cd.lanes[l]->done, 0));
  }
  if (!wav_is_device) HIP_CHECK(hipMemcpyAsync(wav, wav_dev, n_wav * 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace tts
