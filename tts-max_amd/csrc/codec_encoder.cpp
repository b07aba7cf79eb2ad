// codec_encoder.cpp — the prompt-audio encoder: the reference
// Encoder.encode (tts/core/codec/encoder.py:58-128) after the w2v-bert feature model, in
// fp32 on the device.  Time-major [T][C] buffers; every convolution is a GEMM over its
// windows (enc_im2col for k > 1) against the weight re-laid out tap-major [Cout][k*Cin]
// (weight norm folded at load), on the codec's fp32-exact split-bf16 GEMM.
//
//   wav (padded to a whole hop, + one more hop when already whole, as encode() does)
//   AcousticEncoder: Conv(1->48, k7) -> 5 x EncoderBlock(3 x ResidualUnit(dilation 1, 3, 9),
//     Activation1d, strided Conv) -> Activation1d -> Conv(1536 -> 1024, k3)       [T][1024]
//   SemanticEncoder on the w2v-bert layer-16 features: Conv k3 -> r = ReLU (in place: the skip
//     adds r) -> Conv k3 -> ReLU -> Conv k3 + r -> Conv k3                       [T][1024]
//   fusion Linear(2048) on [semantic | acoustic] -> project_in Linear(2048 -> 8) -> FSQ
#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "codec_kernels.h"
#include "enc_kernels.h"
#include "engine.h"

namespace tts {

namespace {

struct EncConv {
  int cin = 0, cout = 0, k = 1, stride = 1, dil = 1, pad = 0;
  int kk = 0;                  // GEMM K = k * cin rounded up to the fp32 GEMM's step of 16
  size_t w = 0, b = SIZE_MAX;  // offsets into the weight slab (b: none)
};
struct EncSnake { int C = 0; size_t a = 0, b = 0; };
struct EncRU { EncSnake s1, s2; EncConv c1, c2; };
struct EncBlock { EncRU ru[3]; EncSnake s; EncConv down; };
// one w2v-bert conformer layer (offsets into the weight slab; every Linear [out][in])
struct W2vLayer {
  size_t ffn_ln[2][2], ffn_w1[2], ffn_b1[2], ffn_w2[2], ffn_b2[2];  // w2 / b2 pre-scaled by 0.5
  size_t att_ln[2], qkv_w, qkv_b, out_w, out_b, dist;
  size_t conv_ln[2], pw1, dw, dw_ln[2], pw2;
  size_t fin_ln[2];
};

}  // namespace

struct AudioEncoder {
  EncConv c0, cf, sem_init, sem_c1, sem_c2, sem_final;
  EncBlock blk[5];
  EncSnake sf;
  size_t fus_w = 0, fus_b = 0, pin_w = 0, pin_b = 0, filt_up = 0, filt_dn = 0;
  int nblk = 5, S = 1024, A = 1024, nl = 8;
  DevBuf weights, planes, levels;
  std::map<const float*, const uint16_t*> bplanes;
  DevBuf x, y, z, win, sem, fused, proj, codes, pre;
  // w2v-bert-2.0 up to hidden_states[16] (optional: loaded when its tensors are given)
  bool w2v = false;
  int wH = 1024, wFF = 4096, wFin = 160, wHeads = 16, wL = 64, wR = 8, wK = 31, wLayers = 16;
  float wEps = 1e-5f;
  size_t fp_ln[2] = {0, 0}, fp_w = 0, fp_b = 0;
  std::vector<W2vLayer> wl;
  DevBuf wx, wln, wbig, wqkv, watt, wfeat;
  const float* W(size_t off) const { return weights.as<float>() + off; }
};

void encoder_destroy(AudioEncoder* a) { delete a; }

namespace {

struct Tensors {
  std::map<std::string, const tts_tensor_desc*> m;
  const tts_tensor_desc& get(const std::string& n, std::initializer_list<int64_t> shape) const {
    auto it = m.find(n);
    if (it == m.end()) throw Error(TTS_E_INVALID, "missing encoder tensor: " + n);
    const tts_tensor_desc& d = *it->second;
    bool ok = (int)shape.size() == d.ndim;
    int i = 0;
    for (int64_t v : shape) { if (ok && d.shape[i] != v) ok = false; ++i; }
    if (!ok) throw Error(TTS_E_INVALID, "bad shape for encoder tensor: " + n);
    TTS_REQUIRE(d.dtype == TTS_DT_F32 && !d.on_device, "encoder tensors must be host f32: " + n);
    return d;
  }
};

}  // namespace

void encoder_load(Engine* e, const tts_tensor_desc* t, int n) {
  Tensors tm;
  for (int i = 0; i < n; ++i) tm.m[t[i].name] = &t[i];
  std::unique_ptr<AudioEncoder> en(new AudioEncoder());
  std::vector<float> slab;
  auto put = [&](const float* p, size_t cnt) {
    const size_t off = slab.size();
    slab.insert(slab.end(), p, p + cnt);
    slab.resize((slab.size() + 63) & ~(size_t)63);  // 256-B aligned sub-buffers
    return off;
  };
  // Conv1d weight [co][ci][k] (optionally legacy weight_norm(dim=0): g * v / ||v||) ->
  // [co][k*ci] tap-major
  auto conv = [&](const std::string& pre, int ci, int co, int k, int stride, int dil, int pad, bool wnorm,
                  bool bias) {
    EncConv c;
    c.cin = ci; c.cout = co; c.k = k; c.stride = stride; c.dil = dil; c.pad = pad;
    c.kk = (k * ci + 15) / 16 * 16;
    std::vector<float> w((size_t)co * ci * k);
    if (wnorm) {
      const tts_tensor_desc& v = tm.get(pre + "weight_v", {co, ci, k});
      const tts_tensor_desc& g = tm.get(pre + "weight_g", {co, 1, 1});
      const float* vp = (const float*)v.data;
      const float* gp = (const float*)g.data;
      const size_t sl = (size_t)ci * k;
      for (int o = 0; o < co; ++o) {
        double ss = 0;
        for (size_t j = 0; j < sl; ++j) ss += (double)vp[o * sl + j] * vp[o * sl + j];
        const float sc = gp[o] / (float)std::sqrt(ss);
        for (size_t j = 0; j < sl; ++j) w[o * sl + j] = vp[o * sl + j] * sc;
      }
    } else {
      const tts_tensor_desc& d = tm.get(pre + "weight", {co, ci, k});
      memcpy(w.data(), d.data, w.size() * 4);
    }
    std::vector<float> r((size_t)co * c.kk, 0.f);  // [co][kk]: taps then zero columns
    for (int o = 0; o < co; ++o)
      for (int c2 = 0; c2 < ci; ++c2)
        for (int j = 0; j < k; ++j) r[(size_t)o * c.kk + (size_t)j * ci + c2] = w[((size_t)o * ci + c2) * k + j];
    c.w = put(r.data(), r.size());
    if (bias) c.b = put((const float*)tm.get(pre + "bias", {co}).data, co);
    return c;
  };
  auto snake = [&](const std::string& pre, int C) {
    EncSnake s;
    s.C = C;
    s.a = put((const float*)tm.get(pre + "act.alpha", {C}).data, C);
    s.b = put((const float*)tm.get(pre + "act.beta", {C}).data, C);
    return s;
  };
  const std::string a = "acoustic_encoder.";
  const int ratios[5] = {2, 2, 4, 4, 5}, dils[3] = {1, 3, 9};
  int d = 48;
  en->c0 = conv(a + "conv_blocks.0.", 1, d, 7, 1, 1, 3, true, true);
  for (int i = 0; i < 5; ++i) {
    const int half = d, s = ratios[i];
    d *= 2;
    EncBlock& b = en->blk[i];
    for (int r = 0; r < 3; ++r) {
      const std::string p = a + "conv_blocks." + std::to_string(i + 1) + ".block." + std::to_string(r) + ".block.";
      b.ru[r].s1 = snake(p + "0.", half);
      b.ru[r].c1 = conv(p + "1.", half, half, 7, 1, dils[r], 3 * dils[r], true, true);
      b.ru[r].s2 = snake(p + "2.", half);
      b.ru[r].c2 = conv(p + "3.", half, half, 1, 1, 1, 0, true, true);
    }
    const std::string p = a + "conv_blocks." + std::to_string(i + 1) + ".block.";
    b.s = snake(p + "3.", half);
    b.down = conv(p + "4.", half, d, 2 * s, s, 1, s / 2 + s % 2, true, true);
  }
  en->sf = snake(a + "conv_final_block.0.", d);
  en->cf = conv(a + "conv_final_block.1.", d, en->A, 3, 1, 1, 1, true, true);
  const std::string se = "semantic_encoder.";
  en->sem_init = conv(se + "initial_conv.", en->S, en->S, 3, 1, 1, 1, false, false);
  en->sem_c1 = conv(se + "residual_blocks.1.", en->S, en->S, 3, 1, 1, 1, false, true);
  en->sem_c2 = conv(se + "residual_blocks.3.", en->S, en->S, 3, 1, 1, 1, false, true);
  en->sem_final = conv(se + "final_conv.", en->S, en->S, 3, 1, 1, 1, false, false);
  const int F = en->S + en->A;
  en->fus_w = put((const float*)tm.get("fusion_layer.weight", {F, F}).data, (size_t)F * F);
  en->fus_b = put((const float*)tm.get("fusion_layer.bias", {F}).data, F);
  en->pin_w = put((const float*)tm.get("quantizer.project_in.weight", {en->nl, F}).data, (size_t)en->nl * F);
  en->pin_b = put((const float*)tm.get("quantizer.project_in.bias", {en->nl}).data, en->nl);
  // the anti-aliasing filters (filters.py kaiser_sinc_filter1d(0.25, 0.3, 12)), identical in
  // every Activation1d: taken from the final block's buffers
  en->filt_up = put((const float*)tm.get(a + "conv_final_block.0.upsample.filter", {1, 1, 12}).data, 12);
  en->filt_dn = put((const float*)tm.get(a + "conv_final_block.0.downsample.lowpass.filter", {1, 1, 12}).data, 12);

  // ---- w2v-bert (transformers Wav2Vec2BertModel state dict under "wav2vec_model.", as the
  // reference Encoder holds it), when present
  const std::string wp = "wav2vec_model.";
  if (tm.m.count(wp + "feature_projection.projection.weight")) {
    en->w2v = true;
    const int H = en->wH, FF = en->wFF, Fi = en->wFin, hd = H / en->wHeads, K = en->wK;
    auto vec = [&](const std::string& nm, std::initializer_list<int64_t> shp, float scale = 1.f) {
      const tts_tensor_desc& d = tm.get(nm, shp);
      std::vector<float> v((const float*)d.data, (const float*)d.data + numel(d));
      if (scale != 1.f) for (auto& x : v) x *= scale;  // (x 0.5: exact)
      return put(v.data(), v.size());
    };
    en->fp_ln[0] = vec(wp + "feature_projection.layer_norm.weight", {Fi});
    en->fp_ln[1] = vec(wp + "feature_projection.layer_norm.bias", {Fi});
    en->fp_w = vec(wp + "feature_projection.projection.weight", {H, Fi});
    en->fp_b = vec(wp + "feature_projection.projection.bias", {H});
    en->wl.resize(en->wLayers);
    for (int l = 0; l < en->wLayers; ++l) {
      W2vLayer& L = en->wl[l];
      const std::string p = wp + "encoder.layers." + std::to_string(l) + ".";
      for (int f = 0; f < 2; ++f) {
        const std::string q = p + (f ? "ffn2" : "ffn1");
        L.ffn_ln[f][0] = vec(q + "_layer_norm.weight", {H});
        L.ffn_ln[f][1] = vec(q + "_layer_norm.bias", {H});
        L.ffn_w1[f] = vec(q + ".intermediate_dense.weight", {FF, H});
        L.ffn_b1[f] = vec(q + ".intermediate_dense.bias", {FF});
        L.ffn_w2[f] = vec(q + ".output_dense.weight", {H, FF}, 0.5f);  // hidden * 0.5 + residual
        L.ffn_b2[f] = vec(q + ".output_dense.bias", {H}, 0.5f);
      }
      L.att_ln[0] = vec(p + "self_attn_layer_norm.weight", {H});
      L.att_ln[1] = vec(p + "self_attn_layer_norm.bias", {H});
      {
        std::vector<float> w((size_t)3 * H * H), b((size_t)3 * H);
        const char* nm[3] = {"q", "k", "v"};
        for (int i = 0; i < 3; ++i) {
          const tts_tensor_desc& wd = tm.get(p + "self_attn.linear_" + nm[i] + ".weight", {H, H});
          const tts_tensor_desc& bd = tm.get(p + "self_attn.linear_" + nm[i] + ".bias", {H});
          memcpy(w.data() + (size_t)i * H * H, wd.data, (size_t)H * H * 4);
          memcpy(b.data() + (size_t)i * H, bd.data, (size_t)H * 4);
        }
        L.qkv_w = put(w.data(), w.size());
        L.qkv_b = put(b.data(), b.size());
      }
      L.out_w = vec(p + "self_attn.linear_out.weight", {H, H});
      L.out_b = vec(p + "self_attn.linear_out.bias", {H});
      L.dist = vec(p + "self_attn.distance_embedding.weight", {en->wL + en->wR + 1, hd});
      L.conv_ln[0] = vec(p + "conv_module.layer_norm.weight", {H});
      L.conv_ln[1] = vec(p + "conv_module.layer_norm.bias", {H});
      L.pw1 = vec(p + "conv_module.pointwise_conv1.weight", {2 * H, H, 1});
      L.dw = vec(p + "conv_module.depthwise_conv.weight", {H, 1, K});
      L.dw_ln[0] = vec(p + "conv_module.depthwise_layer_norm.weight", {H});
      L.dw_ln[1] = vec(p + "conv_module.depthwise_layer_norm.bias", {H});
      L.pw2 = vec(p + "conv_module.pointwise_conv2.weight", {H, H, 1});
      L.fin_ln[0] = vec(p + "final_layer_norm.weight", {H});
      L.fin_ln[1] = vec(p + "final_layer_norm.bias", {H});
    }
  }

  en->weights.alloc(slab.size() * 4);
  HIP_CHECK(hipMemcpy(en->weights.p, slab.data(), slab.size() * 4, hipMemcpyHostToDevice));
  const int lv[8] = {4, 4, 4, 4, 4, 4, 4, 4};
  en->levels.alloc(sizeof(lv));
  HIP_CHECK(hipMemcpy(en->levels.p, lv, sizeof(lv), hipMemcpyHostToDevice));
  // bf16x3 planes of the large GEMM weights (K % 32 == 0 ones: the split-bf16 kernel)
  {
    std::vector<std::pair<const float*, size_t>> bw;
    auto add = [&](const EncConv& c) {
      if (c.kk % 32 == 0) bw.push_back({en->W(c.w), (size_t)c.cout * c.kk});
    };
    for (auto& b : en->blk) {
      for (auto& r : b.ru) { add(r.c1); add(r.c2); }
      add(b.down);
    }
    add(en->cf); add(en->sem_init); add(en->sem_c1); add(en->sem_c2); add(en->sem_final);
    bw.push_back({en->W(en->fus_w), (size_t)F * F});
    for (auto& L : en->wl) {
      const size_t H = en->wH, FF = en->wFF;
      for (int f = 0; f < 2; ++f) {
        bw.push_back({en->W(L.ffn_w1[f]), FF * H});
        bw.push_back({en->W(L.ffn_w2[f]), FF * H});
      }
      bw.push_back({en->W(L.qkv_w), 3 * H * H});
      bw.push_back({en->W(L.out_w), H * H});
      bw.push_back({en->W(L.pw1), 2 * H * H});
      bw.push_back({en->W(L.pw2), H * H});
    }
    size_t tot = 0;
    for (auto& w : bw) tot += (3 * w.second + 127) & ~(size_t)127;
    en->planes.alloc(tot * 2);
    size_t off = 0;
    for (auto& w : bw) {
      uint16_t* p = en->planes.as<uint16_t>() + off;
      launch_split_planes(w.first, p, (long long)w.second, nullptr);
      en->bplanes[w.first] = p;
      off += (3 * w.second + 127) & ~(size_t)127;
    }
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipDeviceSynchronize());
  }
  if (e->encoder) encoder_destroy(e->encoder);
  e->encoder = en.release();
}

namespace {

void grow_buf(DevBuf& b, size_t bytes) {
  if (b.bytes < bytes) b.alloc(bytes);
}

}  // namespace

// w2v-bert-2.0 hidden_states[16] of SeamlessM4T features (host [T][160]) into out (device
// [T][1024]): feature projection (LayerNorm, Linear), then 16 conformer layers
// (Wav2Vec2BertEncoderLayer: x + FFN1/2, x + attention, x + conv module, x + FFN2/2, final
// LayerNorm), every contraction on the fp32-exact GEMM.
static void w2v_forward(AudioEncoder& en, const float* feats, int T, float* out, hipStream_t s,
                        const std::function<void(const float*, int, int, int, const float*, int, const float*, float*,
                                                 int, const float*, int)>& gemm) {
  const int H = en.wH, FF = en.wFF, Fi = en.wFin;
  grow_buf(en.wfeat, (size_t)T * Fi * 4 * 2);
  grow_buf(en.wln, (size_t)T * H * 4);
  grow_buf(en.wbig, (size_t)T * FF * 4);
  grow_buf(en.wqkv, (size_t)T * 3 * H * 4);
  grow_buf(en.watt, (size_t)T * H * 4);
  float* f = en.wfeat.as<float>();
  float* fn = f + (size_t)T * Fi;
  float* x = out;
  float* ln = en.wln.as<float>();
  float* big = en.wbig.as<float>();
  float* qkv = en.wqkv.as<float>();
  float* att = en.watt.as<float>();
  HIP_CHECK(hipMemcpyAsync(f, feats, (size_t)T * Fi * 4, hipMemcpyHostToDevice, s));
  launch_layernorm_f32(f, T, Fi, en.W(en.fp_ln[0]), en.W(en.fp_ln[1]), en.wEps, fn, s);
  gemm(fn, T, Fi, Fi, en.W(en.fp_w), H, en.W(en.fp_b), x, H, nullptr, 0);
  for (const W2vLayer& L : en.wl) {
    for (int f2 = 0; f2 < 2; ++f2) {
      if (f2 == 1) {  // 3. the convolution module (between the attention and FFN2)
        launch_layernorm_f32(x, T, H, en.W(L.conv_ln[0]), en.W(L.conv_ln[1]), en.wEps, ln, s);
        gemm(ln, T, H, H, en.W(L.pw1), 2 * H, nullptr, big, 2 * H, nullptr, 0);
        launch_enc_glu(big, T, H, att, s);
        launch_enc_dwconv(att, T, H, en.W(L.dw), en.wK, ln, s);
        launch_layernorm_f32(ln, T, H, en.W(L.dw_ln[0]), en.W(L.dw_ln[1]), en.wEps, ln, s);
        launch_enc_swish(ln, (long long)T * H, s);
        gemm(ln, T, H, H, en.W(L.pw2), H, nullptr, x, H, x, 0);
      }
      // 1. / 4. x = x + FFN(LN(x)) / 2 (the 0.5 folded into output_dense at load)
      launch_layernorm_f32(x, T, H, en.W(L.ffn_ln[f2][0]), en.W(L.ffn_ln[f2][1]), en.wEps, ln, s);
      gemm(ln, T, H, H, en.W(L.ffn_w1[f2]), FF, en.W(L.ffn_b1[f2]), big, FF, nullptr, 1);
      gemm(big, T, FF, FF, en.W(L.ffn_w2[f2]), H, en.W(L.ffn_b2[f2]), x, H, x, 0);
      if (f2 == 0) {  // 2. x = x + attention(LN(x))
        launch_layernorm_f32(x, T, H, en.W(L.att_ln[0]), en.W(L.att_ln[1]), en.wEps, ln, s);
        gemm(ln, T, H, H, en.W(L.qkv_w), 3 * H, en.W(L.qkv_b), qkv, 3 * H, nullptr, 0);
        launch_enc_relattn(qkv, T, en.wHeads, en.W(L.dist), en.wL, en.wR, att, s);
        gemm(att, T, H, H, en.W(L.out_w), H, en.W(L.out_b), x, H, x, 0);
      }
    }
    launch_layernorm_f32(x, T, H, en.W(L.fin_ln[0]), en.W(L.fin_ln[1]), en.wEps, x, s);
  }
}

// codes[T] of one waveform (host fp32 [n] at 16 kHz) given either its w2v-bert layer-16
// features (host fp32 [T][1024]) or its SeamlessM4T features (host fp32 [T][160], w2v-bert
// run here), T = the number of 320-sample hops of the padded waveform.
int encoder_encode(Engine* e, const float* wav, int n, const float* w2v, int T_w2v, int32_t* codes_out, int cap,
                   float* pre_out, const float* feats) {
  TTS_REQUIRE(e->encoder != nullptr, "tts_encoder_load has not been called");
  TTS_REQUIRE(wav && n >= 1 && (w2v || feats), "null argument");
  TTS_REQUIRE(!feats || e->encoder->w2v, "the encoder was loaded without its w2v-bert tensors");
  AudioEncoder& en = *e->encoder;
  hipStream_t s = e->stream;
  const int Np = n + (320 - n % 320);  // encode(): pad to a whole hop (+ a hop when whole)
  const int T = Np / 320;
  TTS_REQUIRE(T_w2v == T, "w2v-bert features: one frame per 320-sample hop of the padded waveform expected");
  TTS_REQUIRE(cap >= T, "codes buffer too small");
  // workspace: the largest [T][C] map is 16 kHz x 48 (and its k7 windows)
  const size_t big = (size_t)Np * 48;
  grow_buf(en.x, big * 4);
  grow_buf(en.y, big * 4);
  grow_buf(en.z, big * 4);
  grow_buf(en.win, big * 7 * 4 + (size_t)Np * 16 * 4 + (size_t)T * 3 * 2048 * 4);
  grow_buf(en.sem, (size_t)T * en.S * 4 * 2);
  grow_buf(en.fused, (size_t)T * (en.S + en.A) * 4 * 2);
  grow_buf(en.proj, (size_t)T * en.nl * 4);
  grow_buf(en.codes, (size_t)T * 4);
  grow_buf(en.pre, (size_t)T * en.nl * 4);

  auto gemma = [&](const float* A, int M, int K, int lda, const float* B, int N, const float* bias, float* C,
                   int ldc, const float* resid, int act) {
    GemmF32Args g;
    g.A = A; g.M = M; g.K = K; g.lda = lda; g.B = B; g.N = N; g.bias = bias;
    auto it = en.bplanes.find(B);
    if (it != en.bplanes.end()) g.Bp = it->second;
    g.C = C; g.ldc = ldc; g.resid = resid; g.act = act;
    launch_gemm_f32(g, s);
  };
  auto gemm = [&](const float* A, int M, int K, int lda, const float* B, int N, const float* bias, float* C,
                  int ldc, const float* resid) { gemma(A, M, K, lda, B, N, bias, C, ldc, resid, 0); };
  // Conv1d on x [Tin][cin] -> out [To][cout] (+ resid [To][cout]); returns To
  auto conv = [&](const EncConv& c, const float* x, int Tin, float* out, const float* resid) {
    const int To = (Tin + 2 * c.pad - c.dil * (c.k - 1) - 1) / c.stride + 1;
    const float* bias = c.b == SIZE_MAX ? nullptr : en.W(c.b);
    if (c.k == 1 && c.stride == 1 && c.kk == c.cin) {
      gemm(x, To, c.cin, c.cin, en.W(c.w), c.cout, bias, out, c.cout, resid);
    } else {
      if (c.kk != c.k * c.cin) HIP_CHECK(hipMemsetAsync(en.win.p, 0, (size_t)To * c.kk * 4, s));
      launch_enc_im2col(x, Tin, c.cin, c.k, c.stride, c.dil, c.pad, To, c.kk, en.win.as<float>(), s);
      gemm(en.win.as<float>(), To, c.kk, c.kk, en.W(c.w), c.cout, bias, out, c.cout, resid);
    }
    return To;
  };
  auto snake = [&](const EncSnake& sn, const float* x, int Tn, float* y) {
    launch_enc_snake_aa(x, Tn, sn.C, en.W(sn.a), en.W(sn.b), en.W(en.filt_up), en.W(en.filt_dn), y, s);
  };

  // ---- acoustic path
  float* X = en.x.as<float>();
  float* Y = en.y.as<float>();
  float* Z = en.z.as<float>();
  HIP_CHECK(hipMemsetAsync(X, 0, (size_t)Np * 4, s));
  HIP_CHECK(hipMemcpyAsync(X, wav, (size_t)n * 4, hipMemcpyHostToDevice, s));
  int Tc = conv(en.c0, X, Np, Y, nullptr);  // Y = [Np][48]
  std::swap(X, Y);
  for (auto& b : en.blk) {
    for (auto& r : b.ru) {  // X = x + c2(snake(c1(snake(x))))
      snake(r.s1, X, Tc, Y);
      conv(r.c1, Y, Tc, Z, nullptr);
      snake(r.s2, Z, Tc, Y);
      conv(r.c2, Y, Tc, Z, X);
      std::swap(X, Z);
    }
    snake(b.s, X, Tc, Y);
    Tc = conv(b.down, Y, Tc, Z, nullptr);
    std::swap(X, Z);
  }
  TTS_REQUIRE(Tc == T, "acoustic encoder: frame count mismatch");
  snake(en.sf, X, Tc, Y);
  const int F = en.S + en.A;
  float* cat = en.fused.as<float>();                 // [T][semantic | acoustic]
  float* fused = cat + (size_t)T * F;
  // the final conv writes straight into the acoustic half of the concatenation
  {
    const EncConv& c = en.cf;
    launch_enc_im2col(Y, Tc, c.cin, c.k, c.stride, c.dil, c.pad, T, c.kk, en.win.as<float>(), s);
    gemm(en.win.as<float>(), T, c.kk, c.kk, en.W(c.w), c.cout, en.W(c.b), cat + en.S, F, nullptr);
  }
  // ---- semantic path (features in, left half of the concatenation out)
  float* sx = en.sem.as<float>();
  float* sr = sx + (size_t)T * en.S;
  if (feats) w2v_forward(en, feats, T, sx, s, gemma);
  else HIP_CHECK(hipMemcpyAsync(sx, w2v, (size_t)T * en.S * 4, hipMemcpyHostToDevice, s));
  conv(en.sem_init, sx, T, sr, nullptr);
  launch_enc_relu(sr, (long long)T * en.S, s);  // ReLU(inplace=True): the skip sees it too
  conv(en.sem_c1, sr, T, sx, nullptr);
  launch_enc_relu(sx, (long long)T * en.S, s);
  {
    const EncConv& c = en.sem_c2;  // conv + r  -> back into sx (window buffer holds the input)
    launch_enc_im2col(sx, T, c.cin, c.k, c.stride, c.dil, c.pad, T, c.kk, en.win.as<float>(), s);
    gemm(en.win.as<float>(), T, c.kk, c.kk, en.W(c.w), c.cout, en.W(c.b), sx, c.cout, sr);
  }
  {
    const EncConv& c = en.sem_final;
    launch_enc_im2col(sx, T, c.cin, c.k, c.stride, c.dil, c.pad, T, c.kk, en.win.as<float>(), s);
    gemm(en.win.as<float>(), T, c.kk, c.kk, en.W(c.w), c.cout, nullptr, cat, F, nullptr);
  }
  // ---- fusion, project_in, FSQ
  gemm(cat, T, F, F, en.W(en.fus_w), F, en.W(en.fus_b), fused, F, nullptr);
  gemm(fused, T, F, F, en.W(en.pin_w), en.nl, en.W(en.pin_b), en.proj.as<float>(), en.nl, nullptr);
  launch_enc_fsq(en.proj.as<float>(), T, en.nl, en.levels.as<int>(), en.codes.as<int>(), en.pre.as<float>(), s);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(codes_out, en.codes.p, (size_t)T * 4, hipMemcpyDeviceToHost, s));
  if (pre_out) HIP_CHECK(hipMemcpyAsync(pre_out, en.pre.p, (size_t)T * en.nl * 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return T;
}

}  // namespace tts
