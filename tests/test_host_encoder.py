"""Host-side pieces of the prompt-audio encoder (no GPU): the reference's padding, the
checkpoint key mapping of Encoder.load_from_checkpoint, and the synthetic weight names."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tts-max_amd"))
from tts_amd import configs, encoder, synth  # noqa: E402


def test_padding_matches_reference_quirk():
    """encoder.py:117: hop - n % hop, i.e. a whole extra hop when n is already whole."""
    a, ap = encoder.pad_like_reference(torch.zeros(1, 640))
    assert a.shape[-1] == 960 and ap.shape[-1] == 1280
    a, _ = encoder.pad_like_reference(torch.zeros(1, 641))
    assert a.shape[-1] == 960


def test_xcodec2_checkpoint_mapping(tmp_path):
    sd = {"CodecEnc.conv_blocks.0.bias": torch.ones(3), "generator.quantizer.project_in.bias": torch.ones(8),
          "SemanticEncoder_module.final_conv.weight": torch.ones(2), "fc_prior.weight": torch.ones(1),
          "generator.backbone.embed.weight": torch.ones(1)}
    p = tmp_path / "xcodec2.ckpt"
    torch.save({"state_dict": sd}, p)
    w = encoder.load_encoder_checkpoint(str(p))
    assert set(w) == {"acoustic_encoder.conv_blocks.0.bias", "quantizer.project_in.bias",
                      "semantic_encoder.final_conv.weight", "fusion_layer.weight"}
    p2 = tmp_path / "enc.pt"
    torch.save({"fusion_layer.bias": torch.zeros(4)}, p2)
    assert set(encoder.load_encoder_checkpoint(str(p2))) == {"fusion_layer.bias"}


def test_synthetic_weight_names_cover_the_fixture_model():
    """The spec names are the reference modules' parameter names (the fixture generator
    loads them with only the filter buffers missing); the w2v-bert specs are exactly
    transformers' Wav2Vec2BertModel state dict at the hub dimensions."""
    from transformers import Wav2Vec2BertConfig, Wav2Vec2BertModel

    cfg = Wav2Vec2BertConfig(**configs.ENCODER.w2v_hf_config())
    with torch.device("meta"):
        m = Wav2Vec2BertModel(cfg)
    spec = {n: s for n, s, *_ in synth.w2v_tensor_specs(configs.ENCODER)}
    assert spec == {k: tuple(v.shape) for k, v in m.state_dict().items()}
    names = [n for n, *_ in synth.encoder_tensor_specs(configs.ENCODER)]
    assert len(names) == len(set(names)) == 195
    f = synth.kaiser_sinc_filter(0.25, 0.3, 12)
    assert abs(float(f.sum()) - 1.0) < 1e-6 and np.allclose(f.numpy(), f.numpy()[::-1])


def test_caching_encoder_constructor_forms(monkeypatch, tmp_path):
    """CachingAudioEncoder(model_path, device) as the reference builds it (encoding.py:59-63,
    tools/serving/inference.py:115-116) goes through create(); an encoder object is wrapped
    as is.  Both cache per prompt id."""
    calls = []

    class Fake:
        def encode(self, wav):
            calls.append("encode")
            return torch.tensor([[3, 1, 4]]).reshape(-1)

    def fake_create(model_path, device=0, w2v_path=None):
        calls.append((model_path, device, w2v_path))
        return Fake()

    monkeypatch.setattr(encoder, "create", fake_create)
    ck = tmp_path / "encoder.ckpt"
    c1 = encoder.CachingAudioEncoder(str(ck), torch.device("cuda", 0))
    assert calls == [(str(ck), torch.device("cuda", 0), None)]
    c2 = encoder.CachingAudioEncoder(ck, "cuda:0", w2v_path="/local/w2v-bert-2.0")
    assert calls[-1] == (str(ck), "cuda:0", "/local/w2v-bert-2.0")
    c3 = encoder.CachingAudioEncoder(Fake())
    for c in (c1, c2, c3):
        n = calls.count("encode")
        assert c.encode("p0", torch.zeros(1, 320)) == [3, 1, 4]
        assert c.encode("p0", torch.zeros(1, 320)) == [3, 1, 4]
        assert calls.count("encode") == n + 1


def test_feature_extractor_front_end_check():
    from transformers import SeamlessM4TFeatureExtractor

    encoder.check_feature_extractor(SeamlessM4TFeatureExtractor(padding_value=1.0))
    import pytest

    with pytest.raises(ValueError):
        encoder.check_feature_extractor(SeamlessM4TFeatureExtractor())  # padding_value 0.0
