"""Model architectures and the speech-vocabulary layout.

SpeechLM dims are the public Llama configs the reference builds on
(tts/core/tokenization.py:7: "Llama 3.1 8B Instruct and Llama 3.2 1B Instruct with speech
tokens"; example/configs/sft.json:25).  The codec dims are the Generator defaults of
tts/core/codec/decoder_modules.py:403-431 and the configs of example/codec/model_config.json
and example/configs/codec_training_config.json:23-35.
"""

from __future__ import annotations

import dataclasses
import json
import os


@dataclasses.dataclass(frozen=True)
class LmArch:
    name: str
    hidden_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate_size: int
    vocab_size: int
    tie_word_embeddings: bool
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_llama3: bool = True
    rope_factor: float = 32.0
    rope_low_freq_factor: float = 1.0
    rope_high_freq_factor: float = 4.0
    rope_original_max_position: int = 8192
    max_position_embeddings: int = 131072

    def weight_bytes_per_step(self) -> int:
        """bf16 weight bytes streamed by one decode step (every matrix once; embedding
        gather excluded; tied lm_head counted once)."""
        H, KVH, D, HID, FF = self.num_heads, self.num_kv_heads, self.head_dim, self.hidden_size, self.intermediate_size
        per_layer = HID * (H + 2 * KVH) * D + H * D * HID + 3 * HID * FF + 2 * HID
        return 2 * (self.num_layers * per_layer + HID + self.vocab_size * HID)

    def kv_bytes_per_token(self) -> int:
        return 2 * 2 * self.num_layers * self.num_kv_heads * self.head_dim

    def hf_config_dict(self) -> dict:
        d = dict(
            architectures=["LlamaForCausalLM"], model_type="llama", hidden_size=self.hidden_size,
            num_hidden_layers=self.num_layers, num_attention_heads=self.num_heads,
            num_key_value_heads=self.num_kv_heads, head_dim=self.head_dim,
            intermediate_size=self.intermediate_size, vocab_size=self.vocab_size,
            tie_word_embeddings=self.tie_word_embeddings, rms_norm_eps=self.rms_norm_eps,
            rope_theta=self.rope_theta, max_position_embeddings=self.max_position_embeddings,
            hidden_act="silu", attention_bias=False, mlp_bias=False, bos_token_id=128000,
        )
        if self.rope_llama3:
            d["rope_scaling"] = dict(rope_type="llama3", factor=self.rope_factor,
                                     low_freq_factor=self.rope_low_freq_factor,
                                     high_freq_factor=self.rope_high_freq_factor,
                                     original_max_position_embeddings=self.rope_original_max_position)
        return d

    @staticmethod
    def from_hf_config(path_or_dict, name: str = "hf") -> "LmArch":
        c = path_or_dict
        if not isinstance(c, dict):
            with open(path_or_dict) as f:
                c = json.load(f)
        rs = c.get("rope_scaling") or c.get("rope_parameters") or {}
        llama3 = (rs.get("rope_type") or rs.get("type")) == "llama3"
        H = c["num_attention_heads"]
        return LmArch(
            name=name, hidden_size=c["hidden_size"], num_layers=c["num_hidden_layers"], num_heads=H,
            num_kv_heads=c.get("num_key_value_heads", H),
            head_dim=c.get("head_dim") or c["hidden_size"] // H,
            intermediate_size=c["intermediate_size"], vocab_size=c["vocab_size"],
            tie_word_embeddings=bool(c.get("tie_word_embeddings", False)),
            rms_norm_eps=float(c.get("rms_norm_eps", 1e-5)),
            rope_theta=float(c.get("rope_theta", rs.get("rope_theta", 10000.0))), rope_llama3=llama3,
            rope_factor=float(rs.get("factor", 1.0)), rope_low_freq_factor=float(rs.get("low_freq_factor", 1.0)),
            rope_high_freq_factor=float(rs.get("high_freq_factor", 4.0)),
            rope_original_max_position=int(rs.get("original_max_position_embeddings", 8192)),
            max_position_embeddings=int(c.get("max_position_embeddings", 131072)),
        )


# TTS-1 = Llama-3.2-1B dims with the 193,856-token speech vocabulary (tied embeddings).
TTS1 = LmArch("tts1", 2048, 16, 32, 8, 64, 8192, 193856, True, rope_factor=32.0)
# TTS-1-Max = Llama-3.1-8B dims (untied lm_head, llama3 factor 8).
TTS1_MAX = LmArch("tts1-max", 4096, 32, 32, 8, 128, 14336, 193856, False, rope_factor=8.0)
# Small test architectures (same kernels, same GQA group and head dims).
TINY = LmArch("tiny", 256, 2, 4, 1, 64, 512, 2048, True)
SMALL = LmArch("small", 512, 4, 8, 2, 64, 1536, 8192, True)
TINY128 = LmArch("tiny128", 512, 2, 4, 1, 128, 1024, 2048, False, rope_factor=8.0)

# TTS-1-Max dims with 2 layers: every kernel shape of config 4 (hd 128, K 4096 / 14336 in
# K-chunked layouts, untied 193,856-row lm_head) at a size a CPU oracle checks in seconds.
TTS1_MAX_2L = LmArch("tts1-max-2l", 4096, 2, 32, 8, 128, 14336, 193856, False, rope_factor=8.0)

LM_ARCHS = {a.name: a for a in (TTS1, TTS1_MAX, TINY, SMALL, TINY128, TTS1_MAX_2L)}


@dataclasses.dataclass(frozen=True)
class CodecArch:
    """DecoderConfig (tts/core/codec/decoding.py:14-35) + Generator dims."""

    name: str
    sample_rate: int
    token_rate: int
    hop_length: int
    upsample_factors: tuple[int, ...]
    kernel_sizes: tuple[int, ...]
    hidden_dim: int = 1024
    depth: int = 12
    heads: int = 16
    vq_dim: int = 2048
    model_type: str = "xcodec2"

    @property
    def samples_per_code(self) -> int:
        u = 1
        for f in self.upsample_factors:
            u *= f
        return self.hop_length * u

    @staticmethod
    def from_json(path: str | os.PathLike, name: str = "json") -> "CodecArch":
        """DecoderConfig.from_json; `model_type` is optional here (the shipped
        example/codec/model_config.json lacks it, which makes the reference raise).  An
        optional `depth` key (not a reference key) selects the reduced-depth test variants."""
        with open(path) as f:
            c = json.load(f)
        return CodecArch(name=name, sample_rate=c["sample_rate"], token_rate=c["token_rate"],
                         hop_length=c["hop_length"], upsample_factors=tuple(c.get("upsample_factors") or ()),
                         kernel_sizes=tuple(c.get("kernel_sizes") or ()),
                         model_type=c.get("model_type", "xcodec2"), depth=int(c.get("depth", 12)))

    def to_json_dict(self) -> dict:
        return dict(model_type=self.model_type, sample_rate=self.sample_rate, token_rate=self.token_rate,
                    hop_length=self.hop_length, upsample_factors=list(self.upsample_factors) or None,
                    kernel_sizes=list(self.kernel_sizes) or None)


CODEC_16K = CodecArch("xcodec2-16k", 16000, 50, 320, (), ())
CODEC_24K = CodecArch("codec-24k", 24000, 50, 160, (3,), (7,))
CODEC_48K = CodecArch("codec-48k", 48000, 50, 160, (3, 2), (7, 6))
# reduced-depth variant for quick tests (same kernels)
CODEC_24K_D2 = CodecArch("codec-24k-d2", 24000, 50, 160, (3,), (7,), depth=2)

CODEC_ARCHS = {a.name: a for a in (CODEC_16K, CODEC_24K, CODEC_48K, CODEC_24K_D2)}


@dataclasses.dataclass(frozen=True)
class EncoderArch:
    """The prompt-audio codec encoder (tts/core/codec/encoder.py:20-56): SemanticEncoder over
    w2v-bert-2.0 layer-16 features, AcousticEncoder over the 16 kHz waveform, fusion Linear,
    ResidualFSQ (one quantizer, 8 levels of 4).  The w2v-bert dimensions are the hub model's
    (facebook/w2v-bert-2.0, not in the reference tree): parity of those dimensions is
    unpinned; the arithmetic is transformers' Wav2Vec2BertModel."""

    name: str = "encoder-16k"
    sample_rate: int = 16000
    token_rate: int = 50
    hop: int = 320
    ngf: int = 48                                   # AcousticEncoder num_generator_features
    up_ratios: tuple[int, ...] = (2, 2, 4, 4, 5)
    dilations: tuple[int, ...] = (1, 3, 9)
    acoustic_dim: int = 1024
    semantic_dim: int = 1024
    levels: tuple[int, ...] = (4, 4, 4, 4, 4, 4, 4, 4)
    # w2v-bert-2.0 (hub config): only the first `w2v_layers` layers feed hidden_states[16]
    w2v_hidden: int = 1024
    w2v_layers: int = 16
    w2v_heads: int = 16
    w2v_ffn: int = 4096
    w2v_feat_in: int = 160
    w2v_left: int = 64
    w2v_right: int = 8
    w2v_conv_k: int = 31
    w2v_eps: float = 1e-5

    def w2v_hf_config(self) -> dict:
        return dict(hidden_size=self.w2v_hidden, num_hidden_layers=self.w2v_layers,
                    num_attention_heads=self.w2v_heads, intermediate_size=self.w2v_ffn,
                    feature_projection_input_dim=self.w2v_feat_in, hidden_act="swish",
                    position_embeddings_type="relative_key", left_max_position_embeddings=self.w2v_left,
                    right_max_position_embeddings=self.w2v_right, conv_depthwise_kernel_size=self.w2v_conv_k,
                    layer_norm_eps=self.w2v_eps, add_adapter=False, hidden_dropout=0.0,
                    attention_dropout=0.0, activation_dropout=0.0, feat_proj_dropout=0.0,
                    conformer_conv_dropout=0.0, layerdrop=0.0, apply_spec_augment=False)


ENCODER = EncoderArch()


@dataclasses.dataclass(frozen=True)
class SpeechVocab:
    """Token-id layout produced by tts/core/tokenization.py:36-61: the 8 control tokens and
    the 65,536 ``<|s_N|>`` tokens are added in ``sorted()`` (lexicographic) order after the
    base vocabulary, then ``<|extra_token_i|>`` pad the vocabulary to 193,856."""

    base_vocab: int = 128256
    codebook_size: int = 65536
    total: int = 193856
    text_vocab: int = 128000
    bos_id: int = 128000
    newline_id: int = 198

    def _added(self) -> list[str]:
        ctrl = ["<|speech_start|>", "<|speech_end|>", "<|text_prompt_start|>", "<|text_prompt_end|>",
                "<|voice_description_start|>", "<|voice_description_end|>", "<|sound_effect_start|>",
                "<|sound_effect_end|>"]
        return sorted(ctrl + [f"<|s_{i}|>" for i in range(self.codebook_size)])

    def token_ids(self) -> dict[str, int]:
        cache = getattr(self, "_tok_cache", None)
        if cache is None:
            cache = {t: self.base_vocab + i for i, t in enumerate(self._added())}
            object.__setattr__(self, "_tok_cache", cache)
        return cache

    def id_to_code(self):
        import numpy as np

        lut = np.full(self.total, -1, dtype=np.int32)
        for t, i in self.token_ids().items():
            if t.startswith("<|s_"):
                lut[i] = int(t[4:-2])
        return lut

    def code_to_id(self, code: int) -> int:
        return self.token_ids()[f"<|s_{code}|>"]

    @property
    def speech_start_id(self) -> int:
        return self.token_ids()["<|speech_start|>"]

    @property
    def speech_end_id(self) -> int:
        return self.token_ids()["<|speech_end|>"]

    @property
    def text_prompt_start_id(self) -> int:
        return self.token_ids()["<|text_prompt_start|>"]

    @property
    def text_prompt_end_id(self) -> int:
        return self.token_ids()["<|text_prompt_end|>"]


@dataclasses.dataclass(frozen=True)
class SmallVocab:
    """Vocabulary layout for the small test architectures (same roles, tiny ids)."""

    total: int
    codebook_size: int
    base_vocab: int = 256
    text_vocab: int = 200
    bos_id: int = 201
    newline_id: int = 202

    @property
    def speech_start_id(self) -> int:
        return 203

    @property
    def speech_end_id(self) -> int:
        return 204

    @property
    def text_prompt_start_id(self) -> int:
        return 205

    @property
    def text_prompt_end_id(self) -> int:
        return 206

    def code_to_id(self, code: int) -> int:
        return self.base_vocab + code

    def id_to_code(self):
        import numpy as np

        lut = np.full(self.total, -1, dtype=np.int32)
        lut[self.base_vocab:self.base_vocab + self.codebook_size] = np.arange(self.codebook_size, dtype=np.int32)
        return lut


TTS_VOCAB = SpeechVocab()


def vocab_for(arch: LmArch):
    if arch.vocab_size == TTS_VOCAB.total:
        return TTS_VOCAB
    return SmallVocab(total=arch.vocab_size, codebook_size=arch.vocab_size - 256 - 64)
