"""Prompt-audio encoder surface backed by the MI355X engine.

Drop-in for tts/core/codec/encoding.py: ``AudioEncoderInterface`` (9-26), ``AudioEncoder``
(29-52: encode(wav [1, N] at 16 kHz) -> codes, sample_rate, token_rate),
``CachingAudioEncoder`` (55-72: per-prompt-id cache, codes as a list) and ``create`` (75-80).

Split of the work (the reference runs it all in ``Encoder.encode``, encoder.py:115-128):

* host (CPU, as the reference): the padding and transformers' SeamlessM4TFeatureExtractor
  (the reference's own feature extractor class);
* everything after it in fp32 HIP kernels through ``tts_encoder_encode_features``:
  w2v-bert-2.0 up to hidden_states[16] (feature projection, 16 conformer layers with
  relative-key attention and the causal depthwise-conv module), AcousticEncoder over the
  waveform (Snake with the anti-aliased 2x filters, dilated and strided convolutions),
  SemanticEncoder, fusion, ResidualFSQ quantisation.
"""

from __future__ import annotations

import abc
import ctypes

import os

import numpy as np
import torch

from . import _lib, configs, synth


class AudioEncoderInterface(metaclass=abc.ABCMeta):
    """Same abstract surface as tts.core.codec.encoding.AudioEncoderInterface."""

    @abc.abstractmethod
    def encode(self, wav: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    @property
    @abc.abstractmethod
    def sample_rate(self) -> int:
        raise NotImplementedError

    @property
    @abc.abstractmethod
    def token_rate(self) -> int:
        raise NotImplementedError


def pad_like_reference(wav: torch.Tensor, hop: int = 320) -> tuple[torch.Tensor, torch.Tensor]:
    """encoder.py:117-120: pad to a whole hop (a full extra hop when already whole, as the
    reference's ``hop - n % hop`` does), then half a hop each side for the feature extractor."""
    audio = torch.nn.functional.pad(wav.cpu().float(), (0, hop - (wav.shape[-1] % hop)))
    return audio, torch.nn.functional.pad(audio, (hop // 2, hop // 2))


class MI355XAudioEncoder(AudioEncoderInterface):
    """One encoder resident on one MI355X (its own engine)."""

    def __init__(self, weights: dict[str, torch.Tensor], feature_extractor,
                 arch: configs.EncoderArch = configs.ENCODER, device: int = 0):
        """weights: the reference Encoder's state dict (its own modules and, under
        "wav2vec_model.", the w2v-bert-2.0 tensors) plus the anti-aliasing filter buffers."""
        self.arch = arch
        self.device = torch.device("cuda", device)
        self._lib = _lib.load_library()
        h = ctypes.c_void_p()
        _lib.check(self._lib.tts_engine_create(device, ctypes.byref(h)))
        self._h = h
        tensors = {k: v.detach().float().cpu().contiguous() for k, v in weights.items()}
        f = synth.kaiser_sinc_filter(0.25, 0.3, 12).view(1, 1, 12)  # the filters' buffers (filters.py)
        tensors.setdefault("acoustic_encoder.conv_final_block.0.upsample.filter", f)
        tensors.setdefault("acoustic_encoder.conv_final_block.0.downsample.lowpass.filter", f.clone())
        descs, keep = _lib.make_descs(tensors)
        _lib.check(self._lib.tts_encoder_load(self._h, descs, len(tensors)))
        del keep
        self._fe = feature_extractor

    @classmethod
    def synthetic(cls, arch: configs.EncoderArch = configs.ENCODER, seed: int = 0xE2C0, device: int = 0):
        """Random-init weights of the encoder (synth.encoder_tensor_specs, seed) and of the
        w2v-bert model (synth.w2v_tensor_specs, seed + 1) — the generator the golden fixture
        tests/golden/encoder_16k.npz was made with."""
        import transformers

        dev = torch.device("cuda", device)
        w = synth.weights_from_specs_device(synth.encoder_tensor_specs(arch), seed, dev)
        for k, v in synth.weights_from_specs_device(synth.w2v_tensor_specs(arch), seed + 1, dev).items():
            w["wav2vec_model." + k] = v
        fe = transformers.SeamlessM4TFeatureExtractor(padding_value=1.0)
        return cls(w, fe, arch=arch, device=device)

    @property
    def sample_rate(self) -> int:
        return self.arch.sample_rate

    @property
    def token_rate(self) -> int:
        return self.arch.token_rate

    def features(self, wav: torch.Tensor) -> np.ndarray:
        """SeamlessM4TFeatureExtractor input_features of the reference-padded waveform [1, N]
        -> [T, 160] (host, as encoder.py:121-123)."""
        _, audio_pad = pad_like_reference(wav.reshape(1, -1), self.arch.hop)
        feat = self._fe(audio_pad, sampling_rate=self.arch.sample_rate, return_tensors="pt").data["input_features"]
        return np.ascontiguousarray(feat[0].float().numpy())

    def encode_with_features(self, wav: np.ndarray, w2v: np.ndarray, return_pre: bool = False):
        """The HIP part of Encoder.encode: waveform [N] + its w2v-bert features [T, 1024] ->
        codes [T] (and the values the FSQ rounded, [T, 8])."""
        wav = np.ascontiguousarray(wav, dtype=np.float32).reshape(-1)
        w2v = np.ascontiguousarray(w2v, dtype=np.float32)
        T = w2v.shape[0]
        codes = np.zeros(T, dtype=np.int32)
        pre = np.zeros((T, len(self.arch.levels)), dtype=np.float32) if return_pre else None
        n = ctypes.c_int32()
        f32p = ctypes.POINTER(ctypes.c_float)
        _lib.check(self._lib.tts_encoder_encode(
            self._h, wav.ctypes.data_as(f32p), wav.size, w2v.ctypes.data_as(f32p), T,
            codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), T, ctypes.byref(n),
            pre.ctypes.data_as(f32p) if return_pre else None))
        return (codes[: n.value], pre) if return_pre else codes[: n.value]

    def encode_from_features(self, wav: np.ndarray, feats: np.ndarray, return_pre: bool = False):
        """Waveform [N] + its SeamlessM4T features [T, 160] -> codes [T]: w2v-bert and the
        rest of the encoder in HIP (tts_encoder_encode_features)."""
        wav = np.ascontiguousarray(wav, dtype=np.float32).reshape(-1)
        feats = np.ascontiguousarray(feats, dtype=np.float32)
        T = feats.shape[0]
        codes = np.zeros(T, dtype=np.int32)
        pre = np.zeros((T, len(self.arch.levels)), dtype=np.float32) if return_pre else None
        n = ctypes.c_int32()
        f32p = ctypes.POINTER(ctypes.c_float)
        _lib.check(self._lib.tts_encoder_encode_features(
            self._h, wav.ctypes.data_as(f32p), wav.size, feats.ctypes.data_as(f32p), T,
            codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), T, ctypes.byref(n),
            pre.ctypes.data_as(f32p) if return_pre else None))
        return (codes[: n.value], pre) if return_pre else codes[: n.value]

    @torch.no_grad()
    def encode(self, wav: torch.Tensor) -> torch.Tensor:
        """AudioEncoder.encode (encoding.py:42-45 -> encoder.py:115-128): wav [1, N] at
        16 kHz -> codes [T] (int64, CPU; the reference's .squeeze() of the [1, 1, T] codes)."""
        wav = wav.reshape(1, -1)
        codes = self.encode_from_features(wav[0].float().cpu().numpy(), self.features(wav))
        return torch.from_numpy(codes.astype(np.int64))

    def close(self):
        if getattr(self, "_h", None):
            self._lib.tts_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class CachingAudioEncoder:
    """encoding.py:55-72: encodes a prompt once per prompt id; codes as a Python list.

    Constructed as the reference does, ``CachingAudioEncoder(model_path, device)``
    (encoding.py:59-63, called so at tools/serving/inference.py:115-116; the encoder comes from
    ``create``, with ``w2v_path`` = a local facebook/w2v-bert-2.0 when the checkpoint lacks
    it), or around an already built encoder object."""

    def __init__(self, model_path: "str | os.PathLike | AudioEncoderInterface",
                 device: "torch.device | str | int | None" = 0, *, w2v_path: str | None = None):
        if isinstance(model_path, (str, os.PathLike)):
            self._encoder = create(model_path=os.fspath(model_path), device=device, w2v_path=w2v_path)
        else:
            self._encoder = model_path
        self._prompt_encoding_cache: dict[str, list[int]] = {}

    @torch.no_grad()
    def encode(self, prompt_id: str, prompt_wav: torch.Tensor) -> list[int]:
        if prompt_id in self._prompt_encoding_cache:
            return self._prompt_encoding_cache[prompt_id]
        codes = self._encoder.encode(prompt_wav).cpu().tolist()
        self._prompt_encoding_cache[prompt_id] = codes
        return codes


# xcodec2 checkpoint prefixes -> the reference Encoder's module names (encoder.py:87-105)
_XCODEC2_PREFIXES = (("CodecEnc.", "acoustic_encoder."), ("generator.quantizer.", "quantizer."),
                     ("SemanticEncoder_module.", "semantic_encoder."), ("fc_prior.", "fusion_layer."))


def load_encoder_checkpoint(path: str) -> dict[str, torch.Tensor]:
    """Encoder.load_from_checkpoint (encoder.py:80-113) with weights_only=True (no pickled
    code runs): an xcodec2 {"state_dict": ...} checkpoint has its four prefixes mapped onto the
    Encoder's modules (other keys ignored, as there); anything else is the Encoder's own state
    dict (which may include "wav2vec_model.*")."""
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    if "state_dict" in ckpt:
        out = {}
        for k, v in ckpt["state_dict"].items():
            for src, dst in _XCODEC2_PREFIXES:
                if k.startswith(src):
                    out[dst + k[len(src):]] = v
        return out
    return dict(ckpt)


# the w2v-bert-2.0 front end the encoder's weights expect (feature projection input =
# num_mel_bins x stride = 160; 16 kHz; padding with 1.0 as the hub preprocessor_config)
W2V_FEATURES = dict(feature_size=80, num_mel_bins=80, stride=2, sampling_rate=16000, padding_value=1.0)


def check_feature_extractor(fe) -> None:
    bad = {k: getattr(fe, k, None) for k, v in W2V_FEATURES.items() if getattr(fe, k, None) != v}
    if bad:
        raise ValueError(f"feature extractor differs from the w2v-bert-2.0 front end {W2V_FEATURES}: {bad}")


def create(model_path: str, device: "torch.device | str | int | None" = 0,
           w2v_path: str | None = None) -> MI355XAudioEncoder:
    """encoding.create (75-80): the encoder from its checkpoint.  The reference loads
    facebook/w2v-bert-2.0 and its feature extractor from the hub (encoder.py:50-56); offline
    they come from a local copy of that model directory (`w2v_path`: config.json,
    safetensors weights, preprocessor_config.json) unless the checkpoint already holds
    "wav2vec_model.*"."""
    import transformers

    w = load_encoder_checkpoint(model_path)
    if not any(k.startswith("wav2vec_model.") for k in w):
        if w2v_path is None:
            raise ValueError("the checkpoint has no w2v-bert weights: pass w2v_path (a local facebook/w2v-bert-2.0)")
        m = transformers.Wav2Vec2BertModel.from_pretrained(w2v_path)
        for k, v in m.state_dict().items():
            w["wav2vec_model." + k] = v
    if w2v_path:
        fe = transformers.SeamlessM4TFeatureExtractor.from_pretrained(w2v_path)
    else:
        # no preprocessor_config.json at hand: the w2v-bert-2.0 hub values (padding_value 1.0;
        # the rest are SeamlessM4TFeatureExtractor's defaults).  Those hub values cannot be
        # read offline, so the features of real weights are PARITY UNPINNED;
        # the parameters the encoder depends on are checked here
        fe = transformers.SeamlessM4TFeatureExtractor(padding_value=1.0)
    check_feature_extractor(fe)
    dev = torch.device(device) if not isinstance(device, int) else torch.device("cuda", device)
    return MI355XAudioEncoder(w, fe, device=dev.index or 0)
