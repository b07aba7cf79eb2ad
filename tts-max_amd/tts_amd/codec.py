"""Codec decoder surface backed by the MI355X engine.

Drop-in for tts/core/codec/decoding.py: ``AudioDecoderInterface`` (38-56), ``AudioDecoder``
(59-97: decode(speech_ids [T]) -> [1, L] float32 CPU, sample_rate, token_rate) and
``create(model_path, device)`` (100-112, reads model_config.json next to the checkpoint).
"""

from __future__ import annotations

import abc
import ctypes
import os
from typing import Sequence

import numpy as np
import torch

from . import _lib, configs, synth


class AudioDecoderInterface(metaclass=abc.ABCMeta):
    """Same abstract surface as tts.core.codec.decoding.AudioDecoderInterface."""

    @abc.abstractmethod
    def decode(self, speech_ids: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    @property
    @abc.abstractmethod
    def sample_rate(self) -> int:
        raise NotImplementedError

    @property
    @abc.abstractmethod
    def token_rate(self) -> int:
        raise NotImplementedError


def expected_codec_keys(arch: configs.CodecArch) -> set[str]:
    """The reference Decoder's state-dict keys for `arch` (tts/core/codec/decoder.py:14-67;
    the synthetic generator emits exactly these, pinned by load_state_dict(strict=True) in
    oracle/make_golden.py)."""
    keys = {name for name, *_ in synth.codec_tensor_specs(arch)}
    keys |= {"decoder.head.istft.window", "decoder.quantizer.project_in.weight", "decoder.quantizer.project_in.bias"}
    return keys


def load_codec_checkpoint(path: str, arch: configs.CodecArch | None = None) -> dict[str, torch.Tensor]:
    """Decoder.load_from_checkpoint (tts/core/codec/decoder.py:91-119), loaded with
    weights_only=True (no pickled code is executed):

    * {"model": {"generator.<Decoder key>"}}: the prefix stripped, then load_state_dict(strict)
      into the whole Decoder — missing or unexpected keys raise, as there;
    * xcodec2 {"state_dict": {"generator.<Generator key>", "fc_post_a.*"}}: the Generator and
      fc_post_a loaded strictly; the reference leaves an upsampler (none in xcodec2) at its
      random init, which cannot be reproduced, so a config with upsampling raises here.

    ConvTranspose weight-norm pairs (weight_g, weight_v) are folded by the engine at load."""
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    out: dict[str, torch.Tensor] = {}
    xcodec2 = "state_dict" in ckpt
    if xcodec2:
        for k, v in ckpt["state_dict"].items():
            if k.startswith("generator."):
                out["decoder." + k[len("generator."):]] = v
            elif k.startswith("fc_post_a."):
                out[k] = v
    else:
        for k, v in ckpt["model"].items():
            if k.startswith("generator."):
                out[k[len("generator."):]] = v
    if arch is not None:
        want = expected_codec_keys(arch)
        if xcodec2:
            if arch.upsample_factors:
                raise ValueError("xcodec2 state_dict checkpoints carry no upsampler weights; "
                                 f"config {arch.name} has upsample factors {arch.upsample_factors}")
            want = {k for k in want if k.startswith(("decoder.", "fc_post_a."))}
        missing, unexpected = sorted(want - set(out)), sorted(set(out) - want)
        if missing or unexpected:
            raise RuntimeError(f"Error(s) in loading state_dict for Decoder: missing keys {missing[:8]}, "
                               f"unexpected keys {unexpected[:8]}")
    return {k: v.float().contiguous() for k, v in out.items() if torch.is_tensor(v)}


class MI355XAudioDecoder(AudioDecoderInterface):
    """xcodec2-compatible decoder on one MI355X (fp32 arithmetic, like the reference)."""

    def __init__(self, arch: configs.CodecArch, weights: dict[str, torch.Tensor], device: int = 0,
                 max_codes: int = 4096, engine=None):
        self.arch = arch
        self.device = torch.device("cuda", device)
        self._lib = _lib.load_library()
        self._own = engine is None
        if engine is None:
            h = ctypes.c_void_p()
            _lib.check(self._lib.tts_engine_create(device, ctypes.byref(h)))
            self._h = h
        else:
            self._h = engine
        ups = list(arch.upsample_factors)
        ks = list(arch.kernel_sizes)
        cfg = _lib.CodecConfig(sample_rate=arch.sample_rate, token_rate=arch.token_rate, hop_length=arch.hop_length,
                               n_upsample=len(ups), hidden_dim=arch.hidden_dim, depth=arch.depth,
                               heads=arch.heads, vq_dim=arch.vq_dim, max_codes=max_codes)
        for i, (u, k) in enumerate(zip(ups, ks)):
            cfg.upsample_factors[i] = u
            cfg.kernel_sizes[i] = k
        host = {k: v.detach().float().cpu().contiguous() for k, v in weights.items()}
        descs, keep = _lib.make_descs(host)
        _lib.check(self._lib.tts_codec_load(self._h, ctypes.byref(cfg), descs, len(host)))
        del keep
        self.max_codes = max_codes
        self._spc = arch.samples_per_code

    @classmethod
    def synthetic(cls, arch: configs.CodecArch, seed: int = 0xC0DEC, device: int = 0, **kw):
        return cls(arch, synth.codec_weights_cpu(arch, seed), device=device, **kw)

    @property
    def sample_rate(self) -> int:
        return self.arch.sample_rate

    @property
    def token_rate(self) -> int:
        return self.arch.token_rate

    @torch.no_grad()
    def decode(self, speech_ids: torch.Tensor) -> torch.Tensor:
        """[T] int codes -> [1, T * samples_per_code] float32 (CPU), as AudioDecoder.decode."""
        codes = speech_ids.reshape(-1).cpu().to(torch.int32).numpy()
        wav = self.decode_batch([codes])[0]
        return torch.from_numpy(wav)[None]

    def decode_batch(self, utterances: Sequence[Sequence[int]], out: torch.Tensor | None = None) -> list[np.ndarray]:
        """Several utterances in one call (each decoded exactly as alone).  If `out` is a
        device tensor of sum(T)*samples_per_code floats, the waveforms stay in HBM and
        views of it are returned instead of host arrays."""
        lens = np.array([len(u) for u in utterances], dtype=np.int32)
        flat = np.ascontiguousarray(np.concatenate([np.asarray(u, dtype=np.int32) for u in utterances]))
        total = int(lens.sum()) * self._spc
        wav_lens = np.zeros(len(utterances), dtype=np.int64)
        pi32 = ctypes.POINTER(ctypes.c_int32)
        if out is not None:
            assert out.is_cuda and out.dtype == torch.float32 and out.numel() >= total
            _lib.check(self._lib.tts_codec_decode(self._h, flat.ctypes.data_as(pi32), lens.ctypes.data_as(pi32),
                                                  len(utterances), out.data_ptr(), 1,
                                                  wav_lens.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                                  _lib.stream_ptr()))
            res, off = [], 0
            for n in wav_lens:
                res.append(out[off:off + int(n)])
                off += int(n)
            return res
        host = np.zeros(total, dtype=np.float32)
        _lib.check(self._lib.tts_codec_decode(self._h, flat.ctypes.data_as(pi32), lens.ctypes.data_as(pi32),
                                              len(utterances), host.ctypes.data, 0,
                                              wav_lens.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), None))
        res, off = [], 0
        for n in wav_lens:
            res.append(host[off:off + int(n)])
            off += int(n)
        return res

    def close(self):
        if self._own and getattr(self, "_h", None):
            self._lib.tts_engine_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def create(model_path: str, device: torch.device | str | int | None = 0, max_codes: int = 4096) -> MI355XAudioDecoder:
    """decoding.create: model_config.json must sit next to the checkpoint."""
    cfg_path = os.path.join(os.path.dirname(model_path), "model_config.json")
    if not os.path.exists(cfg_path):
        raise ValueError("No model_config.json found in the provided path.")
    arch = configs.CodecArch.from_json(cfg_path, name=os.path.basename(os.path.dirname(model_path)))
    if isinstance(device, torch.device):
        device = device.index or 0
    elif isinstance(device, str):
        device = int(device.split(":")[1]) if ":" in device else 0
    return MI355XAudioDecoder(arch, load_codec_checkpoint(model_path, arch), device=device or 0, max_codes=max_codes)
