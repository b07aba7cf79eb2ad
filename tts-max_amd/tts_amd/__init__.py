"""tts_amd — MI355X-native host side of the SpeechLM-TTS hot path.

The compute lives in libtts_mi355x.so (tts-max_amd/csrc, HIP for gfx950) behind the C ABI
of include/tts_mi355x.h.  This package mirrors the reference's Python surfaces:

* ``speechlm.MI355XSpeechLM.generate``  — HF ``model.generate`` as called by
  tts/inference/inferencing.py:94-107 (and the vLLM form of :75-92)
* ``codec.MI355XAudioDecoder`` / ``codec.create`` — tts/core/codec/decoding.py
* ``inference`` — ``_synthesize_audio`` / ``LocalTtsModel``-style glue
* ``dp`` — utterance sharding over one process per GPU (torch.distributed / RCCL)
"""

import os as _os
import sys as _sys

__all__ = ["configs", "synth", "speechlm", "codec", "dp", "inference"]


def repo_root() -> str:
    return _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))


def _ensure_repo_on_path() -> None:
    r = repo_root()
    if r not in _sys.path:
        _sys.path.insert(0, r)
