"""The synthesis composition around the two engine surfaces.

Restates tts/inference/inferencing.py for callers that hold token ids (the prompt text is
tokenised by the checkpoint's HF tokenizer, which stays as it is — SURVEY §8b):

* ``InferenceSettings``            inferencing.py:15-37 (same fields and defaults)
* ``extract_speech_ids``           inferencing.py:53-63, replaced by the engine's id -> code
                                   LUT built from the checkpoint tokenizer (non-speech ids are
                                   dropped and logged, as the string parse does)
* ``generate_speech_tokens``       inferencing.py:66-107 (HF form and vLLM form)
* ``synthesize_audio``             inferencing.py:110-159: generate, keep
                                   ``generated[P - len(speech_ids) : -1]`` (the last id is
                                   dropped unconditionally, EOS or not), ids -> codes, decode,
                                   cut the prompt audio ``int(len(speech_ids) / token_rate *
                                   sample_rate)`` samples
* ``complete_prompt``              inferencing.py:231-276 (audio prompt completion: ids
                                   ``[speech_start] + prompt codes``, slice ``[1:-1]``)

The arithmetic runs in the engine (speechlm.MI355XSpeechLM, codec.MI355XAudioDecoder); this
module only moves ids, exactly as the reference does.
"""

from __future__ import annotations

import dataclasses
import logging
import time
from typing import Sequence

import torch

_log = logging.getLogger(__name__)


@dataclasses.dataclass
class InferenceSettings:
    """inferencing.py:15-37.  `max_tokens` is HF's `max_length` (prompt included) on the HF
    form and vLLM's `max_tokens` (new tokens) on the vLLM form, as in the reference."""

    temperature: float = 0.8
    max_tokens: int = 1792
    min_tokens: int = 10
    top_p: float = 1.0
    top_k: int = 50
    repetition_penalty: float = 1.1
    frequency_penalty: float = 0.3
    seed: int = 42


DEFAULT_INFERENCE_SETTINGS = InferenceSettings()


@dataclasses.dataclass
class SamplingParams:
    """The fields of vllm.SamplingParams that inferencing.py:78-88 sets."""

    max_tokens: int = 16
    min_tokens: int = 0
    stop_token_ids: list | None = None
    repetition_penalty: float = 1.0
    top_p: float = 1.0
    top_k: int = -1
    frequency_penalty: float = 0.0
    temperature: float = 1.0
    seed: int | None = None
    detokenize: bool = False


def extract_speech_ids(model, ids: Sequence[int]) -> list[int]:
    """Speech codes of `ids` (inferencing.py:53-63): the LUT maps <|s_N|> ids to N and
    every other id to -1, which is logged and dropped like an unexpected token string."""
    codes = model.ids_to_codes(list(ids)) if len(ids) else []
    out = []
    for i, c in zip(ids, codes):
        if c >= 0:
            out.append(int(c))
        else:
            _log.error("Unexpected token: %d", int(i))
    return out


def generate_speech_tokens(model, input_ids: torch.Tensor, settings: InferenceSettings, speech_end_id: int,
                           use_vllm: bool = False):
    """inferencing.py:66-107.  HF form: LongTensor [P + N] on the CPU (prompt included, EOS
    included when produced); vLLM form: the completion ids (list)."""
    if use_vllm:
        sp = SamplingParams(max_tokens=settings.max_tokens, min_tokens=settings.min_tokens,
                            stop_token_ids=[speech_end_id], repetition_penalty=settings.repetition_penalty,
                            top_p=settings.top_p, top_k=settings.top_k, frequency_penalty=settings.frequency_penalty,
                            temperature=settings.temperature)
        out = model.generate(prompt_token_ids=input_ids[0].tolist(), sampling_params=sp)
        return out[0].outputs[0].token_ids
    return model.generate(input_ids=input_ids, max_length=settings.max_tokens, min_new_tokens=settings.min_tokens,
                          eos_token_id=speech_end_id, do_sample=settings.temperature > 0.0,
                          repetition_penalty=settings.repetition_penalty, top_p=settings.top_p,
                          temperature=settings.temperature).cpu().squeeze(0)


def synthesize_audio(model, audio_decoder, input_ids: torch.Tensor | Sequence[int], speech_ids: Sequence[int],
                     speech_end_id: int, settings: InferenceSettings = DEFAULT_INFERENCE_SETTINGS,
                     use_vllm: bool = False) -> tuple[torch.Tensor, float]:
    """inferencing.py:110-159 from the tokenised prompt: (wav [1, L - prompt samples] float32
    CPU, codec seconds).  `speech_ids` are the prompt's speech codes (the audio encoder's
    output the prompt compiler embedded)."""
    if not isinstance(input_ids, torch.Tensor):
        input_ids = torch.tensor([list(input_ids)], dtype=torch.long)
    if input_ids.dim() == 1:
        input_ids = input_ids[None]
    torch.manual_seed(settings.seed)  # transformers.set_seed (inferencing.py:129)
    generated = generate_speech_tokens(model, input_ids, settings, speech_end_id, use_vllm)
    if use_vllm:
        codes = list(speech_ids) + extract_speech_ids(model, list(generated))
    else:
        kept = generated[input_ids.shape[1] - len(speech_ids): -1]
        codes = extract_speech_ids(model, kept.tolist())
    t0 = time.perf_counter()
    wav = audio_decoder.decode(torch.tensor(codes, dtype=torch.long))
    decoding_time = time.perf_counter() - t0
    prompt_samples = int(len(speech_ids) / audio_decoder.token_rate * audio_decoder.sample_rate)
    return wav[:, prompt_samples:], decoding_time


def complete_prompt(model, audio_decoder, prompt_codes: Sequence[int], code_to_id, speech_start_id: int,
                    speech_end_id: int, settings: InferenceSettings = DEFAULT_INFERENCE_SETTINGS) -> torch.Tensor:
    """inferencing.py:231-276 from the encoder's prompt codes: `[speech_start] + ids of the
    codes`, generate, drop the first and the last id, decode, cut the prompt audio."""
    ids = [speech_start_id] + [int(code_to_id(int(c))) for c in prompt_codes]
    generated = generate_speech_tokens(model, torch.tensor([ids]), settings, speech_end_id)
    codes = extract_speech_ids(model, generated[1:-1].tolist())
    wav = audio_decoder.decode(torch.tensor(codes, dtype=torch.long))
    prompt_samples = int(len(prompt_codes) / audio_decoder.token_rate * audio_decoder.sample_rate)
    return wav[:, prompt_samples:]
