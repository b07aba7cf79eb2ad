"""BASELINE configs[0]: the 100 LibriTTS utterances of example/configs/samples.jsonl as
synthesis requests.

Pairing = the reference's RLHF dataset (tts/data/datasets/rlhf.py:56-67): utterance i's
transcript is the audio prompt's transcription and utterance (i + 1) % n's transcript the
text to synthesize; InferencePromptCompiler joins them with a space
(tts/core/prompting.py:130-133) and appends <|speech_start|> + the prompt's speech codes
(:146-151).  Offline there is no Llama-3 tokenizer and no prompt wav, so (§8d) the joined
text becomes ceil(chars / 4) synthetic text ids and the prompt audio ceil(duration_i * 50)
synthetic codes (synth.synthetic_prompt's layout); the request generates exactly
N_i = ceil(duration_{i+1} * 50) codes (max_length = P_i + N_i, min_new_tokens = N_i, greedy,
repetition penalty 1.1), and the codec voices prompt + generated codes.
"""

from __future__ import annotations

import json
import math
from typing import Sequence

from . import configs, synth

TOKEN_RATE = 50


def load_samples(path: str) -> list[dict]:
    """samples.jsonl rows (or the committed fixture tests/golden/config1_samples.json)."""
    with open(path) as f:
        txt = f.read()
    if path.endswith(".json"):
        return json.loads(txt)["samples"]
    return [json.loads(line) for line in txt.splitlines() if line.strip()]


def requests(samples: Sequence[dict], vocab: configs.SpeechVocab, rng_base: int = 4321) -> list[dict]:
    """One request per utterance: prompt ids, the prompt's speech codes, new codes to make."""
    n = len(samples)
    lut = vocab.id_to_code()
    out = []
    for i, s in enumerate(samples):
        nxt = samples[(i + 1) % n]
        text = f"{s['transcript']} {nxt['transcript']}"
        n_text = math.ceil(len(text) / 4)
        n_codes = math.ceil(s["duration"] * TOKEN_RATE)
        prompt = synth.synthetic_prompt(vocab, i, n_text, n_codes, rng_base=rng_base)
        speech_ids = [int(lut[t]) for t in prompt[len(prompt) - n_codes:]]
        out.append(dict(prompt_ids=prompt, speech_ids=speech_ids, n_new=math.ceil(nxt["duration"] * TOKEN_RATE)))
    return out
