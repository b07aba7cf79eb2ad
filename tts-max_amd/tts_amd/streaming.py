"""Streaming synthesis (BASELINE config 5): chunked autoregressive decode + windowed codec.

The reference has no streaming path (the codec's GroupNorm and attention pool
over the whole utterance, so a chunked decode is not equal to a full decode).  This module
defines the streaming contract the build measures:

* the SpeechLM runs the same device loop as ``generate_batch`` (``generate_stream``), paused
  every ``chunk`` codes, so the token ids are identical to a one-shot generation;
* every ``chunk`` new speech codes of a row are voiced by decoding a window of
  ``left_context`` preceding codes (the prompt's speech codes before the first chunk) plus
  the chunk, and emitting the chunk's samples (the window's last ``chunk * samples_per_code``
  samples).  Each window is decoded exactly as the reference ``Decoder.forward`` would decode
  that window alone (tts/core/codec/decoder.py:69-89) — the streaming oracle is "the
  reference decoder applied to the same window";
* the final partial chunk (after EOS / max_length) is voiced the same way.

Latency metric: time from the request to a row's first audio chunk (prefill + ``chunk`` decode
steps + one windowed codec call).
"""

from __future__ import annotations

import time
from typing import Iterator, Sequence

import numpy as np


class StreamingSynthesizer:
    def __init__(self, lm, codec, chunk: int = 25, left_context: int = 25, to_codes=None):
        """to_codes(ids) -> speech codes of a row's new ids; default: the LUT of the
        checkpoint tokenizer, non-speech ids dropped (extract_speech_ids,
        inferencing.py:53-63)."""
        self.lm, self.codec = lm, codec
        self.to_codes = to_codes or (lambda ids: [c for c in lm.ids_to_codes(ids) if c >= 0])
        self.chunk, self.left = chunk, left_context
        self.spc = codec.sample_rate // codec.token_rate

    def stream(self, prompts: Sequence[Sequence[int]], prompt_codes: Sequence[Sequence[int]], max_length: int,
               **gen_kw) -> Iterator[tuple[list[tuple[int, np.ndarray]], float]]:
        """Yields ([(row, audio chunk float32), ...], seconds since the request) whenever at
        least one row has a new chunk voiced."""
        t0 = time.perf_counter()
        B = len(prompts)
        voiced = [0] * B  # speech codes of each row already turned into audio

        def windows_for(new_ids, flush):
            """One window per row with a full chunk pending (or any codes, when flushing)."""
            wins, rows, emit = [], [], []
            for b in range(B):
                codes = self.to_codes(new_ids[b])
                pending = len(codes) - voiced[b]
                if pending >= self.chunk or (flush and pending > 0):
                    n = min(self.chunk, pending)
                    hist = list(prompt_codes[b]) + codes[:voiced[b]]
                    ctx = hist[max(0, len(hist) - self.left):] if self.left > 0 else []
                    wins.append(ctx + codes[voiced[b]:voiced[b] + n])
                    rows.append(b)
                    emit.append(n)
                    voiced[b] += n
            return wins, rows, emit

        for new_ids, done in self.lm.generate_stream(prompts, max_length, chunk=self.chunk, **gen_kw):
            while True:  # after the last step: flush what is pending, chunk by chunk
                wins, rows, emit = windows_for(new_ids, done)
                if not wins:
                    break
                wavs = self.codec.decode_batch(wins)
                yield [(b, w[len(w) - n * self.spc:]) for b, w, n in zip(rows, wavs, emit)], \
                    time.perf_counter() - t0
                if not done:
                    break
