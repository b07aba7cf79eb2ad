"""Continuous-batching serving on the MI355X engine.

The reference serves its SpeechLM through vLLM for RLHF rollouts (``trl vllm-serve``,
``run_rlhf_combine.sh:60``) and the ``--use_vllm`` CLI path (``tools/serving/inference.py:
83-95``, ``inferencing.py:75-92``: ``LLM.generate(prompt_token_ids=..., sampling_params=...)``
-> ``outputs[0].outputs[0].token_ids``).  This module provides the same duck-typed surface
backed by the engine's slot API (``tts_slots_*``):

* ``ContinuousBatcher`` — S persistent decode rows; queued requests are admitted into free
  rows between decode chunks and retired when they stop (EOS / max_tokens), so long and short
  utterances share the GPU without padding or waiting for the longest one.  Every request's
  tokens equal a batch-1 generate of its prompt with the batcher's settings (rows never mix;
  tests/test_gpu_serving.py).
* ``LLM`` — vLLM-shaped facade: ``generate(prompt_token_ids=list | list[list], sampling_params)``.
* ``create_app`` — a FastAPI app (``POST /generate``: ``{"prompt_token_ids": [...],
  "max_tokens": n}`` -> ``{"token_ids": [...]}``) over one batcher; run with uvicorn.

Settings (penalty, EOS, min_tokens, sampling) are per batcher, as the reference's
InferenceSettings are per process; requests differ in prompt and max_tokens.
"""

from __future__ import annotations

import ctypes
import dataclasses
import threading
from concurrent.futures import Future
from typing import Any, Sequence

import numpy as np
import torch

from . import _lib

try:  # the HTTP front end is optional (fastapi / pydantic are in the image)
    from pydantic import BaseModel as _BaseModel

    class GenerateRequest(_BaseModel):
        prompt_token_ids: list[int]
        max_tokens: int = 16
except ImportError:  # pragma: no cover
    GenerateRequest = None


@dataclasses.dataclass
class _Req:
    prompt: list[int]
    max_new: int
    future: Future
    seed: int | None = None  # the request's own sampling key (vLLM SamplingParams.seed)


class ContinuousBatcher:
    def __init__(self, lm, n_slots: int, eos_token_id: int = -1, min_new_tokens: int = 0,
                 repetition_penalty: float = 1.0, do_sample: bool = False, temperature: float = 1.0,
                 top_k: int = 50, top_p: float = 1.0, frequency_penalty: float = 0.0, seed: int | None = None,
                 chunk: int = 8):
        if n_slots < 1 or n_slots > lm.max_batch:
            raise ValueError(f"n_slots {n_slots} outside [1, max_batch={lm.max_batch}]")
        if do_sample and seed is None:
            seed = int(torch.randint(0, 2**62, (1,)).item())
        self.lm, self.S, self.chunk = lm, n_slots, chunk
        self._p = _lib.GenParams(max_length=0, min_new_tokens=min_new_tokens, eos_token_id=eos_token_id,
                                 do_sample=1 if do_sample else 0, repetition_penalty=repetition_penalty,
                                 temperature=temperature, top_p=top_p, top_k=top_k, seed=seed or 0,
                                 frequency_penalty=frequency_penalty)
        self._queue: list[_Req] = []
        self._slot_req: list[_Req | None] = [None] * n_slots
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self._stop = False
        self._opened = False
        self._thread: threading.Thread | None = None
        self._buf = np.zeros(lm.max_seq_len, dtype=np.int32)
        self.error: BaseException | None = None  # set when the engine loop failed (batcher dead)

    # ------------------------------------------------------------------ requests -------
    def submit(self, prompt_ids: Sequence[int], max_new_tokens: int, seed: int | None = None) -> Future:
        """Queues a request.  `seed` fixes the request's sampling stream (vLLM per-request
        seed); None draws a fresh stream per request from the batcher's seed."""
        fut: Future = Future()
        if self.error is not None:
            fut.set_exception(RuntimeError(f"batcher stopped after an engine error: {self.error}"))
            return fut
        with self._lock:
            self._queue.append(_Req(list(map(int, prompt_ids)), int(max_new_tokens), fut,
                                    None if seed is None else int(seed) & (2**64 - 1)))
        self._wake.set()
        return fut

    def busy(self) -> bool:
        with self._lock:
            return bool(self._queue) or any(r is not None for r in self._slot_req)

    def generate(self, prompts: Sequence[Sequence[int]], max_new_tokens: int | Sequence[int],
                 seed: int | None = None) -> list[list[int]]:
        """Blocking: all prompts through the continuous batch, results in order."""
        if isinstance(max_new_tokens, int):
            max_new_tokens = [max_new_tokens] * len(prompts)
        futs = [self.submit(p, n, seed) for p, n in zip(prompts, max_new_tokens)]
        if self._thread is None:  # no background loop: drive it here
            while not all(f.done() for f in futs):
                self._run_guarded()
        return [f.result() for f in futs]

    # ------------------------------------------------------------------ engine loop ----
    def _open(self):
        if not self._opened or self.lm._slot_batcher is not self:
            _lib.check(self.lm._lib.tts_slots_open(self.lm._h, ctypes.byref(self._p), self.S, None))
            self.lm._slot_batcher = self
            self._opened = True

    def _fail_all(self, ex: BaseException) -> None:
        """An engine error ends the batcher: every active and queued request fails with it
        (no future is left pending), and later submissions fail at once."""
        self.error = ex
        with self._lock:
            reqs = [r for r in self._slot_req if r is not None] + self._queue
            self._slot_req = [None] * self.S
            self._queue = []
        for r in reqs:
            if not r.future.done():
                r.future.set_exception(ex)
        if self.lm._slot_batcher is self:
            self.lm._slot_batcher = None
        self._opened = False

    def _run_guarded(self) -> int:
        try:
            return self.run_once()
        except Exception as ex:  # noqa: BLE001 (TtsError and anything else: fail loudly, never hang)
            self._fail_all(ex)
            return 0

    def run_once(self) -> int:
        """Admit queued requests into free slots, run one chunk of decode steps, retire the
        stopped sequences.  Returns the number of rows still generating."""
        with self.lm.lock:
            return self._run_once_locked()

    def _run_once_locked(self) -> int:
        self._open()
        h, L = self.lm._h, self.lm._lib
        pi32 = ctypes.POINTER(ctypes.c_int32)
        with self._lock:
            for s in range(self.S):
                if self._slot_req[s] is None and self._queue:
                    r = self._queue.pop(0)
                    arr = np.ascontiguousarray(np.asarray(r.prompt, dtype=np.int32))
                    try:
                        if r.seed is None:
                            _lib.check(L.tts_slots_add(h, s, arr.ctypes.data_as(pi32), len(arr), r.max_new))
                        else:
                            _lib.check(L.tts_slots_add_seeded(h, s, arr.ctypes.data_as(pi32), len(arr), r.max_new,
                                                              r.seed))
                    except _lib.TtsError as ex:  # bad request: fail it, keep serving
                        r.future.set_exception(ex)
                        continue
                    self._slot_req[s] = r
        act = ctypes.c_int32(0)
        if any(r is not None for r in self._slot_req):
            _lib.check(L.tts_slots_step(h, self.chunk, ctypes.byref(act)))
        n, fin = ctypes.c_int32(0), ctypes.c_int32(0)
        for s, r in enumerate(self._slot_req):
            if r is None:
                continue
            _lib.check(L.tts_slots_read(h, s, self._buf.ctypes.data_as(pi32), len(self._buf), ctypes.byref(n),
                                        ctypes.byref(fin)))
            if fin.value:
                r.future.set_result(self._buf[:n.value].tolist())
                _lib.check(L.tts_slots_release(h, s))
                self._slot_req[s] = None
        return act.value

    def start(self):
        """Serve from a background thread (one engine = one thread, as the C ABI requires)."""
        if self._thread is not None:
            return

        def loop():
            while not self._stop:
                busy = any(r is not None for r in self._slot_req)
                with self._lock:
                    busy = busy or bool(self._queue)
                if not busy:
                    self._wake.wait(0.05)
                    self._wake.clear()
                    continue
                self._run_guarded()
                if self.error is not None:
                    return

        self._thread = threading.Thread(target=loop, name="tts-mi355x-batcher", daemon=True)
        self._thread.start()

    def close(self):
        self._stop = True
        self._wake.set()
        if self._thread is not None:
            self._thread.join()
            self._thread = None


@dataclasses.dataclass
class CompletionOutput:
    token_ids: list[int]


@dataclasses.dataclass
class RequestOutput:
    prompt_token_ids: list[int]
    outputs: list[CompletionOutput]


class LLM:
    """vLLM-shaped facade (inferencing.py:75-92): one ContinuousBatcher per distinct
    SamplingParams configuration."""

    def __init__(self, lm, n_slots: int = 16, chunk: int = 8):
        self.lm, self.n_slots, self.chunk = lm, n_slots, chunk
        self._batchers: dict[tuple, ContinuousBatcher] = {}

    def _batcher(self, sp: Any) -> ContinuousBatcher:
        temperature = float(getattr(sp, "temperature", 1.0) or 0.0)
        stop = list(getattr(sp, "stop_token_ids", None) or [])
        if len(stop) > 1:
            raise NotImplementedError("one stop token id is supported")
        if float(getattr(sp, "presence_penalty", 0.0) or 0.0) != 0.0:
            raise NotImplementedError("vLLM presence_penalty is not implemented")
        top_k = int(getattr(sp, "top_k", -1) or -1)
        if temperature > 0 and top_k <= 0:
            raise NotImplementedError("full-vocabulary sampling (vLLM top_k=-1) is not built; pass top_k")
        key = (temperature, stop[0] if stop else -1, int(getattr(sp, "min_tokens", 0) or 0),
               float(getattr(sp, "repetition_penalty", 1.0) or 1.0), top_k, float(getattr(sp, "top_p", 1.0) or 1.0),
               float(getattr(sp, "frequency_penalty", 0.0) or 0.0))
        old = self._batchers.get(key)
        if old is not None and old.error is not None:  # a batcher that died on an engine error:
            old.close()                                 # replace it instead of failing every later call
            del self._batchers[key]
        if key not in self._batchers:
            for b in self._batchers.values():  # one slot batch open per engine at a time
                b._opened = False
            self._batchers = {}
            self._batchers[key] = ContinuousBatcher(
                self.lm, self.n_slots, eos_token_id=key[1], min_new_tokens=key[2], repetition_penalty=key[3],
                do_sample=temperature > 0, temperature=temperature or 1.0, top_k=top_k if top_k > 0 else 50,
                top_p=key[5], frequency_penalty=key[6], seed=None, chunk=self.chunk)
        return self._batchers[key]

    def generate(self, prompt_token_ids: Sequence[int] | Sequence[Sequence[int]], sampling_params: Any = None,
                 **unused) -> list[RequestOutput]:
        prompts = prompt_token_ids
        if prompts and isinstance(prompts[0], (int, np.integer)):
            prompts = [prompts]
        b = self._batcher(sampling_params)
        outs = b.generate(prompts, int(getattr(sampling_params, "max_tokens", 16)),
                          seed=getattr(sampling_params, "seed", None))
        return [RequestOutput(prompt_token_ids=list(p), outputs=[CompletionOutput(token_ids=o)])
                for p, o in zip(prompts, outs)]


def create_app(batcher: ContinuousBatcher):
    """FastAPI app over a started batcher: POST /generate {"prompt_token_ids", "max_tokens"}."""
    import asyncio

    from fastapi import FastAPI, HTTPException

    app = FastAPI(title="tts-mi355x")
    batcher.start()

    @app.post("/generate")
    async def generate(req: GenerateRequest):
        if not req.prompt_token_ids or req.max_tokens < 1:
            raise HTTPException(status_code=400, detail="empty prompt or max_tokens < 1")
        fut = batcher.submit(req.prompt_token_ids, req.max_tokens)
        try:
            ids = await asyncio.wrap_future(fut)
        except Exception as ex:  # engine rejected the request
            raise HTTPException(status_code=400, detail=str(ex))
        return {"token_ids": ids}

    @app.get("/health")
    async def health():
        if batcher.error is not None:
            raise HTTPException(status_code=503, detail=f"engine error: {batcher.error}")
        return {"ok": True}

    return app
