#!/usr/bin/env python
"""Batched decode on one GPU as ONE engine of R*B rows vs R engines (replicas, each its own
weights, workspace and stream) of B rows decoding concurrently from R host threads (ctypes
releases the GIL during each engine call).  Every engine runs the same greedy job: prompts of
the bench's shape, `new` codes each.  Prints wall time, codes/s and each engine's decode-step
time; the replicas' ids must equal the single engine's rows (same weights seed).

usage: python scripts/replica_probe.py [rows=32] [replicas=2] [new=500]
"""
import hashlib
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))

import torch  # noqa: E402

from tts_amd import configs, synth  # noqa: E402
from tts_amd.speechlm import MI355XSpeechLM  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    new = int(sys.argv[3]) if len(sys.argv) > 3 else 500
    arch = configs.TTS1
    vocab = configs.vocab_for(arch)
    ps = [synth.synthetic_prompt(vocab, 1000 + u, 39, 150) for u in range(rows)]
    P = max(len(p) for p in ps)
    kw = dict(max_length=P + new, min_new_tokens=new, eos_token_id=vocab.speech_end_id, repetition_penalty=1.1)

    one = MI355XSpeechLM.synthetic(arch, seed=0x5EED, max_batch=rows, max_seq_len=P + new + 16)
    for _ in range(2):
        t = time.perf_counter()
        ref = one.generate_batch(ps, **kw)
        el = time.perf_counter() - t
    a, b, k = one.last_timing()
    print(f"1 engine x {rows} rows: {el * 1000:.1f} ms, {rows * new / el:.0f} codes/s, step {b / k * 1000:.1f} us",
          flush=True)
    del one
    torch.cuda.empty_cache()

    B = rows // R
    engs = [MI355XSpeechLM.synthetic(arch, seed=0x5EED, max_batch=B, max_seq_len=P + new + 16) for _ in range(R)]
    outs = [None] * R

    def job(i):
        outs[i] = engs[i].generate_batch(ps[i * B:(i + 1) * B], **kw)

    for _ in range(2):
        th = [threading.Thread(target=job, args=(i,)) for i in range(R)]
        t = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        el = time.perf_counter() - t
    steps = [e.last_timing() for e in engs]
    seq = [engs[i].generate_batch(ps[i * B:(i + 1) * B], **kw) for i in range(R)]  # one after another
    print(f"concurrent ids equal the same engines run one after another: {seq == outs}", flush=True)
    got = [o for out in outs for o in out]
    same = hashlib.md5(str(got).encode()).hexdigest() == hashlib.md5(str(ref).encode()).hexdigest()
    print(f"{R} engines x {B} rows concurrently: {el * 1000:.1f} ms, {rows * new / el:.0f} codes/s, steps "
          + ", ".join(f"{b / k * 1000:.1f} us" for a, b, k in steps) + f"; ids equal the single engine's: {same}",
          flush=True)


if __name__ == "__main__":
    main()
