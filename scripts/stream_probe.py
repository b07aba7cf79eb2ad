"""Streaming latency breakdown (bs=8, 25-code chunks): prefill, first chunk of decode steps,
codec window, host overhead."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))
import torch  # noqa: E402

from tts_amd import configs, synth  # noqa: E402
from tts_amd.codec import MI355XAudioDecoder  # noqa: E402
from tts_amd.speechlm import MI355XSpeechLM  # noqa: E402
from tts_amd.streaming import StreamingSynthesizer  # noqa: E402

arch, carch = configs.LM_ARCHS["tts1"], configs.CODEC_ARCHS["codec-24k"]
vocab = configs.vocab_for(arch)
lm = MI355XSpeechLM.synthetic(arch, seed=0x5EED, max_batch=8, max_seq_len=740)
dec = MI355XAudioDecoder.synthetic(carch, seed=0xC0DEC, max_codes=700)
p8 = [synth.synthetic_prompt(vocab, 1000 + u, 39, 150) for u in range(8)]
pc8 = [[c for c in lm.ids_to_codes(p[-150:]) if c >= 0] for p in p8]
P = max(len(p) for p in p8)
kw = dict(min_new_tokens=500, eos_token_id=vocab.speech_end_id, repetition_penalty=1.1)
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g = lm.generate_stream(p8, P + 500, chunk=25, **kw)
    ids, _ = next(g)
    t1 = time.perf_counter()
    ids, _ = next(g)
    t2 = time.perf_counter()
    wins = [pc8[b][-25:] + [c for c in lm.ids_to_codes(ids[b]) if c >= 0][:25] for b in range(8)]
    t3 = time.perf_counter()
    dec.decode_batch(wins)
    t4 = time.perf_counter()
    for _ in g:
        pass
    a, b, k = lm.last_timing()
    print(f"rep {rep}: begin(prefill+1st) {1e3*(t1-t0):.1f} ms, 25 steps {1e3*(t2-t1):.1f} ms, "
          f"ids->codes {1e3*(t3-t2):.1f} ms, codec window x8 {1e3*(t4-t3):.1f} ms, first audio {1e3*(t4-t0):.1f} ms",
          flush=True)
ss = StreamingSynthesizer(lm, dec)
for rep in range(2):
    for out, el in ss.stream(p8, pc8, max_length=P + 500, **kw):
        print(f"synth first chunk at {1e3*el:.1f} ms", flush=True)
        break

# where does the synthesizer's extra time go?
import functools  # noqa: E402

marks = []


def wrap(obj, name):
    f = getattr(obj, name)

    @functools.wraps(f)
    def g(*a, **k):
        t = time.perf_counter()
        r = f(*a, **k)
        marks.append((name, time.perf_counter() - t))
        return r
    setattr(obj, name, g)


wrap(dec, "decode_batch")
wrap(lm, "ids_to_codes")
orig_gs = lm.generate_stream


def gs(*a, **k):
    it = orig_gs(*a, **k)
    while True:
        t = time.perf_counter()
        try:
            v = next(it)
        except StopIteration:
            return
        marks.append(("gen_next", time.perf_counter() - t))
        yield v


lm.generate_stream = gs
for out, el in ss.stream(p8, pc8, max_length=P + 500, **kw):
    print(f"synth first chunk at {1e3*el:.1f} ms", flush=True)
    break
agg = {}
for n, d in marks:
    agg.setdefault(n, [0, 0.0])
    agg[n][0] += 1
    agg[n][1] += d
print({k: (v[0], round(1e3 * v[1], 1)) for k, v in agg.items()}, flush=True)
