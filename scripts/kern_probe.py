"""Per-kernel decode times of one architecture at `rows` (bench_kernel, HBM-cold layer
rotation) with their algorithmic GB/s, and the graph-replayed decode step.
usage: python scripts/kern_probe.py ARCH ROWS [NEW]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))
from tts_amd import configs, synth  # noqa: E402
from tts_amd.speechlm import MI355XSpeechLM  # noqa: E402

arch = configs.LM_ARCHS[sys.argv[1]]
rows = int(sys.argv[2])
new = int(sys.argv[3]) if len(sys.argv) > 3 else 200
m = MI355XSpeechLM.synthetic(arch, max_batch=rows, max_seq_len=202 + new + 16)
r = {}
for k in m.KERNELS:
    ms, by = m.bench_kernel(k, rows=rows, ctx=202 + new // 2, iters=32)
    r[k] = {"us": round(ms * 1000, 2), "GBs": round(by / ms / 1e6, 1)}
vocab = configs.vocab_for(arch)
ps = [synth.synthetic_prompt(vocab, u, 39, 150) for u in range(rows)]
for _ in range(2):
    m.generate_batch(ps, max_length=len(ps[0]) + new, min_new_tokens=new, eos_token_id=vocab.speech_end_id,
                     repetition_penalty=1.1)
a, b, k = m.last_timing()
r["step_us"] = round(b / k * 1000, 1)
r["step_GBs"] = round((arch.weight_bytes_per_step() + rows * arch.kv_bytes_per_token() * (202 + new // 2)) / (b / k) / 1e6, 1)
print(json.dumps(r), flush=True)
