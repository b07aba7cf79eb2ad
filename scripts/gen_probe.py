"""One batched greedy generation on TTS-1 random weights (for rocprofv3 kernel traces of the
decode step at a given batch).  usage: python scripts/gen_probe.py ROWS NEW"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tts-max_amd"))
from tts_amd import configs, synth  # noqa: E402
from tts_amd.speechlm import MI355XSpeechLM  # noqa: E402

rows, new = int(sys.argv[1]), int(sys.argv[2])
arch = configs.TTS1
vocab = configs.vocab_for(arch)
m = MI355XSpeechLM.synthetic(arch, seed=0x5EED, max_batch=rows, max_seq_len=202 + new + 16)
ps = [synth.synthetic_prompt(vocab, 1000 + u, 39, 150) for u in range(rows)]
for _ in range(2):
    out = m.generate_batch(ps, max_length=202 + new, min_new_tokens=new, eos_token_id=vocab.speech_end_id,
                           repetition_penalty=1.1)
print(m.last_timing())
