import os, sys, time, json
os.environ.setdefault("TTS_STEP", "1")
sys.path.insert(0, "tts-max_amd")
import torch
from tts_amd import configs, synth
from tts_amd.speechlm import MI355XSpeechLM
arch = configs.TTS1
m = MI355XSpeechLM.synthetic(arch, seed=0x5EED, max_batch=1, max_seq_len=1024)
vocab = configs.vocab_for(arch)
p = synth.synthetic_prompt(vocab, 3, 39, 150)
t = time.time()
new = m.generate_batch([p], max_length=len(p) + 64, min_new_tokens=64, eos_token_id=-1, repetition_penalty=1.1)[0]
print("gen ok", len(new), new[:12], time.time() - t, flush=True)
print(json.dumps({"ids": new}))
