"""Same-box A/B of codec forms: decode time of one 650-code utterance and of 32 x 650 codes (one
ragged pass), md5s of the lone utterance's waveform and of the batch, and whether utterance 0
decodes to the same samples alone and in the batch; each setting in its own child process,
alternating.
usage: python scripts/codec_ab.py ROUNDS SETTING...   (SETTING: "VAR=V,VAR2=V2" or "-" for none;
TTS_LIB_PATH=... selects a frozen library)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import hashlib, json, os, sys, time
sys.path.insert(0, os.path.join(sys.argv[1], "tts-max_amd"))
import numpy as np
import torch
from tts_amd import configs
from tts_amd.codec import MI355XAudioDecoder
carch = configs.CODEC_ARCHS["codec-24k"]
dec = MI355XAudioDecoder.synthetic(carch, seed=0xC0DEC, max_codes=660)
rng = np.random.default_rng(0)
utts = [rng.integers(0, 65536, 650).tolist() for _ in range(32)]
r = {}
for n in (1, 32):
    out = torch.empty(n * 650 * carch.samples_per_code, dtype=torch.float32, device="cuda")
    for _ in range(3):
        dec.decode_batch(utts[:n], out=out)
    torch.cuda.synchronize()
    t = []
    for _ in range(7):
        t0 = time.perf_counter()
        dec.decode_batch(utts[:n], out=out)
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1000)
    r[f"codec{n}_ms"] = round(sorted(t)[3], 3)
one = dec.decode_batch(utts[:1])
many = dec.decode_batch(utts)
r["one"] = hashlib.md5(np.concatenate(one).tobytes()).hexdigest()[:10]
r["batch"] = hashlib.md5(np.concatenate(many).tobytes()).hexdigest()[:10]
r["u0_same"] = bool(np.array_equal(one[0], many[0]))
print(json.dumps(r))
'''
rounds = int(sys.argv[1])
for rd in range(rounds):
    for setting in sys.argv[2:]:
        env = dict(os.environ)
        if setting != "-":
            for kv in setting.split(","):
                k, v = kv.split("=", 1)
                env[k] = v
        out = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
        line = out.stdout.strip().splitlines()[-1] if out.returncode == 0 else f"FAILED rc={out.returncode} {out.stderr[-800:]}"
        print(f"round {rd} {setting}: {line}", flush=True)
        if out.returncode != 0:
            sys.exit(1)
