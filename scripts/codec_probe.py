"""Codec decode timing: one utterance of T codes, and a batch of B (lanes), 24 kHz config."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tts_amd import configs  # noqa: E402
from tts_amd.codec import MI355XAudioDecoder  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 650
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
carch = configs.CODEC_ARCHS["codec-24k"]
dec = MI355XAudioDecoder.synthetic(carch, seed=0xC0DEC, max_codes=T + 8)
rng = np.random.default_rng(0)
utts = [rng.integers(0, 65536, T).tolist() for _ in range(B)]
out = torch.empty(B * T * carch.samples_per_code, dtype=torch.float32, device="cuda")
for i in range(3):
    dec.decode_batch(utts, out=out)
torch.cuda.synchronize()
t = time.perf_counter()
for i in range(5):
    dec.decode_batch(utts, out=out)
torch.cuda.synchronize()
ms = (time.perf_counter() - t) / 5 * 1000
gf = 260.0 * T / 650 * B
print(f"codec T={T} B={B}: {ms:.2f} ms per batch, ~{gf / ms:.1f} TFLOP/s", flush=True)
