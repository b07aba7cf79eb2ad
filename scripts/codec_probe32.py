"""Codec decode of B utterances of T codes (24 kHz) for rocprofv3 traces.  usage: codec_probe32.py B T"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tts-max_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tts_amd import configs  # noqa: E402
from tts_amd.codec import MI355XAudioDecoder  # noqa: E402

B, T = int(sys.argv[1]), int(sys.argv[2])
carch = configs.CODEC_ARCHS["codec-24k"]
dec = MI355XAudioDecoder.synthetic(carch, seed=0xC0DEC, max_codes=T + 8)
rng = np.random.default_rng(0)
utts = [rng.integers(0, 65536, T).tolist() for _ in range(B)]
out = torch.empty(B * T * carch.samples_per_code, dtype=torch.float32, device="cuda")
for _ in range(2):
    dec.decode_batch(utts, out=out)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(3):
    dec.decode_batch(utts, out=out)
torch.cuda.synchronize()
import hashlib  # noqa: E402
md5 = hashlib.md5(out.cpu().numpy().tobytes()).hexdigest()[:10]
print(f"{B} x {T} codes: {(time.perf_counter() - t) / 3 * 1000:.2f} ms  wav md5 {md5}")
