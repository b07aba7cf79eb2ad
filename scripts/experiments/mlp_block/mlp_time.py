"""Live HIP-event time of the one-row MLP launch (lm_mlp1.hip) against the gate/up + down
launches it replaces, at the bench's mid context."""
import sys
sys.path.insert(0, "tts-max_amd")
from tts_amd import configs  # noqa: E402
from tts_amd.speechlm import MI355XSpeechLM  # noqa: E402

m = MI355XSpeechLM.synthetic(configs.TTS1, seed=0x5EED, max_batch=1, max_seq_len=2048)
for k in ["mlp", "gate_up", "down", "qkv_attn", "o_proj", "lm_head"]:
    ms, by = m.bench_kernel(k, rows=1, ctx=390, iters=50)
    print(f"{k:10s} {ms * 1000:9.2f} us  {by / ms / 1e6:8.1f} GB/s", flush=True)
