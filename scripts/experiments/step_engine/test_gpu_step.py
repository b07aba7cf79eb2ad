"""The persistent one-row decode step (lm_step.hip, opt-in TTS_STEP=1) against the per-layer
launches: the same layer stack over the same row and KV cache (tts_lm_step_probe), and the
same greedy codes.  The two paths sum fp32 in different orders, so they agree to bf16
rounding per layer, and the stack's drift stays far inside the transformers logit bar."""
import ctypes
import dataclasses
import os

import numpy as np
import pytest

from tts_amd import _lib, configs, synth

pytestmark = pytest.mark.gpu


def _model(layers):
    from tts_amd.speechlm import MI355XSpeechLM

    old = os.environ.get("TTS_STEP")
    os.environ["TTS_STEP"] = "1"
    try:
        arch = dataclasses.replace(configs.TTS1, num_layers=layers, name=f"tts1-{layers}l")
        return MI355XSpeechLM.synthetic(arch, seed=0x5EED, max_batch=1, max_seq_len=1024)
    finally:
        if old is None:
            del os.environ["TTS_STEP"]
        else:
            os.environ["TTS_STEP"] = old


def _probe(m, token, pos, path):
    a = m.arch
    n = a.hidden_size + (a.num_heads + 2 * a.num_kv_heads) * a.head_dim + a.num_heads * a.head_dim
    out = np.zeros(n, dtype=np.float32)
    _lib.check(m._lib.tts_lm_step_probe(m._h, token, pos, path, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
    return out


@pytest.mark.parametrize("path", [1, 5])  # 1: the persistent step, 5: launches + the MLP block
def test_step_one_layer_matches_launches(path):
    m = _model(1)
    if not m.step_available():
        pytest.skip("the persistent step needs 256 CUs")
    H = m.arch.hidden_size
    for pos in (0, 1, 5, 40, 700):
        a, b = _probe(m, 128300 + pos, pos, 0), _probe(m, 128300 + pos, pos, path)
        # q|k|v and the attention output bit-identical, the residual within one bf16 ulp
        np.testing.assert_array_equal(a[H:], b[H:])
        assert np.abs(a[:H] - b[:H]).max() <= 2.0 ** -7 * max(1.0, np.abs(a[:H]).max())


@pytest.mark.parametrize("path", [1, 5])
def test_step_full_stack_close_to_launches(path):
    m = _model(configs.TTS1.num_layers)
    if not m.step_available():
        pytest.skip("the persistent step needs 256 CUs")
    H = m.arch.hidden_size
    for pos in (0, 2, 40):
        a, b = _probe(m, 128300 + pos, pos, 0), _probe(m, 128300 + pos, pos, path)
        d = np.abs(a[:H] - b[:H])
        assert np.isfinite(b).all()
        assert d.max() < 0.75 and d.mean() < 0.1, (d.max(), d.mean())


@pytest.mark.parametrize("mode", [1, 2])
def test_step_chain_fixture_ids(mode):
    """Decisive ids through the persistent step: the transformers chain fixture
    (tests/golden/lm_chain.npz, TTS-1 dims at V = 193,856) at batch 1, every id."""
    import json

    import torch
    from tts_amd.speechlm import MI355XSpeechLM

    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lm_chain.npz"))
    old = os.environ.get("TTS_STEP")
    os.environ["TTS_STEP"] = "1"
    try:
        m = MI355XSpeechLM.synthetic(configs.LM_ARCHS[str(z["arch"])], seed=int(z["seed"]),
                                     chain=synth.ChainSpec(**json.loads(str(z["chain"]))), max_batch=1,
                                     max_seq_len=1024)
    finally:
        if old is None:
            del os.environ["TTS_STEP"]
        else:
            os.environ["TTS_STEP"] = old
    if not m.step_available():
        pytest.skip("the persistent step needs 256 CUs")
    m.set_step(mode)
    po = no = 0
    for i, P in enumerate(z["prompt_lens"][:4]):
        n = int(z["hf_new_lens"][i])
        prompt, ref = z["prompt_ids"][po:po + P].tolist(), z["hf_new"][no:no + n].tolist()
        po += P
        no += n
        out = m.generate(input_ids=torch.tensor([prompt]), max_length=int(z["max_length"][i]),
                         min_new_tokens=int(z["min_new"][i]), eos_token_id=int(z["eos"][i]), do_sample=False,
                         repetition_penalty=float(z["rep"][i]), top_p=1.0, temperature=0.0)
        new = out[0, len(prompt):].tolist()
        assert new == ref, (i, next(j for j, (a, b) in enumerate(zip(new + [-9], ref + [-8])) if a != b))
