"""Host-side logic of the synthesis composition and the decisive-parity model (CPU only)."""

import numpy as np
import torch

from tts_amd import configs, inference, synth


class _FakeLM:
    """generate() returns the prompt + a fixed continuation; ids >= 1000 are speech codes."""

    def __init__(self, cont):
        self.cont = cont
        self.calls = []

    def generate(self, input_ids=None, prompt_token_ids=None, sampling_params=None, **kw):
        if prompt_token_ids is not None:
            self.calls.append(("vllm", sampling_params))

            class O:
                pass
            o, c = O(), O()
            c.token_ids = list(self.cont)
            o.outputs = [c]
            return [o]
        self.calls.append(("hf", kw))
        return torch.tensor([input_ids[0].tolist() + list(self.cont)])

    def ids_to_codes(self, ids):
        return [i - 1000 if i >= 1000 else -1 for i in ids]


class _FakeDecoder:
    sample_rate, token_rate = 24000, 50

    def decode(self, codes):
        self.codes = codes.tolist()
        return torch.arange(len(codes) * 480, dtype=torch.float32)[None]


def test_synthesize_audio_slice_and_trim():
    """inferencing.py:145-159: keep generated[P - len(speech_ids) : -1] (the prompt's speech
    ids included, the last id dropped even when it is not EOS), drop non-speech ids, decode,
    cut int(len(speech_ids) / 50 * 24000) samples."""
    prompt = [1, 2, 3, 1005, 1006, 1007]  # three prompt speech codes at the end
    cont = [1010, 7, 1011, 1012, 99]       # 7 is a non-speech id, 99 (last) is dropped
    lm, dec = _FakeLM(cont), _FakeDecoder()
    st = inference.InferenceSettings(temperature=0.0, max_tokens=20, min_tokens=2, repetition_penalty=1.3)
    wav, t = inference.synthesize_audio(lm, dec, prompt, [5, 6, 7], speech_end_id=99, settings=st)
    assert dec.codes == [5, 6, 7, 10, 11, 12]
    assert wav.shape == (1, (6 - 3) * 480) and wav[0, 0].item() == 3 * 480
    kind, kw = lm.calls[0]
    assert kind == "hf" and kw["max_length"] == 20 and kw["min_new_tokens"] == 2 and kw["eos_token_id"] == 99
    assert kw["do_sample"] is False and kw["repetition_penalty"] == 1.3


def test_synthesize_audio_vllm_form():
    """inferencing.py:139-142: prompt codes + every speech code of the completion."""
    lm, dec = _FakeLM([1010, 1011, 99]), _FakeDecoder()
    wav, _ = inference.synthesize_audio(lm, dec, [1, 1005], [5], speech_end_id=99, use_vllm=True)
    assert dec.codes == [5, 10, 11]
    sp = lm.calls[0][1]
    assert sp.stop_token_ids == [99] and sp.max_tokens == 1792 and sp.top_k == 50 and sp.frequency_penalty == 0.3


def test_complete_prompt_drops_first_and_last():
    lm, dec = _FakeLM([1020, 1021, 99]), _FakeDecoder()
    wav = inference.complete_prompt(lm, dec, [3, 4], code_to_id=lambda c: 1000 + c, speech_start_id=500,
                                    speech_end_id=99)
    assert dec.codes == [3, 4, 20, 21]
    assert wav.shape == (1, 2 * 480)


def test_chain_rows_are_exact_in_bf16():
    """Every value the chain model writes is exactly representable in bf16 (so numpy on the
    CPU and torch on the device produce the same weights), the rows are orthogonal, and the
    chain prompts end with the lagged chain ids."""
    arch = configs.TTS1
    spec = synth.ChainSpec()
    ov = synth.chain_overrides(arch, spec)
    for name, (idx, rows) in ov.items():
        r = torch.from_numpy(rows)
        assert torch.equal(r.to(torch.bfloat16).float(), r), name
    emb = ov["model.embed_tokens.weight"][1]
    g = emb @ emb.T
    assert np.allclose(g, np.diag(np.diag(g)))  # Hadamard rows: exactly orthogonal
    vocab = configs.vocab_for(arch)
    toks = synth.chain_tokens(vocab, spec)
    lut = vocab.id_to_code()
    assert len(set(toks)) == spec.units and all(lut[t] >= 0 for t in toks)
    p = synth.chain_prompt(vocab, spec, 0, 300, 40, 150)
    assert p[-(spec.lag + 2):] == toks[300 - spec.lag - 1: 301]
