"""The synthesis composition and the checkpoint loaders, through the engine.

* ``tts_amd.inference.synthesize_audio`` against tests/golden/synth_tiny.npz, which the
  reference's own ``_synthesize_audio`` (tts/inference/inferencing.py:110-159) produced:
  transformers' generate on the tiny LM, the slice ``[P - len(speech_ids) : -1]`` (last id
  dropped even on a length stop), the id -> code parse, the reference codec loaded by its
  own ``decoding.create``, and the prompt-audio trim.  Greedy ids are decisive for this LM
  (HF margins >= 6, manifest lm_tiny), the waveform is compared at the codec tolerance.
* ``MI355XSpeechLM.from_pretrained`` on a serving directory in the layout of
  tools/serving/convert_checkpoint.py (config.json, *.safetensors, tokenizer.json,
  generation_config.json), in bf16 and in the fp16 the serving CLI loads
  (tools/serving/inference.py:103-107; converted to bf16 on load).
"""

import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_synthesize_audio_matches_reference_composition():
    from tts_amd import configs, inference
    from tts_amd.codec import MI355XAudioDecoder
    from tts_amd.speechlm import MI355XSpeechLM

    z = np.load(os.path.join(GOLDEN, "synth_tiny.npz"))
    arch = configs.LM_ARCHS[str(z["lm_arch"])]
    vocab = configs.vocab_for(arch)
    lm = MI355XSpeechLM.synthetic(arch, seed=int(z["lm_seed"]), max_batch=1, max_seq_len=512)
    dec = MI355XAudioDecoder.synthetic(configs.CODEC_ARCHS[str(z["codec_arch"])], seed=int(z["codec_seed"]),
                                       max_codes=256)
    po = so = wo = 0
    for i, P in enumerate(z["prompt_lens"]):
        prompt = z["prompt_ids"][po:po + P].tolist()
        n_sp = int(z["speech_lens"][i])
        speech_ids = z["speech_ids"][so:so + n_sp].tolist()
        new, min_new, rep = z["settings"][i]
        st = inference.InferenceSettings(temperature=0.0, max_tokens=P + int(new), min_tokens=int(min_new),
                                         repetition_penalty=float(rep))
        wav, t_dec = inference.synthesize_audio(lm, dec, prompt, speech_ids, vocab.speech_end_id, st)
        L = int(z["wav_lens"][i])
        ref = z["wav"][wo:wo + L]
        assert wav.shape == (1, L) and wav.dtype == torch.float32 and t_dec >= 0
        rel = np.linalg.norm(wav[0].numpy() - ref) / max(np.linalg.norm(ref), 1e-30)
        assert rel <= 1e-4, (i, rel)
        po += P
        so += n_sp
        wo += L
    lm.close()
    dec.close()


def _write_serving_dir(path, arch, weights, dtype, vocab):
    from safetensors.torch import save_file

    os.makedirs(path)
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(arch.hf_config_dict(), f)
    sd = {k: v.to(dtype).contiguous() for k, v in weights.items()}
    if arch.tie_word_embeddings:
        sd.pop("lm_head.weight", None)
    save_file(sd, os.path.join(path, "model.safetensors"))
    lut = vocab.id_to_code()
    added = [{"id": int(i), "content": f"<|s_{int(c)}|>", "special": False} for i, c in enumerate(lut) if c >= 0]
    added.append({"id": vocab.speech_end_id, "content": "<|speech_end|>", "special": False})
    with open(os.path.join(path, "tokenizer.json"), "w") as f:
        json.dump({"added_tokens": added, "model": {"vocab": {}}}, f)
    with open(os.path.join(path, "generation_config.json"), "w") as f:
        json.dump({"eos_token_id": vocab.speech_end_id}, f)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_from_pretrained_serving_dir(tmp_path, dtype):
    """A serving directory round trip reproduces transformers' greedy ids (lm_tiny golden)
    and the LUT / EOS of its tokenizer and generation config."""
    from tts_amd import configs, synth
    from tts_amd.speechlm import MI355XSpeechLM

    z = np.load(os.path.join(GOLDEN, "lm_tiny.npz"))
    arch = configs.LM_ARCHS[str(z["arch"])]
    vocab = configs.vocab_for(arch)
    w = synth.lm_weights_cpu(arch, int(z["seed"]))
    d = str(tmp_path / "tiny_serving")
    _write_serving_dir(d, arch, w, dtype, vocab)
    m = MI355XSpeechLM.from_pretrained(d, max_batch=1, max_seq_len=256)
    assert m.generation_config.eos_token_id == vocab.speech_end_id
    assert m.ids_to_codes([vocab.base_vocab + 5, 7]) == [5, -1]
    P = int(z["prompt_lens"][0])
    prompt = z["prompt_ids"][:P].tolist()
    n = int(z["hf_new_lens"][0])
    out = m.generate(input_ids=torch.tensor([prompt]), max_length=int(z["max_length"][0]),
                     min_new_tokens=int(z["min_new"][0]), do_sample=False, repetition_penalty=float(z["rep"][0]),
                     temperature=0.0)  # eos from generation_config.json
    assert out[0, P:].tolist() == z["hf_new"][:n].tolist()
    m.close()
