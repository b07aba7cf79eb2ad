"""Pins the CPU oracle to the reference: the golden fixtures were produced by the reference
implementations themselves (transformers LlamaForCausalLM.generate; the reference codec
Decoder) — see oracle/make_golden.py and tests/golden/manifest.json."""

import json
import os

import numpy as np
import pytest
import torch

from oracle import codec_oracle, lm_oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _lm_cases(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    po = no = 0
    out = []
    for i, P in enumerate(z["prompt_lens"]):
        n = int(z["hf_new_lens"][i])
        out.append((z["prompt_ids"][po:po + P].tolist(), z["hf_new"][no:no + n].tolist(), int(z["max_length"][i]),
                    int(z["min_new"][i]), float(z["rep"][i]), int(z["eos"][i])))
        po += P
        no += n
    return str(z["arch"]), int(z["seed"]), out


@pytest.mark.parametrize("name", ["lm_tiny", "lm_small", "lm_tiny128"])
def test_lm_oracle_reproduces_hf_generate(name):
    from tts_amd import configs, synth

    arch, seed, cases = _lm_cases(name)
    a = configs.LM_ARCHS[arch]
    orc = lm_oracle.LlamaOracle(a, synth.lm_weights_cpu(a, seed))
    for prompt, hf_new, max_length, min_new, rep, eos in cases:
        new, margins = orc.generate(prompt, max_length, min_new, eos, rep)
        assert new == hf_new
        assert min(margins) >= 0.0


def test_manifest_records_oracle_agreement():
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    for name, m in man.items():
        if m["kind"] == "config1":  # the samples.jsonl sweep: checked by tests/test_config1.py
            assert m["n"] == 100 and m["total_new"] > 0, (name, m)
            continue
        for c in m["cases"]:
            if m["kind"] == "lm":
                # the oracle follows the reference up to the reference's first near-tie step
                # (margins below 0.25 are backend noise: exp/summation order)
                assert c["identical"] or c["agree_prefix"] >= (c["first_hf_near_tie"] or 0), (name, c)
            elif m["kind"] == "lm_chain":
                # the decisive model: HF margins >= 7.8 against a <= 1-logit HF/oracle deviation
                assert c["hf_min_margin"] >= 4 * max(c["top2_dev_vs_oracle_max"], 1.0), (name, c)
            elif m["kind"] == "codec":
                assert c["oracle_rel_l2"] < 1e-4, (name, c)
            elif m["kind"] == "encoder":
                # decisive codes: every rounded value far from a rounding boundary
                assert c["min_round_margin"] > 0.01 and c["distinct_codes"] > 1, (name, c)


@pytest.mark.parametrize("name", ["codec_24k_d2", "codec_16k"])
def test_codec_oracle_matches_reference_waveform(name):
    from tts_amd import configs, synth

    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    arch = configs.CODEC_ARCHS[str(z["arch"])]
    w = synth.codec_weights_cpu(arch, int(z["seed"]))
    T, L = int(z["lens"][0]), int(z["wav_lens"][0])
    wav = codec_oracle.decode(w, torch.tensor(z["codes"][:T]), arch.hop_length, arch.upsample_factors,
                              arch.kernel_sizes, arch.depth)[0].numpy()
    ref = z["wav"][:L]
    assert np.linalg.norm(wav - ref) / np.linalg.norm(ref) < 1e-5


def test_rope_table_matches_transformers():
    from transformers import LlamaConfig
    from transformers.models.llama.modeling_llama import LlamaRotaryEmbedding

    from tts_amd import configs
    from tts_amd.speechlm import hf_rope_table

    for arch in (configs.TTS1, configs.TTS1_MAX):
        cfg = LlamaConfig(**arch.hf_config_dict())
        rope = LlamaRotaryEmbedding(cfg)
        x = torch.zeros(1, 1, dtype=torch.bfloat16)
        cos_hf, sin_hf = rope(x, torch.arange(3000)[None])
        cos, sin = hf_rope_table(arch, 3000)
        assert torch.equal(cos, cos_hf[0]) and torch.equal(sin, sin_hf[0])


def test_fsq_and_rope_quirk_match_hf_xcodec2_port():
    """Cross-check of the restated third-party pieces against transformers' independent
    Xcodec2 port: FSQ implicit codebook and the RoPE-over-head-index quirk."""
    import importlib

    mx = importlib.import_module("transformers.models.xcodec2.modeling_xcodec2")
    cfgm = importlib.import_module("transformers.models.xcodec2.configuration_xcodec2")
    cfg = cfgm.Xcodec2Config()
    fsq = mx.Xcodec2FiniteScalarQuantization(cfg)
    idx = torch.arange(65536)
    assert torch.equal(fsq.codebook.float(), codec_oracle.fsq_codes(idx))


def test_synth_generator_known_values():
    from tts_amd import synth

    v = synth.synth_values(1, 4, 1.0)
    v2 = synth.synth_values(1, 4, 1.0, chunk=1)
    assert np.array_equal(v, v2)
    assert np.all(np.abs(v) <= 1.0)
    assert synth.tensor_seed(0x5EED, "a") != synth.tensor_seed(0x5EED, "b")


@pytest.mark.parametrize("T,k,p", [(0.8, 50, 1.0), (1.0, 50, 1.0), (0.7, 20, 0.9), (1.3, 5, 0.5), (0.8, 1, 1.0)])
def test_sample_probs_match_transformers_warpers(T, k, p):
    """The oracle's sampling distribution == transformers' warpers + softmax (the reference's
    dependency, installed here), on rows with ties, -inf (masked EOS) and a peaked head."""
    from transformers.generation.logits_process import (LogitsProcessorList, TemperatureLogitsWarper,
                                                        TopKLogitsWarper, TopPLogitsWarper)

    g = torch.Generator().manual_seed(int(T * 100) + k)
    for trial in range(4):
        s = torch.randn(1, 3000, generator=g) * 3
        s = s.to(torch.bfloat16).float()  # bf16-rounded logits: many exact ties
        s[0, 17] = float("-inf")
        if trial == 1:
            s[0, :40] = 9.0  # a tie block straddling k
        warpers = LogitsProcessorList()
        if T != 1.0:
            warpers.append(TemperatureLogitsWarper(T))
        warpers.append(TopKLogitsWarper(k))
        if p < 1.0:
            warpers.append(TopPLogitsWarper(p))
        ref = torch.softmax(warpers(None, s.clone()), dim=-1)[0]
        got = lm_oracle.sample_probs(s[0], T, k, p)
        assert torch.allclose(got, ref, atol=1e-7, rtol=0), (got - ref).abs().max()


def test_encoder_oracle_reproduces_reference():
    """oracle/encoder_oracle.py (a functional restatement of the reference Encoder after
    w2v-bert) reproduces the reference's codes on the fixture's waveforms and features."""
    from tts_amd import configs, synth
    from oracle import encoder_oracle

    z = np.load(os.path.join(GOLDEN, "encoder_16k.npz"))
    w = synth.weights_from_specs_cpu(synth.encoder_tensor_specs(configs.ENCODER), int(z["seed"]))
    filt = synth.kaiser_sinc_filter(0.25, 0.3, 12)
    wo = to = 0
    for n, T in zip(z["wav_lens"], z["T"]):
        n, T = int(n), int(T)
        with torch.no_grad():
            codes, pre = encoder_oracle.encode(w, torch.from_numpy(z["wav"][wo:wo + n]),
                                               torch.from_numpy(z["w2v"][to:to + T]), filt)
        np.testing.assert_array_equal(codes.numpy(), z["codes"][to:to + T])
        assert np.abs(pre.numpy() - z["pre_round"][to:to + T]).max() < 5e-3
        wo += n
        to += T


@pytest.mark.parametrize("name", ["lm_tts1_long", "lm_max2l_long"])
def test_long_context_fixtures_well_formed(name):
    """The decode-path teacher-forcing fixtures (transformers' cached decode, make_golden.py
    LONG_CASES): every sequence decodes its last n_last positions, crossing the decode
    attention's first pass (1,024 positions at head dim 64, 512 at head dim 128); the stored
    HF top-16 values are sorted and finite; the prompt is the reference prompt shape.  (The CPU
    oracle's agreement on these sequences is in the manifest: a 1,792-position forward is too
    slow for this suite.)"""
    import json

    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    from tts_amd import configs

    arch = configs.LM_ARCHS[str(z["arch"])]
    lens, n_last = z["lens"], int(z["n_last"])
    assert z["ids"].size == lens.sum() and z["tf_idx"].shape == (lens.size, n_last, 32)
    assert z["tf_val"].shape == z["tf_idx"].shape and np.isfinite(z["tf_val"]).all()
    top = z["tf_val"][:, :, :16]
    assert (np.diff(top, axis=-1) <= 0).all()
    assert ((z["tf_idx"] >= 0) & (z["tf_idx"] < arch.vocab_size)).all()
    pass_len = 1024 if arch.head_dim == 64 else 512
    assert int(lens.max()) > pass_len and int(lens.min()) - n_last < pass_len
    vocab = configs.vocab_for(arch)
    assert z["ids"][0] == vocab.bos_id
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))[name]
    assert man["cases"][0]["oracle_prefill_vs_hf_decode_max"] <= 0.5
