"""Host-side logic (CPU): vocabulary layout, configs, sharding, and the world_size-2
data-parallel path over gloo (the same code runs over RCCL on the GPU box)."""

import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tts_amd import configs, dp, synth


def test_speech_vocab_layout_matches_reference_tokenizer_build():
    """tokenization.py:36-61 adds sorted() speech/control tokens after the 128,256 base ids
    (ids probed in SURVEY Appendix A3)."""
    v = configs.TTS_VOCAB
    ids = v.token_ids()
    assert ids["<|s_0|>"] == 128256
    assert ids["<|s_1|>"] == 139367
    assert ids["<|s_65535|>"] == 189960
    assert v.speech_end_id == 193794
    assert v.speech_start_id == 193795
    assert 128256 + len(ids) + 56 == v.total
    lut = v.id_to_code()
    assert lut[128256] == 0 and lut[139367] == 1 and lut[193794] == -1 and lut[5] == -1
    assert (lut >= 0).sum() == 65536


def test_tokenizer_json_lut(tmp_path):
    from tts_amd.speechlm import id_to_code_from_tokenizer_json

    tj = {"added_tokens": [{"id": 10, "content": "<|s_7|>"}, {"id": 11, "content": "<|speech_end|>"},
                           {"id": 12, "content": "<|s_65535|>"}], "model": {"vocab": {"a": 0}}}
    p = tmp_path / "tokenizer.json"
    p.write_text(json.dumps(tj))
    lut = id_to_code_from_tokenizer_json(str(p), 16)
    assert lut[10] == 7 and lut[12] == 65535 and lut[11] == -1 and lut[0] == -1


def test_codec_config_model_type_optional(tmp_path):
    p = tmp_path / "model_config.json"
    p.write_text(json.dumps({"sample_rate": 16000, "token_rate": 50, "hop_length": 320,
                             "upsample_factors": None, "kernel_sizes": None}))
    a = configs.CodecArch.from_json(str(p))
    assert a.samples_per_code == 320 and a.upsample_factors == ()
    assert configs.CODEC_24K.samples_per_code == 480 and configs.CODEC_48K.samples_per_code == 960


def test_weight_bytes_match_survey():
    assert configs.TTS1.weight_bytes_per_step() == 2740326400  # SURVEY 8(d) W_read (norm weights included)
    assert configs.TTS1.kv_bytes_per_token() == 32768
    assert configs.TTS1_MAX.kv_bytes_per_token() == 131072


def test_synthetic_prompt_shape():
    v = configs.TTS_VOCAB
    p = synth.synthetic_prompt(v, 0, 39, 150)
    assert p[0] == v.bos_id and v.speech_start_id in p and len(p) == 1 + 8 + 1 + 39 + 3 + 150
    lut = v.id_to_code()
    assert all(lut[t] >= 0 for t in p[-150:])


def test_shards_cover_everything_once():
    for n in (0, 1, 7, 64, 100):
        for world in (1, 2, 3, 8):
            got = sorted(i for r in range(world) for i in dp.contiguous_shard(n, r, world))
            assert got == list(range(n))
            costs = [(i * 37) % 11 + 1 for i in range(n)]
            got = sorted(i for r in range(world) for i in dp.lpt_shard(costs, r, world))
            assert got == list(range(n))
    # LPT balances: max load within one item of the ideal
    costs = [50, 49, 30, 30, 20, 10, 10, 5]
    loads = [sum(costs[i] for i in dp.lpt_shard(costs, r, 2)) for r in range(2)]
    assert max(loads) - min(loads) <= max(costs)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, balance, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    prompts = [[i] * (1 + i % 5) for i in range(11)] if rank == 0 else None

    def work(batch):  # stand-in for the engine: deterministic per-utterance output
        return [[t * 2 + len(p) for t in p] + [len(p)] for p in batch]

    out = dp.run_sharded(prompts, 11, work, torch.device("cpu"), balance=balance)
    # float payloads (waveforms) through the same ragged gather: item i = i * 0.5 + [0, 1, ...]
    mine = dp.shard_of([[0] * (1 + i % 5) for i in range(11)], rank, world, balance)
    fl = dp.gather_ragged({i: torch.arange(3 + 7 * (i % 4), dtype=torch.float32) + 0.5 * i for i in mine}, 11,
                          torch.float32, torch.device("cpu"))
    if rank == 0:
        q.put((out, [f.tolist() for f in fl]))
    dist.destroy_process_group()


@pytest.mark.parametrize("balance,world", [("contiguous", 2), ("lpt", 2), ("contiguous", 12)])
def test_dp_world2_gloo_equals_single(balance, world):
    """world 12 > 11 requests: one rank owns nothing and still joins every collective."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, balance, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
    prompts = [[i] * (1 + i % 5) for i in range(11)]
    ref = [[t * 2 + len(p) for t in p] + [len(p)] for p in prompts]
    assert out[0] == ref
    assert out[1] == [(torch.arange(3 + 7 * (i % 4), dtype=torch.float32) + 0.5 * i).tolist() for i in range(11)]


def test_codes_format_roundtrip_matches_reference_reader(tmp_path):
    """tts_amd.codes_io reads the reference's layout (raw int32 memmap + np.save'd offsets,
    data_vectorizer.py:122-146 / data_utils.py:106-148) back exactly."""
    import numpy as np

    from tts_amd import codes_io

    rng = np.random.default_rng(0)
    utts = [rng.integers(0, 65536, n).tolist() for n in (5, 1, 17, 40)]
    codes_io.write_codes(str(tmp_path), "train", utts, rank=3)
    # the reference reader's arithmetic, verbatim in spirit: memmap + index spans
    raw = np.memmap(tmp_path / "train_codes_3.npy", dtype=np.int32, mode="r")
    idx = np.load(tmp_path / "train_codes_index_3.npy")
    assert idx.tolist() == [0, 5, 6, 23] and raw.shape[0] == 63
    codes, spans = codes_io.read_codes(str(tmp_path), "train", rank=3)
    assert [codes[l:r].tolist() for l, r in spans] == utts
    assert list(codes_io.batches(spans, 2, 20)) == [[0, 1], [2]]  # 40 > max_codes: skipped
