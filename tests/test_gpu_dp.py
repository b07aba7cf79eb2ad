"""Data-parallel synthesis with the real engine (the reference's rank partition
tts/inference/quality_validation.py:171-182): two processes on the one GPU, gloo for the
collectives (the driver's 8-GPU runs use RCCL through the same code: tts_amd/dp.py), each
with its own engine, run dp.synthesize_sharded — broadcast of the request batch, greedy
generation of the rank's shard, codec decode of prompt + generated codes, gather of codes
AND waveforms to rank 0 — and the result equals a one-process run id for id and waveform
bit for bit, under the contiguous and the LPT partition."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N_UTT, MAX_NEW = 7, 24


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, balance, q):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tts-max_amd"))
    import torch.distributed as dist

    from tts_amd import configs, dp, synth
    from tts_amd.codec import MI355XAudioDecoder
    from tts_amd.speechlm import MI355XSpeechLM

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    arch = configs.LM_ARCHS["tiny"]
    vocab = configs.vocab_for(arch)
    lm = MI355XSpeechLM.synthetic(arch, seed=11, max_batch=N_UTT, max_seq_len=256)
    dec = MI355XAudioDecoder.synthetic(configs.CODEC_ARCHS["codec-24k-d2"], seed=0xC0DEC + 3, max_codes=256)
    # ragged prompts: 5..47 text tokens, 4..60 prompt codes
    prompts = [synth.synthetic_prompt(vocab, u, 5 + 7 * u, 4 + 9 * (u % 7)) for u in range(N_UTT)] if rank == 0 else None
    lut = lm.ids_to_codes

    def to_codes(ids):  # random weights emit non-speech ids too: voice id % 65536 for those
        return [c if c >= 0 else i % 65536 for i, c in zip(ids, lut(ids))]

    ids, wavs, _ = dp.synthesize_sharded(prompts, lm, dec, torch.device("cpu"), max_new=MAX_NEW,
                                         prompt_codes=lambda p: to_codes(p[-8:]), to_codes=to_codes,
                                         balance=balance, min_new_tokens=4, eos_token_id=vocab.speech_end_id,
                                         repetition_penalty=1.1)
    if rank == 0:
        q.put((ids, [w.numpy() for w in wavs]))
    dist.destroy_process_group()


def _run(world, balance):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, balance, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = q.get(timeout=150)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("balance", ["contiguous", "lpt"])
def test_dp_two_ranks_equal_one_rank(balance):
    ids1, wav1 = _run(1, balance)
    ids2, wav2 = _run(2, balance)
    assert len(ids1) == N_UTT and all(len(i) >= 4 for i in ids1)
    assert ids2 == ids1
    for a, b in zip(wav1, wav2):
        assert a.shape == b.shape and a.size > 0
        assert np.array_equal(a, b)
