#!/usr/bin/env python
"""Benchmark: audio-codes/s + RTF of the tts.inference hot path on MI355X.

One "step" = one pass of the hot path over one batch of synthetic utterances per GPU:
greedy SpeechLM generation of N codes after a P-token prompt (prefill + N decode steps,
`max_length = P + N`, `min_new_tokens = N`, repetition penalty 1.1: the semantics of
tts/inference/inferencing.py:94-107) followed by the codec decode of each utterance's
prompt + generated codes at 24 kHz (decoding.py:84-89).  Timing boundary = the reference's
(generate + codec decode, inferencing.py:153-155,209-220).

Default workload (BASELINE.json configs[1]): TTS-1 bf16 (Llama-3.2-1B dims, V=193,856),
batch 1 per GPU, P = 200 (150 prompt codes), N = 500 codes (10 s of audio), codec 24 kHz
(hop 160, ups [3]) on 650 codes.  Random-init weights of that architecture (no checkpoint
is reachable offline); synthetic token ids of the reference prompt shape.

Multi-GPU: one process per GPU (tts_amd/dp.py synthesize_sharded).  `--gpus N` without a
launcher spawns the N ranks itself (tts_amd/launch.py; the parent never touches the GPU);
under torchrun the ranks come from the environment.  Rank 0 builds the request batch and
broadcasts it over RCCL; each rank generates and voices its contiguous shard (the
reference's rank partition, quality_validation.py:171-182); codes and waveforms are
gathered back to rank 0 (the only exchange steps of the path).  Weak scaling.

Named workloads (--workload): config2 = the default above; config3 = TTS-1 32 utterances
per GPU; config4 = TTS-1-Max 8 utterances per GPU (BASELINE configs[3]: bs=64 over 8 GPUs).

Prints ONE JSON line (rank 0).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tts-max_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MODEL_NAMES = {"tts1": "TTS-1 (Llama-3.2-1B dims, V=193856, tied)",
               "tts1-max": "TTS-1-Max (Llama-3.1-8B dims, V=193856, untied)"}


# BASELINE.json configs by name: (arch, utterances per GPU)
WORKLOADS = {"config2": ("tts1", 1), "config3": ("tts1", 32), "config4": ("tts1-max", 8)}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1, help="utterances per GPU per step")
    ap.add_argument("--arch", default="tts1")
    ap.add_argument("--codec", default="codec-24k")
    ap.add_argument("--prompt-codes", type=int, default=150)
    ap.add_argument("--text-tokens", type=int, default=39)
    ap.add_argument("--new", type=int, default=500)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=96)
    ap.add_argument("--kernel-iters", type=int, default=30)
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the N=1 secondary lines (bs=32 batched decode, bs=8 streaming latency)")
    ap.add_argument("--no-max-line", action="store_true",
                    help="distributed runs: skip the TTS-1-Max 8-per-GPU line (BASELINE configs[3])")
    ap.add_argument("--max-steps", type=int, default=2, help="timed repetitions of the TTS-1-Max sharded job")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default=None,
                    help="named BASELINE workload (sets --arch / --batch per GPU)")
    args = ap.parse_args()
    if args.workload:
        args.arch, args.batch = WORKLOADS[args.workload]

    from tts_amd import launch

    if launch.needs_spawn(args.gpus):
        # one process per GPU: spawn the ranks before anything initialises HIP here
        # (torch.cuda.device_count() does not), rank 0 prints the line
        sys.exit(launch.spawn(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                              torch.cuda.device_count()))

    from tts_amd import configs, dp, synth
    from tts_amd.codec import MI355XAudioDecoder
    from tts_amd.speechlm import MI355XSpeechLM

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # TTS_BENCH_DIST=1: the RCCL (torchrun) path even at one rank — rehearses the driver's
    # multi-GPU run (broadcast, per-rank shard, gather of codes and waveforms, MAX/SUM
    # all-reduce) on a one-GPU box
    if world > 1 or os.environ.get("TTS_BENCH_DIST") == "1":
        import torch.distributed as dist  # noqa: F811

        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        # RCCL prints its version banner to stdout when the communicator comes up: send it to
        # stderr, so rank 0's stdout stays the one JSON line
        sys.stdout.flush()
        saved_fd = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved_fd, 1)
            os.close(saved_fd)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local)

    arch = configs.LM_ARCHS[args.arch]
    carch = configs.CODEC_ARCHS[args.codec]
    vocab = configs.vocab_for(arch)
    B = args.batch
    N = args.new

    # ---- requests: rank 0 builds all world*B prompts (broadcast over RCCL by dp.synthesize_sharded)
    prompts_all = [synth.synthetic_prompt(vocab, u, args.text_tokens, args.prompt_codes) for u in range(world * B)]
    P = max(len(p) for p in prompts_all)

    max_seq = P + N + 16
    t0 = time.time()
    secondary = (world == 1 and not args.no_secondary and args.arch == "tts1" and B == 1)
    lm = MI355XSpeechLM.synthetic(arch, seed=0x5EED, device=local, max_batch=max(B, 32 if secondary else 1),
                                  max_seq_len=max_seq)
    dec = MI355XAudioDecoder.synthetic(carch, seed=0xC0DEC, device=local, max_codes=args.prompt_codes + N + 8)
    log(f"[rank {rank}] engine ready in {time.time() - t0:.1f}s")
    codes_per_utt = args.prompt_codes + N

    def one_step(B=B, local_prompts=None):
        if dist is not None and local_prompts is None:
            # rank 0's request batch broadcast over RCCL, each rank generates +
            # voices its contiguous shard, codes AND waveforms gathered to rank 0 (dp.py)
            _, wavs, (n, _) = dp.synthesize_sharded(
                prompts_all if rank == 0 else None, lm, dec, dev, max_new=N,
                prompt_codes=lambda p: synthetic_codes(lm, p[-args.prompt_codes:]),
                to_codes=lambda ids: synthetic_codes(lm, ids), balance="contiguous", min_new_tokens=N,
                eos_token_id=vocab.speech_end_id, repetition_penalty=1.1, wav_out=wav_buf)
            return n, wavs  # (rank 0: waveforms as host tensors, as AudioDecoder.decode returns them)
        prompts = local_prompts if local_prompts is not None else prompts_all[rank * B:(rank + 1) * B]
        new = lm.generate_batch(prompts, max_length=P + N, min_new_tokens=N, eos_token_id=vocab.speech_end_id,
                                repetition_penalty=1.1)
        # codec input = prompt speech codes + generated codes.  Random-init weights emit
        # non-speech ids too (a trained TTS-1 emits speech codes); every generated token is
        # voiced as one code (synthetic_codes) so the codec workload has the configured size
        utts = [synthetic_codes(lm, p[-args.prompt_codes:] + n) for p, n in zip(prompts, new)]
        # waveforms to host memory inside the timed region: the reference's boundary
        # (decoding.py:84-89 returns `.detach().cpu()`), ~1.25 MB per 10-s utterance
        wav = dec.decode_batch(utts)
        return sum(len(n) for n in new), wav

    wav_buf = torch.empty(max(B, 32 if secondary else 1) * codes_per_utt * carch.samples_per_code,
                          dtype=torch.float32, device=dev)
    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    n_codes = 0
    lm_prefill = lm_decode = 0.0
    dec_steps = 0
    for _ in range(args.steps):
        n, _ = one_step()
        n_codes += n
        a, b, k = lm.last_timing()
        lm_prefill += a
        lm_decode += b
        dec_steps += k
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    tot = torch.tensor([n_codes], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    elapsed = float(el.item())
    total_codes = float(tot.item())
    ms_per_step = 1000.0 * elapsed / args.steps
    codes_per_s = total_codes / elapsed
    audio_s = N / carch.token_rate  # seconds of audio per utterance
    rtf = (elapsed / args.steps) / audio_s  # wall per utterance-batch / audio seconds (per GPU)

    # ---- the codec leg alone (B utterances of prompt + N codes, one ragged pass), after the timed region
    rngc = np.random.default_rng(7)
    uttsc = [rngc.integers(0, 65536, size=codes_per_utt).tolist() for _ in range(B)]
    dec.decode_batch(uttsc, out=wav_buf)
    torch.cuda.synchronize()
    tc = time.perf_counter()
    for _ in range(3):
        dec.decode_batch(uttsc, out=wav_buf)
    torch.cuda.synchronize()
    codec_ms = (time.perf_counter() - tc) / 3 * 1000
    tc = time.perf_counter()
    for _ in range(3):
        dec.decode_batch(uttsc)  # (+ the copy of the waveforms to host memory)
    codec_host_ms = (time.perf_counter() - tc) / 3 * 1000

    # ---- roofline of the dominant kernel (and the whole decode step), live HIP events
    kern = {}
    ctx_mid = P + N // 2
    for k in lm.KERNELS:
        ms, by = lm.bench_kernel(k, rows=B, ctx=ctx_mid, iters=args.kernel_iters)
        kern[k] = dict(avg_ms=ms, bytes=by, gbs=by / ms / 1e6)
    # the one-row step runs QKV with the attention fused in (one launch for both), and with
    # o_proj fused behind the attention where that fits (TTS_FUSED_OPROJ, default on)
    fused, fused_o = False, False
    try:
        ms, by = lm.bench_kernel("qkv_attn", rows=B, ctx=ctx_mid, iters=args.kernel_iters)
        kern["qkv_attn"] = dict(avg_ms=ms, bytes=by, gbs=by / ms / 1e6)
        fused = True
        ms, by = lm.bench_kernel("qkv_attn_oproj", rows=B, ctx=ctx_mid, iters=args.kernel_iters)
        kern["qkv_attn_oproj"] = dict(avg_ms=ms, bytes=by, gbs=by / ms / 1e6)
        fused_o = True
    except Exception:  # noqa: BLE001 (not this shape: separate launches)
        pass
    # the greedy step's lm_head: the int8 screen + exact recheck of the tiles that can hold the
    # argmax (lm_head_screen.hip; TTS_HEAD_SCREEN=0: the full bf16 lm_head launch)
    screened = False
    if os.environ.get("TTS_HEAD_SCREEN", "1") != "0":
        try:
            for k in ("head_screened", "head_screen"):
                ms, by = lm.bench_kernel(k, rows=B, ctx=ctx_mid, iters=args.kernel_iters)
                kern[k] = dict(avg_ms=ms, bytes=by, gbs=by / ms / 1e6)
            screened = True
        except Exception:  # noqa: BLE001 (not this shape: the full lm_head)
            pass
    # per-step share: the layer kernels once per layer, the head once
    in_step = [k for k in kern if not (fused and k in ("qkv", "attention"))
               and not (fused_o and k in ("qkv_attn", "o_proj")) and k != "head_screen"
               and not (screened and k == "lm_head")]
    share = {k: kern[k]["avg_ms"] * (1 if k in ("lm_head", "head_screened") else arch.num_layers) for k in in_step}
    dom = max(share, key=share.get)
    step_ms = lm_decode / max(dec_steps, 1)
    kv_ctx_bytes = B * arch.kv_bytes_per_token() * ctx_mid
    step_bytes = arch.weight_bytes_per_step() + kv_ctx_bytes
    if screened:  # (the int8 head and its recheck instead of the bf16 lm_head's V x hidden x 2 bytes)
        step_bytes += round(kern["head_screened"]["bytes"]) - 2 * arch.vocab_size * arch.hidden_size
    # HBM traffic of that kernel from the PMC passes of scripts/pmc_traffic.sh (FETCH_SIZE x2
    # + WRITE_SIZE per launch, committed under profiles/), when one exists for this shape
    def pmc(k, rows):
        """(HBM bytes per launch, source file) of kernel k at `rows` rows, or (None, None)."""
        import glob

        pre = "" if arch.name == "tts1" else arch.name.replace("-", "") + "_"
        hits = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*pmc_{pre}{k}_{rows}.json")))
        if arch.name == "tts1":  # (not the other architectures' files)
            hits = [h for h in hits if os.path.basename(h).split("pmc_")[1].split("_")[0] not in ("tts1max",)]
        if not hits:
            return None, None
        return round(json.load(open(hits[-1]))["hbm_bytes_per_launch"]), os.path.relpath(hits[-1], ROOT)

    traffic, traffic_src = pmc(dom, B)
    kname = {"attention": "attn_decode"}.get(dom, f"wgemm/{dom}")
    roofline = dict(bound="hbm", kernel=kname,
                    achieved=round(kern[dom]["gbs"], 1), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(kern[dom]["gbs"] / HBM_PEAK_GBS, 4), traffic=traffic, traffic_source=traffic_src,
                    bytes_per_launch=kern[dom]["bytes"], avg_launch_ms=round(kern[dom]["avg_ms"], 5),
                    per_step_share_ms={k: round(v, 4) for k, v in share.items()},
                    decode_step=dict(ms=round(step_ms, 4), bytes=step_bytes,
                                     achieved_gbs=round(step_bytes / step_ms / 1e6, 1),
                                     frac=round(step_bytes / step_ms / 1e6 / HBM_PEAK_GBS, 4)),
                    kernels={k: dict(avg_ms=round(v["avg_ms"], 5), gbs=round(v["gbs"], 1), bytes=round(v["bytes"]),
                                     traffic=pmc(k, B)[0]) for k, v in kern.items()})

    sec = None
    if secondary:
        sec = {}
        # configs[2]: bs=32 batched greedy decode (+ codec), same prompt shape
        p32 = [synth.synthetic_prompt(vocab, 1000 + u, args.text_tokens, args.prompt_codes) for u in range(32)]
        one_step(32, p32)
        torch.cuda.synchronize()
        t = time.perf_counter()
        reps = max(3, args.steps)
        n32 = sum(one_step(32, p32)[0] for _ in range(reps))
        torch.cuda.synchronize()
        e32 = (time.perf_counter() - t) / reps
        a32, b32, k32 = lm.last_timing()
        # the codec leg alone: the same 32 utterances of prompt + N codes as one ragged pass
        rng32 = np.random.default_rng(32)
        utts32 = [rng32.integers(0, 65536, size=codes_per_utt).tolist() for _ in range(32)]
        dec.decode_batch(utts32, out=wav_buf)
        torch.cuda.synchronize()
        tc = time.perf_counter()
        for _ in range(3):
            dec.decode_batch(utts32, out=wav_buf)
        torch.cuda.synchronize()
        codec32_ms = (time.perf_counter() - tc) / 3 * 1000
        sec["bs32"] = dict(value=round(n32 / reps / e32, 2), unit="audio-codes/s", ms_per_step=round(1000 * e32, 3),
                           x_realtime=round(32 * N / carch.token_rate / e32, 2), lm_prefill_ms=round(a32, 3),
                           lm_decode_ms=round(b32, 3), decode_step_ms=round(b32 / max(k32, 1), 4),
                           codec_ms=round(codec32_ms, 3), codec_utterances=32, codec_codes_per_utterance=codes_per_utt,
                           codec_roofline=codec_roofline(carch, codes_per_utt, 32, codec32_ms),
                           prefill_roofline=prefill_roofline(arch, [len(q) for q in p32], a32))
        # the 32-row decode kernels: live HIP-event time, algorithmic bytes, PMC HBM traffic
        k32s = {}
        for k in list(lm.KERNELS) + (["head_screened"] if screened else []):
            try:
                ms, by = lm.bench_kernel(k, rows=32, ctx=ctx_mid, iters=args.kernel_iters)
            except Exception:  # noqa: BLE001 (the screen not on at 32 rows: the full lm_head)
                continue
            k32s[k] = dict(avg_ms=round(ms, 5), bytes=round(by), gbs=round(by / ms / 1e6, 1), traffic=pmc(k, 32)[0])
        sec["bs32"]["kernels"] = k32s
        # configs[4]: streaming, bs=8, chunks of 25 codes voiced with 25 codes of left context
        from tts_amd.streaming import StreamingSynthesizer

        p8 = p32[:8]
        pc8 = [synthetic_codes(lm, p[-args.prompt_codes:]) for p in p8]
        ss = StreamingSynthesizer(lm, dec, chunk=25, left_context=25, to_codes=lambda ids: synthetic_codes(lm, ids))
        firsts, totals = [], []
        for r in range(3):
            first = None
            t = time.perf_counter()
            for out, el in ss.stream(p8, pc8, max_length=P + N, min_new_tokens=N,
                                     eos_token_id=vocab.speech_end_id, repetition_penalty=1.1):
                if first is None:
                    first = el
            if r > 0:  # first run warms the graph for batch 8
                firsts.append(first)
                totals.append(time.perf_counter() - t)
        sec["stream_bs8"] = dict(p50_first_audio_ms=round(1000 * float(np.median(firsts)), 3),
                                 chunk_codes=25, left_context_codes=25,
                                 codes_per_s=round(8 * N / float(np.median(totals)), 2))
        # the prompt-audio encoder on the prompt's length of audio: host
        # SeamlessM4T features, then w2v-bert + acoustic + semantic + FSQ in HIP
        from tts_amd.encoder import MI355XAudioEncoder

        enc = MI355XAudioEncoder.synthetic(device=dev.index or 0)
        wav_p = torch.from_numpy(synth.synthetic_wav(5, args.prompt_codes * 320))[None]
        t = time.perf_counter()
        feats = enc.features(wav_p)
        feat_ms = (time.perf_counter() - t) * 1000
        enc.encode_from_features(wav_p[0].numpy(), feats)
        t = time.perf_counter()
        for _ in range(3):
            enc_codes = enc.encode_from_features(wav_p[0].numpy(), feats)
        sec["encoder"] = dict(prompt_s=round(wav_p.shape[1] / 16000, 3), frames=int(enc_codes.size),
                              encode_ms=round((time.perf_counter() - t) / 3 * 1000, 3),
                              host_feature_ms=round(feat_ms, 3),
                              note="w2v-bert-2.0 (16 layers) + acoustic + semantic + fusion + FSQ in HIP (fp32); "
                                   "SeamlessM4T features on the host CPU as the reference computes them")
        enc.close()
        del enc
        log(f"secondary: {sec}")

    # BASELINE configs[3] on the same ranks whenever the job is distributed: TTS-1-Max, 8
    # utterances per GPU (bs=64 over 8 GPUs), the reference's contiguous rank partition
    # (quality_validation.py:172-182) through dp.synthesize_sharded
    if dist is not None and not args.no_max_line and args.arch == "tts1":
        if sec is None:
            sec = {}
        sec["tts1max_bs64"] = tts1max_sharded(args, dist, dev, rank, world)
        if rank == 0:
            log(f"secondary tts1max_bs64: {sec['tts1max_bs64']}")

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        # (rank 0 only, after every timed region; at N > 1 the other ranks are done)
        cpu = cpu_baseline(arch, carch, prompts_all[0], N, args)

    if rank == 0:
        line = {
            "metric": "audio-codes/sec + RTF@24kHz, TTS-1 bs=1/32, at 1/2/4/8 MI355X",
            "value": round(codes_per_s, 2),
            "unit": "audio-codes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": f"synthetic (random-init {arch.name} weights, synthetic prompt ids of the reference prompt shape)",
            "rtf": round(rtf, 5),
            "x_realtime": round(1.0 / rtf * B, 2),
            "lm_prefill_ms": round(lm_prefill / args.steps, 3),
            "lm_decode_ms": round(lm_decode / args.steps, 3),
            "codec_ms": round(codec_ms, 3),
            "codec_to_host_ms": round(codec_host_ms, 3),
            "codec_roofline": codec_roofline(carch, codes_per_utt, B, codec_ms),
            "prefill_roofline": prefill_roofline(arch, [len(q) for q in prompts_all[rank * B:(rank + 1) * B]],
                                                 lm_prefill / args.steps),
            "config": {
                "workload": f"{arch.name} bf16 bs={B}/GPU: prompt {P} tokens ({args.prompt_codes} codes), "
                            f"{N} greedy codes, codec {carch.name} on {codes_per_utt} codes",
                "model": MODEL_NAMES.get(arch.name, arch.name) + f" + xcodec2-style codec {carch.name}",
                "global_batch": B * world,
                "seq_len": P + N,
                "parallelism": f"dp{world}",
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "secondary": sec,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def tts1max_sharded(args, dist, dev, rank, world, per_gpu=8):
    """BASELINE configs[3]: TTS-1-Max bf16, `per_gpu` utterances per GPU (64 global at 8
    GPUs), each rank generating + voicing its contiguous shard of rank 0's broadcast request
    batch (dp.synthesize_sharded: RCCL broadcast, ragged gathers of codes and waveforms to rank
    0), 500 codes each.  One untimed warm-up job, then `--max-steps` jobs bracketed by barrier +
    synchronize; codes/s = all ranks' codes / the slowest rank's time."""
    from tts_amd import configs, dp, synth
    from tts_amd.codec import MI355XAudioDecoder
    from tts_amd.speechlm import MI355XSpeechLM

    arch = configs.LM_ARCHS["tts1-max"]
    carch = configs.CODEC_ARCHS[args.codec]
    vocab = configs.vocab_for(arch)
    N = args.new
    G = per_gpu * world
    prompts = [synth.synthetic_prompt(vocab, 2000 + u, args.text_tokens, args.prompt_codes) for u in range(G)]
    P = max(len(p) for p in prompts)
    t0 = time.time()
    lm = MI355XSpeechLM.synthetic(arch, seed=0x5EED, device=dev.index or 0, max_batch=per_gpu,
                                  max_seq_len=P + N + 16)
    dec = MI355XAudioDecoder.synthetic(carch, seed=0xC0DEC, device=dev.index or 0,
                                       max_codes=args.prompt_codes + N + 8)
    log(f"[rank {rank}] TTS-1-Max engine ready in {time.time() - t0:.1f}s")
    wav = torch.empty(per_gpu * (args.prompt_codes + N) * carch.samples_per_code, dtype=torch.float32, device=dev)
    kw = dict(max_new=N, prompt_codes=lambda p: synthetic_codes(lm, p[-args.prompt_codes:]),
              to_codes=lambda ids: synthetic_codes(lm, ids), balance="contiguous", min_new_tokens=N,
              eos_token_id=vocab.speech_end_id, repetition_penalty=1.1, wav_out=wav)

    def job():
        _, _, (n, items) = dp.synthesize_sharded(prompts if rank == 0 else None, lm, dec, dev, **kw)
        return n, items

    job()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    n_codes, items, pre, dec_ms, steps = 0, 0, 0.0, 0.0, 0
    for _ in range(args.max_steps):
        n, items = job()
        n_codes += n
        a, b, k = lm.last_timing()
        pre, dec_ms, steps = pre + a, dec_ms + b, steps + k
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=dev)
    tot = torch.tensor([n_codes], dtype=torch.float64, device=dev)
    shard = torch.tensor([items, n_codes / args.max_steps, dec_ms / max(steps, 1)], dtype=torch.float64, device=dev)
    shards = [torch.zeros_like(shard) for _ in range(world)]
    dist.all_gather(shards, shard)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    elapsed, total = float(el.item()), float(tot.item())
    lm.close()
    dec.close()
    del lm, dec, wav
    torch.cuda.empty_cache()
    return dict(value=round(total / elapsed, 2), unit="audio-codes/s", n_gpus=world, global_batch=G,
                utterances_per_gpu=per_gpu, steps=args.max_steps, ms_per_step=round(1000 * elapsed / args.max_steps, 3),
                x_realtime=round(G * N / carch.token_rate / (elapsed / args.max_steps), 2),
                decode_step_ms=round(dec_ms / max(steps, 1), 4), lm_prefill_ms=round(pre / args.max_steps, 3),
                shards=[dict(rank=r, utterances=int(s[0].item()), codes=int(s[1].item()),
                             decode_step_ms=round(float(s[2].item()), 4)) for r, s in enumerate(shards)],
                partition="contiguous (quality_validation.py:172-182)", scaling="weak",
                model=MODEL_NAMES["tts1-max"], codec=carch.name, codes_per_utterance=N,
                workload=f"TTS-1-Max bf16, {per_gpu} utterances per GPU ({G} global), prompt {P} tokens, "
                         f"{N} greedy codes each, codec {carch.name} on {args.prompt_codes + N} codes; "
                         f"codes + waveforms gathered to rank 0 over RCCL")


BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
CODEC_PRODUCTS = 6  # bf16 MFMA products per fp32 multiply-add in the codec's split-bf16 GEMMs


def codec_flops(carch, T):
    """fp32 FLOPs of Decoder.forward (decoder.py:69-89) on T codes as the engine computes it:
    FSQ project_out (8 -> vq) + fc_post_a, embed Conv1d(k7), 4 ResnetBlocks (2 Conv1d(k3)),
    `depth` transformer blocks (c_attn, QK^T and PV over T positions, c_proj, fc1, fc2), each
    upsampler stage (ConvTranspose1d as a GEMM over every tap, ResnetBlock at the new rate),
    out_proj, the iSTFT head Linear and the windowed inverse DFT as a basis GEMM."""
    D, VQ = carch.hidden_dim, carch.vq_dim
    f = 2.0 * T * 8 * VQ + 2.0 * T * VQ * D + 2.0 * T * 7 * D * D + 4 * 2 * (2.0 * T * 3 * D * D)
    f += carch.depth * (2.0 * T * D * (3 * D + D + 4 * D + 4 * D) + 4.0 * T * T * D)
    C, t = D, T
    for u, k in zip(carch.upsample_factors, carch.kernel_sizes):
        f += 2.0 * t * C * k * (C // 2)
        C, t = C // 2, t * u
        f += 2 * (2.0 * t * 3 * C * C)
    if carch.upsample_factors:
        f += 2.0 * t * C * D
    nfft = 4 * carch.hop_length
    f += 2.0 * t * D * (nfft + 2) + 2.0 * t * (nfft + 2) * nfft
    return f


def codec_roofline(carch, T, n_utt, ms):
    """MFMA roofline of a codec pass: fp32-equivalent FLOP/s against the split-bf16 ceiling
    (dense bf16 MFMA peak / 6 products per fp32 multiply-add)."""
    fl = codec_flops(carch, T) * n_utt
    ach = fl / (ms * 1e-3) / 1e12
    peak = BF16_MFMA_PEAK_TFLOPS / CODEC_PRODUCTS
    return dict(bound="mfma", achieved=round(ach, 1), peak=round(peak, 1), unit="TFLOP/s (fp32-equivalent)",
                frac=round(ach / peak, 4), flops=fl, ms=round(ms, 3), utterances=n_utt, codes_per_utterance=T,
                note="split-bf16 GEMMs: 6 bf16 MFMA products per fp32 multiply-add; peak = 2.5 PF / 6")


def prefill_flops(arch, lens):
    """SURVEY 8(d) prefill FLOPs of a batch of prompts: 2 * (layer weights) * P per prompt +
    causal attention 2 * 2 * P^2 / 2 * (H * D) per layer + the lm_head on each prompt's last
    token (inferencing.py:94-107, the first generate iteration)."""
    H, KVH, D, HID, FF = arch.num_heads, arch.num_kv_heads, arch.head_dim, arch.hidden_size, arch.intermediate_size
    w_layers = arch.num_layers * (HID * (H + 2 * KVH) * D + H * D * HID + 3 * HID * FF + 2 * HID)
    f = 0.0
    for P in lens:
        f += 2.0 * w_layers * P + arch.num_layers * 2.0 * P * P * H * D + 2.0 * arch.vocab_size * HID
    return f


def prefill_roofline(arch, lens, ms):
    """MFMA roofline of the prefill (prefill GEMMs + causal attention + the first lm_head):
    bf16 FLOP/s against the dense bf16 MFMA peak."""
    fl = prefill_flops(arch, lens)
    ach = fl / (ms * 1e-3) / 1e12
    return dict(bound="mfma", achieved=round(ach, 1), peak=BF16_MFMA_PEAK_TFLOPS, unit="TFLOP/s", frac=round(
        ach / BF16_MFMA_PEAK_TFLOPS, 4), flops=fl, ms=round(ms, 3), prompts=len(lens), prompt_tokens=sum(lens))


def synthetic_codes(lm, ids):
    """Speech codes of `ids` through the LUT; a non-speech id (emitted by random weights)
    stands for the code id % 65536, so every token is voiced."""
    return [c if c >= 0 else i % 65536 for i, c in zip(ids, lm.ids_to_codes(ids))]


def _cpu_quota():
    """CPUs this process may actually use: the cgroup CPU quota when one is set (the GPU box
    gives a job a share of the host, while its affinity mask lists every host CPU)."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, -(-q // per))
    except (OSError, ValueError):
        pass
    return None


def _cpu_info():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return model, os.cpu_count(), avail


def cpu_baseline(arch, carch, prompt, N, args):
    """The reference's CPU path on the host cores, bounded sample of the same job: the
    SpeechLM as transformers' own LlamaForCausalLM.generate (the arithmetic the reference
    calls, tts/inference/inferencing.py:94-107: bf16, greedy, repetition penalty 1.1,
    min_new_tokens) on the same synthetic weights — prefill of the same prompt + `cpu_steps`
    generated codes — and the codec as the fp32 port (oracle/codec_oracle.py; the reference
    codec cannot travel to the box) on the whole utterance (prompt + N codes, no
    extrapolation); the LM decode is scaled to the N-code job.

    Threads: torch.set_num_threads at every core the process may run on (the affinity
    count), and at 16 (the box's CPU share per GPU) beside it; the faster
    is `value`, with the thread count that won in `cores`."""
    from oracle import codec_oracle
    from oracle.hf_ref import hf_model
    from tts_amd import configs, synth

    cpu_model, ncpu, avail = _cpu_info()
    quota = _cpu_quota()
    usable = min(avail, quota) if quota else avail
    t0 = time.time()
    model = hf_model(arch, synth.lm_weights_cpu(arch, 0x5EED))
    log(f"cpu baseline: transformers model ready in {time.time() - t0:.1f}s ({cpu_model}, affinity {avail}, "
        f"cgroup quota {quota})")
    ids = torch.tensor([prompt])
    eos = configs.vocab_for(arch).speech_end_id
    saved = torch.get_num_threads()

    def lm_leg(threads, S, max_time):
        """(prefill s, s per generated code, codes generated); the generate call stops after
        max_time seconds (HF MaxTimeCriteria), so an oversubscribed leg stays bounded."""
        torch.set_num_threads(threads)
        with torch.no_grad():
            model(ids[:, :16])  # thread-pool warm-up
            t1 = time.perf_counter()
            model(ids)  # prefill alone (its time is subtracted from the generate call below)
            t_prefill = time.perf_counter() - t1
            log(f"cpu baseline: {threads} threads: prefill {t_prefill:.2f}s")
            t2 = time.perf_counter()
            out = model.generate(input_ids=ids, max_length=len(prompt) + S, min_new_tokens=S,
                                 eos_token_id=eos, do_sample=False, repetition_penalty=1.1, max_time=max_time)
            t_gen = time.perf_counter() - t2
        n = out.shape[1] - len(prompt)
        assert n >= 2, "cpu baseline: the generate call produced fewer than 2 codes in its time budget"
        return t_prefill, max(t_gen - t_prefill, 1e-9) / (n - 1), n  # the first new code comes from the prefill

    legs = {}
    for threads in sorted({usable, 16}):
        # (above the box's CPU share the leg oversubscribes it: a short, time-bounded sample)
        S, budget = (args.cpu_steps, 60.0) if threads <= 16 else (max(16, args.cpu_steps // 4), 20.0)
        log(f"cpu baseline: {threads} threads, prefill + up to {S} codes ({budget:.0f} s budget) ...")
        t_p, t_d, n = lm_leg(threads, S, budget)
        legs[threads] = (n, t_p, t_d)
        log(f"cpu baseline: {threads} threads: {n} codes, {t_d * 1000:.1f} ms/code")
    best = min(legs, key=lambda t: legs[t][1] + (N - 1) * legs[t][2])
    # HF generate in fp32 as well as bf16 (the reference CLI loads bf16 or fp16;
    # fp32 is the CPU's native arithmetic): a shorter bounded sample at the winning thread count
    model = model.float()
    S32 = max(8, args.cpu_steps // 3)
    log(f"cpu baseline: fp32, {best} threads, prefill + up to {S32} codes (30 s budget) ...")
    t_p32, t_d32, n32 = lm_leg(best, S32, 30.0)
    log(f"cpu baseline: fp32: {n32} codes, {t_d32 * 1000:.1f} ms/code")
    del model
    torch.set_num_threads(best)
    cw = synth.codec_weights_cpu(carch, 0xC0DEC)
    T_s = args.prompt_codes + N
    t3 = time.perf_counter()
    codec_oracle.decode(cw, torch.randint(0, 65536, (T_s,)), carch.hop_length, carch.upsample_factors,
                        carch.kernel_sizes, carch.depth)
    t_codec = time.perf_counter() - t3
    torch.set_num_threads(saved)
    S, t_prefill, t_dec = legs[best]
    full = t_prefill + (N - 1) * t_dec + t_codec
    return {
        "value": round(N / full, 3),
        "unit": "audio-codes/s",
        "cores": best,
        "kind": "reference",
        "cpu": {"model": cpu_model, "nproc": ncpu, "affinity": avail, "cgroup_quota_cpus": quota,
                "usable": usable},
        "by_threads": {str(t): {"codes_per_s": round(N / (v[1] + (N - 1) * v[2] + t_codec), 3),
                                "prefill_s": round(v[1], 3), "ms_per_code": round(1000 * v[2], 2),
                                "sample_codes": v[0]} for t, v in legs.items()},
        "by_dtype": {"bf16": {"codes_per_s": round(N / full, 3), "prefill_s": round(t_prefill, 3),
                              "ms_per_code": round(1000 * t_dec, 2), "sample_codes": S, "threads": best},
                     "fp32": {"codes_per_s": round(N / (t_p32 + (N - 1) * t_d32 + t_codec), 3),
                              "prefill_s": round(t_p32, 3), "ms_per_code": round(1000 * t_d32, 2),
                              "sample_codes": n32, "threads": best}},
        "sample": (f"transformers {__import__('transformers').__version__} LlamaForCausalLM.generate (bf16, greedy, "
                   f"rep 1.1; the reference's LM call) on the same weights at {best} threads: prefill {len(prompt)} "
                   f"tokens ({t_prefill:.2f}s) + {S} generated codes ({t_dec * 1000:.1f} ms/code), extrapolated to "
                   f"{N} codes; codec as the fp32 port on the whole {T_s}-code utterance ({t_codec:.2f}s); "
                   f"value = the bf16 leg, by_dtype adds the same job in fp32 ({n32} codes sampled)"),
    }


if __name__ == "__main__":
    main()
