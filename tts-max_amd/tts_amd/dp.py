"""Utterance-level data parallelism: one process per GPU, RCCL (torch.distributed "nccl"
backend on ROCm) for the only two exchange steps of the path — broadcast of the request
batch from rank 0 and gather of the generated codes back to rank 0.

Utterances are independent (no exchange inside a decode), so every rank runs its shard
end to end on its own engine.  Partitions:

* ``contiguous_shard`` — the reference's rank partition
  (tts/inference/quality_validation.py:171-182 `_select_test_combinations`);
* ``lpt_shard`` — longest-processing-time-first by expected length (prompt + max new
  tokens), which balances ragged batches better; deterministic for a given input.
"""

from __future__ import annotations

from typing import Callable, Sequence

import torch


def contiguous_shard(n_items: int, rank: int, world: int) -> list[int]:
    if world == 1:
        return list(range(n_items))
    left = (rank * n_items) // world
    right = min(((rank + 1) * n_items) // world, n_items)
    return list(range(left, right))


def lpt_shard(costs: Sequence[int], rank: int, world: int) -> list[int]:
    """Greedy LPT: items sorted by cost (desc, index asc), each to the least-loaded rank
    (ties to the lowest rank).  Returns this rank's item indices in ascending order."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    load = [0] * world
    owner = [0] * len(costs)
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        owner[i] = r
        load[r] += costs[i]
    return [i for i in range(len(costs)) if owner[i] == rank]


def _pack(prompts: Sequence[Sequence[int]], device) -> tuple[torch.Tensor, torch.Tensor]:
    lens = torch.tensor([len(p) for p in prompts], dtype=torch.int32)
    flat = torch.tensor([t for p in prompts for t in p], dtype=torch.int32)
    return lens.to(device), flat.to(device)


def broadcast_requests(prompts: Sequence[Sequence[int]] | None, device, src: int = 0) -> list[list[int]]:
    """Rank `src` passes the prompts; every rank returns the full list (two broadcasts:
    the sizes, then lengths+ids in one flat int32 buffer)."""
    import torch.distributed as dist

    rank = dist.get_rank()
    if rank == src:
        lens, flat = _pack(prompts, device)
        hdr = torch.tensor([lens.numel(), flat.numel()], dtype=torch.int64, device=device)
    else:
        hdr = torch.zeros(2, dtype=torch.int64, device=device)
    dist.broadcast(hdr, src)
    n, m = int(hdr[0]), int(hdr[1])
    buf = torch.empty(n + m, dtype=torch.int32, device=device)
    if rank == src:
        buf[:n] = lens
        buf[n:] = flat
    dist.broadcast(buf, src)
    host = buf.cpu().tolist()
    out, off = [], n
    for L in host[:n]:
        out.append(host[off:off + L])
        off += L
    return out


def gather_ragged(items: dict[int, Sequence], n_items: int, dtype: torch.dtype, device,
                  dst: int = 0) -> list[torch.Tensor] | None:
    """Each rank passes {item index: 1-D values} for the items it owns; rank `dst` returns
    all n_items in index order (CPU tensors).  One flat payload per rank (its items
    concatenated) and one int64 header [k, (index, length) * k], both padded to the longest
    rank's (one all_reduce of two sizes) and moved by one gather each: the bytes on the
    wire are the payload + 16 B per item, not n_items x the longest item per rank."""
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    keys = sorted(items)
    vals = [torch.as_tensor(items[i]).reshape(-1).to(dtype) for i in keys]
    hdr = torch.tensor([len(keys)] + [x for i, v in zip(keys, vals) for x in (i, v.numel())], dtype=torch.int64)
    pay = torch.cat(vals) if vals else torch.zeros(0, dtype=dtype)
    sizes = torch.tensor([hdr.numel(), pay.numel()], dtype=torch.int64, device=device)
    dist.all_reduce(sizes, op=dist.ReduceOp.MAX)
    H, Pn = int(sizes[0]), int(sizes[1])
    hb = torch.zeros(H, dtype=torch.int64, device=device)
    hb[:hdr.numel()] = hdr.to(device)
    pb = torch.zeros(max(Pn, 1), dtype=dtype, device=device)
    pb[:pay.numel()] = pay.to(device)
    hl = [torch.empty_like(hb) for _ in range(world)] if rank == dst else None
    pl = [torch.empty_like(pb) for _ in range(world)] if rank == dst else None
    dist.gather(hb, hl, dst=dst)
    dist.gather(pb, pl, dst=dst)
    if rank != dst:
        return None
    out: list[torch.Tensor | None] = [None] * n_items
    for h, pv in zip(hl, pl):
        h, pv = h.cpu().tolist(), pv.cpu()
        off = 0
        for j in range(h[0]):
            i, L = h[1 + 2 * j], h[2 + 2 * j]
            out[i] = pv[off:off + L].clone()
            off += L
    assert all(o is not None for o in out), "an item was not produced by any rank"
    return out


def gather_results(results: dict[int, list[int]], n_items: int, device, dst: int = 0) -> list[list[int]] | None:
    """Each rank passes {item index: generated ids}; rank `dst` receives all items in order."""
    g = gather_ragged(results, n_items, torch.int32, device, dst)
    return None if g is None else [t.tolist() for t in g]


def shard_of(prompts: Sequence[Sequence[int]], rank: int, world: int, balance: str = "contiguous",
             costs: Sequence[int] | None = None) -> list[int]:
    """This rank's item indices: the reference's contiguous blocks, or LPT by cost (default:
    prompt length)."""
    if balance == "lpt":
        return lpt_shard(list(costs) if costs is not None else [len(p) for p in prompts], rank, world)
    return contiguous_shard(len(prompts), rank, world)


def run_sharded(prompts: Sequence[Sequence[int]] | None, n_items: int, work: Callable[[list[list[int]]], list[list[int]]],
                device, balance: str = "contiguous") -> list[list[int]] | None:
    """Broadcast requests, run `work` on this rank's shard, gather to rank 0."""
    import torch.distributed as dist

    allp = broadcast_requests(prompts, device)
    mine = shard_of(allp, dist.get_rank(), dist.get_world_size(), balance)
    outs = work([allp[i] for i in mine]) if mine else []
    return gather_results({i: o for i, o in zip(mine, outs)}, len(allp), device)


def synthesize_sharded(prompts: Sequence[Sequence[int]] | None, lm, decoder, device, *, max_new: int,
                       prompt_codes: Callable[[list[int]], list[int]], to_codes: Callable[[list[int]], list[int]],
                       balance: str = "contiguous", min_new_tokens: int = 0, eos_token_id: int = -1,
                       repetition_penalty: float = 1.0, costs: Sequence[int] | None = None, wav_out=None,
                       wav_to_host: bool = True):
    """The whole DP job of BASELINE configs[3] / SURVEY §8e on this rank: broadcast the
    request batch from rank 0, generate this rank's shard (greedy, `max_length` = longest
    prompt + max_new), voice prompt codes + generated codes with the codec (one ragged
    batch), gather codes AND waveforms to rank 0.  Returns (ids, wavs) on rank 0 (lists in
    request order; the waveforms as host tensors unless wav_to_host=False), (None, None)
    elsewhere, plus this rank's (n_codes, n_items)."""
    import torch.distributed as dist

    allp = broadcast_requests(prompts, device)
    rank, world = dist.get_rank(), dist.get_world_size()
    mine = shard_of(allp, rank, world, balance, costs)
    ids, wavs = {}, {}
    if mine:
        batch = [allp[i] for i in mine]
        P = max(len(p) for p in allp)  # one max_length for every rank: per-row limits equal
        new = lm.generate_batch(batch, max_length=P + max_new, min_new_tokens=min_new_tokens,
                                eos_token_id=eos_token_id, repetition_penalty=repetition_penalty)
        utts = [prompt_codes(p) + to_codes(n) for p, n in zip(batch, new)]
        wl = decoder.decode_batch(utts, out=wav_out)  # host arrays, or views of wav_out in HBM
        for i, n, w in zip(mine, new, wl):
            ids[i] = n
            wavs[i] = torch.as_tensor(w)
    g_ids = gather_ragged(ids, len(allp), torch.int32, device)
    g_wav = gather_ragged(wavs, len(allp), torch.float32, device)
    n_codes = sum(len(v) for v in ids.values())
    if g_ids is None:
        return None, None, (n_codes, len(mine))
    if wav_to_host:  # AudioDecoder.decode's boundary: waveforms in host memory (decoding.py:84-89)
        g_wav = [w.cpu() for w in g_wav]
    return [t.tolist() for t in g_ids], g_wav, (n_codes, len(mine))
