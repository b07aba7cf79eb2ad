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


def gather_results(results: dict[int, list[int]], n_items: int, device, dst: int = 0) -> list[list[int]] | None:
    """Each rank passes {item index: generated ids}; rank `dst` receives all items in order.
    Variable lengths travel as one padded [n_items, Lmax+1] int32 block per rank (row i of a
    rank's block is item i if that rank owns it, else length 0), reduced by a gather."""
    import torch.distributed as dist

    world = dist.get_world_size()
    Lmax = torch.tensor([max((len(v) for v in results.values()), default=0)], dtype=torch.int64, device=device)
    dist.all_reduce(Lmax, op=dist.ReduceOp.MAX)
    L = int(Lmax.item())
    # row = [owned, len, ids...]
    blk = torch.zeros(n_items, L + 2, dtype=torch.int32, device=device)
    for i, ids in results.items():
        blk[i, 0] = 1
        blk[i, 1] = len(ids)
        if ids:
            blk[i, 2:2 + len(ids)] = torch.tensor(ids, dtype=torch.int32, device=device)
    gl = [torch.empty_like(blk) for _ in range(world)] if dist.get_rank() == dst else None
    dist.gather(blk, gl, dst=dst)
    if dist.get_rank() != dst:
        return None
    out: list[list[int]] = [[] for _ in range(n_items)]
    for g in gl:
        g = g.cpu()
        for i in range(n_items):
            if int(g[i, 0]):
                out[i] = g[i, 2:2 + int(g[i, 1])].tolist()
    return out


def run_sharded(prompts: Sequence[Sequence[int]] | None, n_items: int, work: Callable[[list[list[int]]], list[list[int]]],
                device, balance: str = "contiguous") -> list[list[int]] | None:
    """Broadcast requests, run `work` on this rank's shard, gather to rank 0."""
    import torch.distributed as dist

    allp = broadcast_requests(prompts, device)
    rank, world = dist.get_rank(), dist.get_world_size()
    if balance == "lpt":
        mine = lpt_shard([len(p) for p in allp], rank, world)
    else:
        mine = contiguous_shard(len(allp), rank, world)
    outs = work([allp[i] for i in mine]) if mine else []
    return gather_results({i: o for i, o in zip(mine, outs)}, len(allp), device)
