"""One process per GPU for `bench.py --gpus N` (and any other entry point that wants it).

The driver runs `python bench.py --gpus N` without torchrun.  When WORLD_SIZE is unset and
N > 1 the parent becomes a launcher: it never touches the GPU (torch.cuda.device_count()
does not initialise HIP on this image), spawns N fresh child processes of the same command
with the rank environment torch.distributed's env:// rendezvous reads (RANK, LOCAL_RANK,
WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_ADDR, MASTER_PORT), waits for them, and exits with the
first non-zero child status (the others are terminated).  Rank 0 prints the result line.

This mirrors the reference's rank partition of inference work (every rank owns a contiguous
block of the utterances, tts/inference/quality_validation.py:172-182); the sharding itself is
tts_amd/dp.py.
"""

from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n: int, port: int, base: dict | None = None) -> list[dict]:
    """The environment of each of the n ranks (one process per GPU, one node)."""
    if n < 1:
        raise ValueError("world size must be >= 1")
    base = dict(os.environ if base is None else base)
    out = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # the host driver supports dmabuf IPC only (RCCL / CUDA-tensor sharing across processes)
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        out.append(e)
    return out


def check_world(n: int, visible: int) -> None:
    """Refuse a world larger than the visible devices (one rank per GPU)."""
    if n < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {n})")
    if n > visible:
        raise SystemExit(f"--gpus {n} asks for more GPUs than are visible ({visible}); "
                         "one rank runs per GPU")


def needs_spawn(n: int, env: dict | None = None) -> bool:
    """True when this process must launch the ranks itself (N > 1 and no launcher set WORLD_SIZE)."""
    env = os.environ if env is None else env
    return n > 1 and "WORLD_SIZE" not in env


def spawn(n: int, argv: list[str], visible: int, poll_s: float = 0.2) -> int:
    """Run `argv` as n ranks; returns the exit status for the parent (0 = all ranks ok)."""
    check_world(n, visible)
    envs = rank_envs(n, free_port())
    procs = [subprocess.Popen(argv, env=e, start_new_session=True) for e in envs]
    status = 0
    try:
        live = set(range(n))
        while live:
            for r in sorted(live):
                rc = procs[r].poll()
                if rc is None:
                    continue
                live.discard(r)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    print(f"[launch] rank {r} exited with status {rc}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for q in live:
                        _terminate(procs[q])
            time.sleep(poll_s)
    except KeyboardInterrupt:
        for p in procs:
            _terminate(p)
        raise
    return status


def _terminate(p: subprocess.Popen) -> None:
    if p.poll() is not None:
        return
    try:
        os.killpg(p.pid, signal.SIGTERM)  # the rank's own process group (start_new_session)
    except (ProcessLookupError, PermissionError):
        pass
    try:
        p.wait(timeout=20)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except (ProcessLookupError, PermissionError):
            pass
