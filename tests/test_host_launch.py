"""bench.py --gpus N: the one-process-per-GPU launcher (tts_amd/launch.py), on CPU.

The driver runs `python bench.py --gpus N` without torchrun; the parent must spawn N ranks
with the env:// rendezvous variables and never touch the GPU itself.  Here the ranks are
small gloo programs: their world, ranks and an all-reduce prove the environment is right."""

import os
import subprocess
import sys
import textwrap

import pytest

from tts_amd import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 8])
def test_rank_envs(n):
    envs = launch.rank_envs(n, 29555, base={"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert len(envs) == n
    for r, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == str(n)
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/bin"
    assert len({e["RANK"] for e in envs}) == n


def test_world_checks():
    launch.check_world(8, 8)
    with pytest.raises(SystemExit, match="more GPUs than are visible"):
        launch.check_world(8, 1)
    with pytest.raises(SystemExit):
        launch.check_world(0, 8)
    assert launch.needs_spawn(2, {}) and not launch.needs_spawn(1, {})
    assert not launch.needs_spawn(8, {"WORLD_SIZE": "8"})  # under torchrun: ranks already exist


RANK_PROG = textwrap.dedent("""
    import os, sys, torch, torch.distributed as dist
    dist.init_process_group("gloo")
    r, n = dist.get_rank(), dist.get_world_size()
    assert r == int(os.environ["LOCAL_RANK"]) and n == int(os.environ["WORLD_SIZE"])
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    assert t.item() == n * (n + 1) / 2
    if r == 0:
        print("RESULT", n, int(t.item()), flush=True)
    fail = int(sys.argv[1]) if len(sys.argv) > 1 else -1
    dist.destroy_process_group()
    sys.exit(3 if r == fail else 0)
""")


def _run_launcher(tmp_path, n, fail=-1):
    prog = tmp_path / "rank.py"
    prog.write_text(RANK_PROG)
    drv = tmp_path / "drv.py"
    drv.write_text(textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {os.path.join(ROOT, 'tts-max_amd')!r})
        from tts_amd import launch
        sys.exit(launch.spawn({n}, [sys.executable, {str(prog)!r}, "{fail}"], visible=8))
    """))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    return subprocess.run([sys.executable, str(drv)], capture_output=True, text=True, timeout=300, env=env)


def test_spawn_two_ranks_gloo(tmp_path):
    p = _run_launcher(tmp_path, 2)
    assert p.returncode == 0, p.stderr
    assert "RESULT 2 3" in p.stdout


def test_spawn_propagates_rank_failure(tmp_path):
    p = _run_launcher(tmp_path, 2, fail=1)
    assert p.returncode == 3, (p.returncode, p.stderr)


def test_bench_refuses_more_gpus_than_visible():
    """No GPU here: `bench.py --gpus 2` must refuse before any rank starts."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=300, env=env)
    assert p.returncode != 0 and "more GPUs than are visible" in p.stderr
