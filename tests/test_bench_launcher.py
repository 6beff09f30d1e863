"""bench.py --gpus N on the CPU: the rank launcher and
the world-size checks, which run before anything touches the GPU.

The GPU form (the real bench with --dist-backend gloo, its gathered totals
against one process over N*B lanes) is tests/test_gpu_dist.py."""
import json
import os
import subprocess
import sys
import time

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE = os.path.join(ROOT, "tests", "fake_rank.py")


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                          "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    e.update(kw)
    return e


def test_launcher_starts_ranks_and_relays_rank0_line(capfd):
    n, B = 3, 1000
    rc = bench.launch_ranks(n, ["--gpus", str(n), "--batch", str(B)], backend="gloo", script=FAKE)
    assert rc == 0
    out, err = capfd.readouterr()
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1, out  # only the JSON line on stdout; rank 0's other output goes to stderr
    line = json.loads(lines[0])
    ids = range(n * B)
    assert line == {"n_gpus": n, "lanes": n * B, "sum": sum(3 * i + 1 for i in ids)}
    assert "not JSON" in err


def test_launcher_fails_when_a_rank_fails(capfd):
    t0 = time.time()
    rc = bench.launch_ranks(2, ["--gpus", "2", "--fail-rank", "1"], backend="gloo", script=FAKE)
    assert rc != 0
    assert time.time() - t0 < 60  # rank 0, blocked in the rendezvous / collective, was stopped
    out, err = capfd.readouterr()
    assert not out.strip() and "rank 1 exited with 3" in err


def test_gpus_disagreeing_with_world_size_exits_nonzero():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=_env(WORLD_SIZE="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and not r.stdout.strip()
    assert "disagrees with WORLD_SIZE=1" in r.stderr


def test_gpus_beyond_visible_devices_exits_nonzero():
    """nccl (RCCL) runs one rank per GPU: more ranks than visible GPUs is an
    error before any rank starts (this container has none)."""
    import torch
    n = torch.cuda.device_count() + 1
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(max(n, 2))], env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and not r.stdout.strip()
    assert "visible GPUs" in r.stderr


@pytest.mark.parametrize("n", [0, -1])
def test_gpus_below_one_exits_nonzero(n):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n)], env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and not r.stdout.strip()
