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


def _fake_kfd(tmp_path, simd_counts):
    root = tmp_path / "nodes"
    for i, c in enumerate(simd_counts):
        d = root / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {0 if c else 16}\nsimd_count {c}\narray_count 32\n")
    return str(root)


def test_visible_gpus_from_kfd_topology(tmp_path):
    """The launcher's GPU count: KFD nodes with SIMDs,
    narrowed by ROCR_VISIBLE_DEVICES and HIP / CUDA_VISIBLE_DEVICES."""
    root = _fake_kfd(tmp_path, [0, 1024, 1024, 1024, 0])  # 2 CPU nodes, 3 GPUs
    assert bench.visible_gpus(root, env={}) == 3
    assert bench.visible_gpus(root, env={"HIP_VISIBLE_DEVICES": "0,2"}) == 2
    assert bench.visible_gpus(root, env={"CUDA_VISIBLE_DEVICES": "1"}) == 1
    assert bench.visible_gpus(root, env={"HIP_VISIBLE_DEVICES": "0,1", "CUDA_VISIBLE_DEVICES": "0"}) == 2
    assert bench.visible_gpus(root, env={"ROCR_VISIBLE_DEVICES": "GPU-aaaa,GPU-bbbb"}) == 2
    assert bench.visible_gpus(root, env={"ROCR_VISIBLE_DEVICES": "0,1", "HIP_VISIBLE_DEVICES": "1"}) == 1
    assert bench.visible_gpus(root, env={"HIP_VISIBLE_DEVICES": ""}) == 0
    assert bench.visible_gpus(root, env={"HIP_VISIBLE_DEVICES": "0,1,2,3,4,5"}) == 3
    assert bench.visible_gpus(str(tmp_path / "absent"), env={}) == 0


def test_launcher_parent_never_imports_torch(tmp_path):
    """The parent of `bench.py --gpus N` starts its ranks without importing
    torch (so it cannot initialise HIP before it starts the children): run
    the launcher in a fresh interpreter with fake ranks and check sys.modules
    there, for both backends' paths."""
    code = (
        "import sys; sys.path.insert(0, %r); import bench\n"
        "rc = bench.launch_ranks(2, ['--gpus', '2', '--batch', '10'], backend='gloo', script=%r)\n"
        "n = bench.visible_gpus()\n"
        "assert rc == 0, rc\n"
        "assert 'torch' not in sys.modules, 'the launcher imported torch'\n"
        "print('ok', n)\n") % (ROOT, FAKE)
    r = subprocess.run([sys.executable, "-c", code], env=_env(), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr
    assert "ok" in r.stdout


def test_gpus_beyond_visible_devices_exits_nonzero():
    """nccl (RCCL) runs one rank per GPU: more ranks than visible GPUs is an
    error before any rank starts (this container has none)."""
    n = bench.visible_gpus() + 1
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(max(n, 2))], env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and not r.stdout.strip()
    assert "visible GPUs" in r.stderr


@pytest.mark.parametrize("n", [0, -1])
def test_gpus_below_one_exits_nonzero(n):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n)], env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and not r.stdout.strip()
