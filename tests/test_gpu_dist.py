"""C5 on the HIP engine: env-id sharding over 2 processes, per-episode
returns gathered (BASELINE config 5).

Two fresh child processes (tests/dist_hip_worker.py), each initialising the
GPU itself, run libcoup_mi355x on their shards of the global env ids and
all-gather the per-lane finished-episode counts and player-0 return sums
(Returns(), coup.cc:1016-1032) with open_spiel_coup_amd.distributed.collate
over gloo -- both ranks on the box's one GPU, since RCCL refuses two ranks
on one device.  Rank 0's gathered tensors must equal a single-process HIP
run over all 2B lanes and the oracle's per-lane statistics.

The second test runs bench.py itself under torch.distributed.run with 2
ranks (--dist-backend gloo): the exact multi-GPU bench code path, whose
timed region ends with the all-gather of the per-episode returns.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B, SEED, K_FUSED, K_STEP = 3000, 2024, 200, 96


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run_ranks(cmd_for_rank, world, timeout):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd_for_rank(r), env=env, cwd=ROOT, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-3000:]
    return outs


def test_two_process_hip_shards_gather_episode_returns(tmp_path):
    import torch
    from open_spiel_coup_amd import BatchedCoupEnv

    world = 2
    _run_ranks(lambda r: [sys.executable, "-u", os.path.join(ROOT, "tests", "dist_hip_worker.py"), str(tmp_path),
                          str(B), str(SEED), str(K_FUSED), str(K_STEP)], world, timeout=100)
    assert int(np.load(tmp_path / "errors.npy")[0]) == 0
    fused_stats = np.load(tmp_path / "fused_stats.npy")
    step_stats = np.load(tmp_path / "step_stats.npy")
    n = world * B
    assert fused_stats.shape == (n, 3) and step_stats.shape == (n, 2)

    # one process over all 2B lanes, same engine
    fused = BatchedCoupEnv(n, seed=SEED, obs=False)
    stats = fused.new_stats()
    fused.rollout(K_FUSED, stats)
    single = torch.stack([stats["episodes"], stats["return_sum"], stats["length_sum"]], 1).cpu().numpy()
    np.testing.assert_array_equal(fused_stats, single)
    np.testing.assert_array_equal(np.load(tmp_path / "fused_rec.npy"), fused.export_state().cpu().numpy())
    stepped = BatchedCoupEnv(n, seed=SEED, obs=False, episode_stats=True)
    for _ in range(K_STEP):
        stepped.step()
    eps, ret = stepped.episode_stats()
    np.testing.assert_array_equal(step_stats, torch.stack([eps, ret], 1).cpu().numpy())
    np.testing.assert_array_equal(np.load(tmp_path / "step_rec.npy"), stepped.export_state().cpu().numpy())

    # the oracle, lane by lane
    ref = oracle.rollout(seed=SEED, n=n, steps=K_FUSED, want_trajectory=False)
    np.testing.assert_array_equal(fused_stats[:, 0], ref["lane_episodes"])
    np.testing.assert_array_equal(fused_stats[:, 1], ref["lane_return_sum"])
    assert int(fused_stats[:, 0].sum()) == int(ref["episodes_done"][0])
    assert int(fused_stats[:, 1].sum()) == int(ref["return_sum_p0"][0])
    ref = oracle.rollout(seed=SEED, n=n, steps=K_STEP, want_trajectory=False)
    np.testing.assert_array_equal(step_stats[:, 0], ref["lane_episodes"])
    np.testing.assert_array_equal(step_stats[:, 1], ref["lane_return_sum"])
    np.testing.assert_array_equal(np.load(tmp_path / "step_rec.npy").astype(np.uint32), ref["final_state"])


@pytest.mark.parametrize("config", ["c2", "c3"])
def test_bench_two_ranks_gloo(config):
    """bench.py's multi-GPU path (torchrun environment, env-id shards,
    barrier, per-episode all-gather, max over ranks) with 2 ranks sharing the
    GPU; the line reports the gathered episodes and no lane errors."""
    batch = 1 << 16 if config == "c3" else 1 << 14
    outs = _run_ranks(lambda r: [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config",
                                 config, "--steps", "8", "--warmup", "2", "--power-warm-ms", "0", "--gate-steps", "0",
                                 "--settle", "16",
                                 "--batch", str(batch), "--dist-backend", "gloo"], 2, timeout=110)
    lines = [ln for ln in outs[0].splitlines() if ln.startswith("{")]
    assert len(lines) == 1, outs[0][-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 2 * batch
    assert rec["lane_errors"] == 0
    assert rec["episodes"]["finished"] > 0 and rec["episodes"]["collective"].startswith("all_gather")
    assert "int16" in rec["episodes"]["collective"]  # K = 8: 2 bytes per lane
    assert -2.0 <= rec["episodes"]["mean_return_p0"] <= 2.0
    # the same 2B env ids in one process (no gate and no power warm-up, whose
    # step counts are timed: the runs play identical games): the gathered
    # totals match
    one = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "1", "--config", config,
                          "--steps", "8", "--warmup", "2", "--power-warm-ms", "0", "--gate-steps", "0",
                          "--settle", "16",
                          "--batch", str(2 * batch), "--no-cpu-baseline"], capture_output=True, text=True,
                         timeout=110, cwd=ROOT)
    assert one.returncode == 0, one.stderr[-2000:]
    single = json.loads([ln for ln in one.stdout.splitlines() if ln.startswith("{")][-1])
    assert single["config"]["hip_graph"] == rec["config"]["hip_graph"]
    assert single["config"]["gate_steps"] == rec["config"]["gate_steps"] == 0
    assert single["episodes"]["finished"] == rec["episodes"]["finished"]
    assert single["episodes"]["mean_return_p0"] == rec["episodes"]["mean_return_p0"]


@pytest.mark.parametrize("config", ["c2t", "c4t"])
def test_bench_two_ranks_gloo_trajectory(config):
    """The fused-trajectory configs through bench.py's multi-rank path: one
    coup_step_trajectory launch per rank, every step's outputs stored, the
    per-episode accumulators all-gathered."""
    batch = 1 << 14
    outs = _run_ranks(lambda r: [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config",
                                 config, "--steps", "16", "--warmup", "2", "--power-warm-ms", "0", "--gate-steps", "0",
                                 "--settle", "64",
                                 "--batch", str(batch), "--dist-backend", "gloo"], 2, timeout=110)
    lines = [ln for ln in outs[0].splitlines() if ln.startswith("{")]
    assert len(lines) == 1, outs[0][-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 2 * batch
    assert rec["config"]["fused_steps_per_launch"] == 16 and "trajectory" in rec["config"]["outputs"]
    assert rec["lane_errors"] == 0
    assert rec["episodes"]["finished"] > 0 and rec["episodes"]["collective"].startswith("all_gather")
    assert "trajectory" in rec["roofline"]["kernel"]


def test_rccl_one_rank_collectives(tmp_path):
    """The RCCL branch of collate / max_over_ranks (never reached by the
    gloo rehearsals): one fresh process, init_process_group("nccl",
    device_id=...), all_gather_into_tensor of bench.py's three payload widths
    at the headline batch, unpacked == env.episode_stats()."""
    out = tmp_path / "nccl.json"
    _run_ranks(lambda r: [sys.executable, "-u", os.path.join(ROOT, "tests", "dist_nccl_worker.py"), str(out),
                          str(1 << 20), "20"], 1, timeout=100)
    res = json.loads(out.read_text())
    assert res["backend"] == "nccl" and res["world"] == 1 and res["episodes"] > 0
    assert res["width_at_k"] == 2 and set(res["widths"]) == {"2", "4", "8"}
    assert res["widths"]["2"]["payload_bytes"] == 2 << 20
    print("\nRCCL one-rank all-gather ms:", {w: round(v["all_gather_ms"], 3) for w, v in res["widths"].items()})


def test_bench_one_rank_rccl_line():
    """bench.py --force-collective --dist-backend nccl at one rank: the
    multi-GPU line's code path over a one-rank RCCL communicator, with the
    collective tail timed (episodes.collective_ms)."""
    outs = _run_ranks(lambda r: [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--config", "c3", "--steps",
                                 "20", "--warmup", "5", "--power-warm-ms", "0", "--gate-steps", "0", "--settle", "64",
                                 "--dist-backend", "nccl", "--force-collective", "--no-cpu-baseline"], 1, timeout=110)
    rec = json.loads([ln for ln in outs[0].splitlines() if ln.startswith("{")][-1])
    ep = rec["episodes"]
    assert ep["collective_backend"].startswith("nccl") and "int16" in ep["collective"]
    assert ep["finished"] > 0 and rec["lane_errors"] == 0
    assert ep["collective_ms"] > 0  # reported, not bounded: a one-rank communicator prices no xGMI hop
    print("\nc3 one-rank RCCL line:", json.dumps({k: rec[k] for k in ("value", "ms_per_step")}), json.dumps(ep))


def _bench(args, timeout):
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT,
                       env={k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_gpus_flag_starts_the_ranks(tmp_path):
    """`bench.py --gpus 2` with no torchrun starts its 2
    rank processes itself (gloo here: both share the box's GPU) and prints
    rank 0's line with n_gpus 2; the gathered per-lane episode counts and
    return sums equal one process over the same 2B env ids."""
    batch = 1 << 14
    common = ["--config", "c2", "--steps", "8", "--warmup", "2", "--power-warm-ms", "0", "--gate-steps", "0",
              "--settle", "16"]
    two = _bench(["--gpus", "2", "--batch", str(batch), "--dist-backend", "gloo",
                  "--dump-episodes", str(tmp_path / "two.npz")] + common, timeout=140)
    assert two["n_gpus"] == 2 and two["config"]["global_batch"] == 2 * batch and two["lane_errors"] == 0
    assert len(two["episodes"]["collective_ms_ranks"]) == 2
    one = _bench(["--gpus", "1", "--batch", str(2 * batch), "--no-cpu-baseline",
                  "--dump-episodes", str(tmp_path / "one.npz")] + common, timeout=140)
    a, b = np.load(tmp_path / "two.npz"), np.load(tmp_path / "one.npz")
    for k in ("episodes", "return_sum"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert int(a["episodes"].sum()) == two["episodes"]["finished"] == one["episodes"]["finished"] > 0


def test_config5_rehearsal_eight_ranks_of_2_20(tmp_path):
    """BASELINE config 5's workload at its size -- 8 ranks
    x 2^20 lanes (2^23 games), env ids sharded by rank, the timed region
    ending in the all-gather of every lane's episode count and player-0
    return sum (Returns(), coup.cc:1016-1032) -- as a one-box rehearsal: 8
    gloo ranks share the GPU (RCCL takes one rank per GPU), launched by
    `bench.py --gpus 8`.  Rank 0's gathered arrays must equal one process over
    the 2^23 lanes, and the oracle at every rank boundary (256 lanes from
    r * 2^20 - 128).  collective_ms per rank is reported, not bounded: ranks
    sharing one GPU and gloo say nothing about xGMI."""
    B, K, W, settle, seed = 1 << 20, 20, 5, 256, 1
    common = ["--config", "c2", "--steps", str(K), "--warmup", str(W), "--power-warm-ms", "0", "--gate-steps", "0",
              "--settle", str(settle),
              "--seed", str(seed)]
    eight = _bench(["--gpus", "8", "--batch", str(B), "--dist-backend", "gloo",
                    "--dump-episodes", str(tmp_path / "eight.npz")] + common, timeout=170)
    assert eight["n_gpus"] == 8 and eight["config"]["global_batch"] == 8 * B and eight["lane_errors"] == 0
    assert "int16" in eight["episodes"]["collective"]
    one = _bench(["--gpus", "1", "--batch", str(8 * B), "--no-cpu-baseline",
                  "--dump-episodes", str(tmp_path / "one.npz")] + common, timeout=140)
    g, s = np.load(tmp_path / "eight.npz"), np.load(tmp_path / "one.npz")
    assert g["episodes"].shape == (8 * B,)
    for k in ("episodes", "return_sum"):
        np.testing.assert_array_equal(g[k], s[k], err_msg=k)
    for r in range(9):
        base = min(max(r * B - 128, 0), 8 * B - 256)
        ref = oracle.rollout(seed=seed, n=256, steps=settle + W + K, env_id_base=base, want_trajectory=False)
        pre = oracle.rollout(seed=seed, n=256, steps=settle + W, env_id_base=base, want_trajectory=False)
        np.testing.assert_array_equal(g["episodes"][base:base + 256], ref["lane_episodes"] - pre["lane_episodes"],
                                      err_msg=f"episodes at {base}")
        np.testing.assert_array_equal(g["return_sum"][base:base + 256],
                                      ref["lane_return_sum"] - pre["lane_return_sum"], err_msg=f"returns at {base}")
    print("\nconfig 5 rehearsal (8 gloo ranks x 2^20 on one GPU):",
          json.dumps({"finished": eight["episodes"]["finished"], "mean_return_p0": eight["episodes"]["mean_return_p0"],
                      "collective_ms_ranks": eight["episodes"]["collective_ms_ranks"],
                      "ms_per_step": eight["ms_per_step"]}))
