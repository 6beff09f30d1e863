"""The multi-GPU path on CPU: world size 2 over gloo.

Each rank runs its env-id shard with the oracle as the
per-rank engine (there is no GPU here), gathers the per-lane results with
open_spiel_coup_amd.distributed.collate and takes the max-over-ranks time;
rank 0 checks the gathered records against one process running all lanes.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from open_spiel_coup_amd import distributed as D
from oracle import oracle

PER_RANK, STEPS, SEED = 192, 70, 4242


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    dev = D.init("gloo")
    r, w, _ = D.world_info()
    ref = oracle.rollout(seed=SEED, n=PER_RANK, steps=STEPS, env_id_base=D.env_id_base(r, PER_RANK),
                         want_trajectory=True)
    final = torch.from_numpy(ref["final_state"].astype(np.int64))
    rewards = torch.from_numpy(ref["rewards"][-1].astype(np.int64))
    gathered = D.collate(final)
    gathered_rw = D.collate(rewards)
    traj = D.collate(torch.from_numpy(ref["actions"].astype(np.int64)), dim=1)  # [T, B] trajectories
    # per-lane finished episodes and player-0 return sums (the bench's collective)
    eps = D.collate(torch.from_numpy(np.stack([ref["lane_episodes"], ref["lane_return_sum"]], 1)))
    t = D.max_over_ranks(float(rank + 1), dev)
    if rank == 0:
        np.save(os.path.join(out_dir, "gathered.npy"), gathered.numpy())
        np.save(os.path.join(out_dir, "gathered_rw.npy"), gathered_rw.numpy())
        np.save(os.path.join(out_dir, "traj.npy"), traj.numpy())
        np.save(os.path.join(out_dir, "eps.npy"), eps.numpy())
        with open(os.path.join(out_dir, "tmax.txt"), "w") as f:
            f.write(str(t))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_equals_single_process(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    full = oracle.rollout(seed=SEED, n=world * PER_RANK, steps=STEPS)
    np.testing.assert_array_equal(np.load(tmp_path / "gathered.npy").astype(np.uint32), full["final_state"])
    np.testing.assert_array_equal(np.load(tmp_path / "gathered_rw.npy"), full["rewards"][-1].astype(np.int64))
    np.testing.assert_array_equal(np.load(tmp_path / "traj.npy"), full["actions"].astype(np.int64))
    eps = np.load(tmp_path / "eps.npy")
    np.testing.assert_array_equal(eps[:, 0], full["lane_episodes"])
    np.testing.assert_array_equal(eps[:, 1], full["lane_return_sum"])
    assert int(eps[:, 0].sum()) == int(full["episodes_done"][0]) > 0
    assert float(open(tmp_path / "tmax.txt").read()) == 2.0


def test_env_id_base_ranges_are_disjoint():
    ranges = [range(D.env_id_base(r, 1 << 20), D.env_id_base(r, 1 << 20) + (1 << 20)) for r in range(8)]
    for a in range(8):
        for b in range(a + 1, 8):
            assert ranges[a].stop <= ranges[b].start
    assert ranges[-1].stop == 8 << 20


@pytest.mark.parametrize("world", [1])
def test_collate_single_process_is_identity(world):
    t = torch.arange(6)
    assert D.collate(t) is t
