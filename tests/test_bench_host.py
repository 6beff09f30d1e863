"""bench.py's host logic on the CPU: the collective's payload packing at the
limits of each width, and the config table."""
import pytest
import torch

import bench


@pytest.mark.parametrize("players,steps", [(2, 20), (2, 63), (6, 12), (2, 64), (6, 100), (2, 1000), (2, 5000)])
def test_episode_payload_round_trip(players, steps):
    B = 4096
    width = bench.payload_width(players, steps, B)
    assert width == (2 if 2 * (players - 1) * steps <= 127 else 4 if steps <= 1000 else 8)
    g = torch.Generator().manual_seed(steps)
    eps = torch.randint(0, steps + 1, (B,), generator=g, dtype=torch.int32)
    bound = 2 * (players - 1) * eps
    ret = (torch.rand(B, generator=g) * (2 * bound + 1)).to(torch.int32) - bound
    eps[:2] = steps  # the extremes
    ret[0], ret[1] = 2 * (players - 1) * steps, -2 * (players - 1) * steps
    p = bench.pack_episodes(eps, ret, width)
    assert p.element_size() * p.numel() == width * B
    # the collective concatenates ranks: unpack a 3-rank gather
    gathered = torch.cat([p, p, p])
    e2, r2 = bench.unpack_episodes(gathered, width)
    assert torch.equal(e2, eps.repeat(3)) and torch.equal(r2, ret.repeat(3))


def test_config_table():
    for name, (batch, obs, info, fused, nbytes, workload, players) in bench.CONFIGS.items():
        assert batch > 0 and nbytes > 0 and players in (2, 6)
        assert fused in (False, "rollout", "traj")
        assert not (fused and (obs or info)), name  # the fused kernels write no tensors
    assert bench.CONFIGS["c3"][4] == 824
