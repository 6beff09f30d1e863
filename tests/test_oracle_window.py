"""The oracle's every-lane window driver (oc_rollout_window /
np_rollout_window, oracle.window) against the oracle's own full rollouts,
and the device-side tensor hash (tests/lane_digest.py, run here on CPU
tensors) against the driver's host hashes: the checker of the bench-size
parity tests (tests/test_gpu_every_lane.py) checked on the CPU.  Test
infrastructure only."""
import numpy as np
import pytest
import torch

from oracle import oracle
from tests import lane_digest


@pytest.mark.parametrize("auto_reset", [True, False])
def test_window_equals_rollout_2p(auto_reset):
    n, steps, frm, seed, base = 300, 70, 45, 3, 1000
    ref = oracle.rollout(seed=seed, n=n, steps=steps, env_id_base=base, auto_reset=auto_reset, want_obs=True)
    w = oracle.window(2, seed, n, steps, frm, env_id_base=base, auto_reset=auto_reset, obs_hash=True,
                      snaps=(steps, 50), stats_from=frm, threads=3, chunk=64)
    np.testing.assert_array_equal(w["actions"], ref["actions"][frm:])
    np.testing.assert_array_equal(w["rewards"], ref["rewards"][frm:])
    np.testing.assert_array_equal(w["step_type"], ref["step_type"][frm:])
    np.testing.assert_array_equal(w["legal"], ref["legal"][frm:])
    np.testing.assert_array_equal(w["snap_state"][steps], ref["final_state"])
    mid = oracle.rollout(seed=seed, n=n, steps=50, env_id_base=base, auto_reset=auto_reset, want_trajectory=False)
    np.testing.assert_array_equal(w["snap_state"][50], mid["final_state"])
    pre = oracle.rollout(seed=seed, n=n, steps=frm, env_id_base=base, auto_reset=auto_reset, want_trajectory=False)
    np.testing.assert_array_equal(w["snap_eps"][steps], ref["lane_episodes"] - pre["lane_episodes"])
    np.testing.assert_array_equal(w["snap_ret"][steps], ref["lane_return_sum"] - pre["lane_return_sum"])
    np.testing.assert_array_equal(w["snap_eps"][50], mid["lane_episodes"] - pre["lane_episodes"])
    # the device-side hash (torch, here on the CPU) of the oracle's own rows
    for t in range(steps - frm):
        got = lane_digest.tensor_hash(torch.from_numpy(ref["obs"][frm + t]))
        np.testing.assert_array_equal(got, w["obs_hash"][t], err_msg=f"step {frm + t}")
    # CurrentPlayer after each step (auto-reset lanes are never at a chance node)
    if auto_reset:
        np.testing.assert_array_equal(w["cur_player"] >= 0, True)


def test_window_info_hash_2p():
    n, steps, frm, seed = 40, 12, 9, 5
    ref = oracle.rollout(seed=seed, n=n, steps=steps, want_info=True)
    w = oracle.window(2, seed, n, steps, frm, info_hash=True, threads=2, chunk=16)
    for t in range(steps - frm):
        got = lane_digest.tensor_hash(torch.from_numpy(ref["info"][frm + t]), chunk_elems=10000)
        np.testing.assert_array_equal(got, w["info_hash"][t])


def test_hash_sees_one_float():
    x = torch.zeros(5, 2, 98)
    x[:, 0, 3] = 1.0
    h = lane_digest.tensor_hash(x)
    y = x.clone()
    y[2, 1, 97] = 1.0
    g = lane_digest.tensor_hash(y)
    assert (g[2] != h[2]).all() and (np.delete(g, 2, 0) == np.delete(h, 2, 0)).all()
    assert lane_digest.first_mismatch(g, h, "obs").startswith("obs: 1 of 5 lanes differ, first lane 2")


@pytest.mark.parametrize("players", [3, 6])
def test_window_equals_rollout_np(players):
    n, steps, frm, seed = 257, 50, 30, 2
    ref = oracle.np_rollout(players, seed=seed, n=n, steps=steps)
    w = oracle.window(players, seed, n, steps, frm, snaps=(steps,), stats_from=frm, threads=4, chunk=50)
    for k in ("actions", "rewards", "step_type", "legal", "cur_player"):
        np.testing.assert_array_equal(w[k], ref[k][frm:], err_msg=k)
    np.testing.assert_array_equal(w["snap_state"][steps], ref["final_state"])
    pre = oracle.np_rollout(players, seed=seed, n=n, steps=frm)
    np.testing.assert_array_equal(w["snap_eps"][steps], ref["lane_episodes"] - pre["lane_episodes"])
    np.testing.assert_array_equal(w["snap_ret"][steps], ref["lane_return_sum"] - pre["lane_return_sum"])
