"""Measurement build (tests/ab_variants/conftest.py): the regrouped
N-player trajectory's round-2 store form (COUP_TRAJ_STAGE=0) against
coup_step launched once per step."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv, _native  # noqa: E402

KEYS = ("actions", "rewards", "step_type", "legal_mask", "current_player")


def _stepped(env, steps, buf):
    env._bind_stream()
    for t in range(steps):
        _native.check(env.lib.coup_step(env._h, None, ctypes.byref(env._slice_outputs(buf, t))))
    return buf


@pytest.mark.parametrize("n", [1501, 1502, 1503, 2048])
@pytest.mark.parametrize("players", [3, 6])
def test_regrouped_trajectory_store_forms(monkeypatch, n, players):
    """The regrouped N-player trajectory stages each step's outputs by lane
    and stores them from each lane's home thread (default) or where the lane
    is played (COUP_TRAJ_STAGE=0), on ragged batches (slices not 4-lane
    aligned) and whole ones: both equal coup_step launched once per step."""
    monkeypatch.setenv("COUP_REGROUP", "1")
    T = 40
    kw = dict(seed=7 + n, env_id_base=5 << 20, auto_reset=True, obs=False, num_players=players, episode_stats=True)
    ref = BatchedCoupEnv(n, **kw)
    br = _stepped(ref, T, ref.trajectory_buffers(T))
    for form in ("0",):
        monkeypatch.setenv("COUP_TRAJ_STAGE", form)
        env = BatchedCoupEnv(n, **kw)
        bf = env.collect_trajectory(T)
        for k in KEYS:
            assert torch.equal(bf[k], br[k]), (form, k)
        assert torch.equal(env.export_state(), ref.export_state()), form
        for a, b in zip(env.episode_stats(), ref.episode_stats()):
            assert torch.equal(a, b), form
