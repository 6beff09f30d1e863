"""coup_step_trajectory: `steps` uniform env steps in one launch with every
step's outputs in [T][B] buffers, against `steps` coup_step launches."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv, _native  # noqa: E402

KEYS = ("actions", "rewards", "step_type", "legal_mask", "current_player")


def _stepped(env, steps, buf):
    """The same trajectory through one coup_step per slice."""
    env._bind_stream()
    for t in range(steps):
        _native.check(env.lib.coup_step(env._h, None, ctypes.byref(env._slice_outputs(buf, t))))
    return buf


@pytest.mark.parametrize("regroup", ["0", "1"], ids=["steps-in-place", "steps-regrouped"])
@pytest.mark.parametrize("auto_reset", [True, False])
@pytest.mark.parametrize("players,generic", [(2, False), (2, True), (3, False), (6, False)],
                         ids=["2p", "2p-generic", "3p", "6p"])
def test_trajectory_equals_steps(monkeypatch, regroup, auto_reset, players, generic):
    """Every output of every step, the final records and the per-episode
    accumulators equal those of coup_step launched once per step (in place
    or regrouped by decision), over three consecutive collections."""
    monkeypatch.setenv("COUP_REGROUP", regroup)
    n, T, seed = 1500, 48, 31 + players
    kw = dict(seed=seed, env_id_base=1 << 20, auto_reset=auto_reset, obs=False, num_players=players,
              generic=generic, episode_stats=True)
    fused, ref = BatchedCoupEnv(n, **kw), BatchedCoupEnv(n, **kw)
    bf, br = fused.trajectory_buffers(T), ref.trajectory_buffers(T)
    assert fused._fused_trajectory(bf)
    last = 0
    for rep in range(3):
        fused.collect_trajectory(T, bf)
        _stepped(ref, T, br)
        for k in KEYS:
            assert torch.equal(bf[k], br[k]), (rep, k)
        assert torch.equal(fused.export_state(), ref.export_state()), rep
        for a, b in zip(fused.episode_stats(), ref.episode_stats()):
            assert torch.equal(a, b), rep
        last += int((bf["step_type"] == 2).sum())
    assert last > 0
    assert fused.error_count() == ref.error_count() == 0


@pytest.mark.parametrize("players", [2, 6])
def test_trajectory_graph_and_full_batch(players):
    """capture_trajectory records the single launch in a HIP graph; at the
    2^20 benchmark batch the fused trajectory (2 players: lanes in place;
    6: regrouped by decision every step) equals the regrouped per-step
    kernels on sampled lanes, after settling into mixed game phases."""
    n, T = 1 << 20, 24
    a = BatchedCoupEnv(n, seed=3, auto_reset=True, obs=False, episode_stats=True, num_players=players)
    b = BatchedCoupEnv(n, seed=3, auto_reset=True, obs=False, episode_stats=True, num_players=players)
    a.rollout(40)
    b.rollout(40)
    g, buf = a.capture_trajectory(T)
    g.replay()
    rb = _stepped(b, T, b.trajectory_buffers(T))
    lanes = torch.arange(0, n, 4099, device=buf["actions"].device)
    for k in KEYS:
        assert torch.equal(buf[k][:, lanes], rb[k][:, lanes]), k
    assert torch.equal(a.export_state(), b.export_state())
    assert torch.equal(a.episodes, b.episodes) and torch.equal(a.return_sum, b.return_sum)


def test_trajectory_with_tensors_and_refusals():
    """With observation / information-state slices coup_step_trajectory runs
    one coup_step per slice inside the library (the rules-trajectory split
    step from 2^20 lanes: tests/test_gpu_step_many.py), equal to stepping slice by
    slice; a history env without tensors and negative steps are refused."""
    kw = dict(seed=1, obs=True, episode_stats=True)
    env, ref = BatchedCoupEnv(64, **kw), BatchedCoupEnv(64, **kw)
    buf, rb = env.trajectory_buffers(4), ref.trajectory_buffers(4)
    assert env._fused_trajectory(buf)
    env.collect_trajectory(4, buf)
    _stepped(ref, 4, rb)
    for k in KEYS + ("obs",):
        assert torch.equal(buf[k], rb[k]), k
    assert torch.equal(env.export_state(), ref.export_state())
    hist = BatchedCoupEnv(64, seed=1, obs=False, info_state=True, episode_stats=True)
    href = BatchedCoupEnv(64, seed=1, obs=False, info_state=True, episode_stats=True)
    hb, hr = hist.trajectory_buffers(4), href.trajectory_buffers(4)
    assert "info_state" in hb and hist._fused_trajectory(hb)
    hist.collect_trajectory(4, hb)
    _stepped(href, 4, hr)
    for k in KEYS + ("info_state",):
        assert torch.equal(hb[k], hr[k]), k
    assert hist.lib.coup_step_trajectory(hist._h, 4, None) == _native.COUP_E_INVALID
    assert env.lib.coup_step_trajectory(env._h, -1, None) == _native.COUP_E_INVALID
    bad = _native.StepOutputs(buf["actions"].data_ptr(), None, None, None, None, None, None,
                              env.episodes.data_ptr(), None, None, 0)  # episodes without return_sum
    assert env.lib.coup_step_trajectory(env._h, 4, ctypes.byref(bad)) == _native.COUP_E_INVALID
    assert env.lib.coup_step_many(env._h, 4, ctypes.byref(bad)) == _native.COUP_E_INVALID


@pytest.mark.parametrize("n", [1501, 1502, 1503, 2048])
@pytest.mark.parametrize("players", [3, 6])
def test_regrouped_trajectory_store_forms(monkeypatch, n, players):
    """The regrouped N-player trajectory stages each step's outputs by lane
    and stores them from each lane's home thread (default) or where the lane
    is played (COUP_TRAJ_STAGE=0: the measurement build,
    tests/ab_variants/test_ab_trajectory.py), on ragged batches (slices not
    4-lane aligned) and whole ones: equal to coup_step launched once per step."""
    monkeypatch.setenv("COUP_REGROUP", "1")
    T = 40
    kw = dict(seed=7 + n, env_id_base=5 << 20, auto_reset=True, obs=False, num_players=players, episode_stats=True)
    ref = BatchedCoupEnv(n, **kw)
    br = _stepped(ref, T, ref.trajectory_buffers(T))
    for form in ("1",):
        monkeypatch.setenv("COUP_TRAJ_STAGE", form)
        env = BatchedCoupEnv(n, **kw)
        bf = env.collect_trajectory(T)
        for k in KEYS:
            assert torch.equal(bf[k], br[k]), (form, k)
        assert torch.equal(env.export_state(), ref.export_state()), form
        for a, b in zip(env.episode_stats(), ref.episode_stats()):
            assert torch.equal(a, b), form
