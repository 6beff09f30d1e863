"""The packed per-lane episode word (csrc/coup_episodes.h):
every step, trajectory and rollout kernel accumulates `return_sum << 8 |
episodes` (int16) or `<< 16` (int32) in place, and the bench all-gathers the
word as it stands.  Against twin envs with the int32 pair (the form every
other GPU test checks against the oracle): the word equals
bench.pack_episodes of the pair, episode_stats() unpacks to the pair, and
the records are unchanged by the form.  Reference quantity: Returns()[0]
(coup.cc:1016-1032) of every game that ends."""
import ctypes

import pytest
import torch

import bench

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv, _native  # noqa: E402


def _twins(n, width, **kw):
    return BatchedCoupEnv(n, episode_stats=True, **kw), BatchedCoupEnv(n, episode_stats=width, **kw)


def _check(pair, packed, width):
    eps, ret = pair.episode_stats()
    assert int(eps.sum()) > 0 and int((ret < 0).sum()) > 0  # negative sums exercised
    assert torch.equal(packed.export_state(), pair.export_state())
    e2, r2 = packed.episode_stats()
    assert torch.equal(e2, eps) and torch.equal(r2, ret)
    if packed._ep_fold is None:
        assert torch.equal(packed.episode_payload(), bench.pack_episodes(eps, ret, width))


@pytest.mark.parametrize("width", [2, 4])
@pytest.mark.parametrize("players", [2, 6])
@pytest.mark.parametrize("regroup", ["0", "1"], ids=["in-place", "regrouped"])
@pytest.mark.parametrize("obs", [False, True])
def test_step_word_equals_pair(monkeypatch, width, players, regroup, obs):
    """coup_step (uniform policy): in place and regrouped kernels, with and
    without observations (the c3 writer k_step<true, 9, 256, 0>), 2 and 6
    players, after settling into mixed phases."""
    if obs and regroup == "1" and players == 2:
        pytest.skip("2-player steps with observations are never regrouped")
    monkeypatch.setenv("COUP_REGROUP", regroup)
    n = 3000
    steps = min(40, BatchedCoupEnv(2, episode_stats=width, num_players=players).episode_capacity())
    pair, packed = _twins(n, width, seed=11, env_id_base=7, obs=obs, num_players=players)
    for e in (pair, packed):
        e.rollout(50)
        e.clear_episode_stats()
        for _ in range(steps):
            e.step()
    _check(pair, packed, width)
    assert packed._ep_fold is None


@pytest.mark.parametrize("width", [2, 4])
def test_caller_action_and_history_steps(width):
    """The caller-action kernels (k_step<false, ...>, SyncVectorEnv's form)
    and the history / InformationStateTensor kernel (c3i)."""
    n = 1024
    pair, packed = _twins(n, width, seed=5, obs=False, info_state=True)
    g = torch.Generator(device="cpu").manual_seed(1)
    for t in range(30):
        if t % 2:
            for e in (pair, packed):
                e.step()
        else:
            q = pair.query(obs=False)
            m = q["legal_mask"].cpu()
            acts = torch.full((n,), -1, dtype=torch.int8)
            for i in range(0, n, 3):  # every third lane acts, the rest skip
                bits = [a for a in range(18) if (int(m[i]) >> a) & 1]
                if bits:
                    acts[i] = bits[int(torch.randint(len(bits), (1,), generator=g))]
            for e in (pair, packed):
                e.step(acts)
    _check(pair, packed, width)


@pytest.mark.parametrize("width", [2, 4])
@pytest.mark.parametrize("players", [2, 6])
@pytest.mark.parametrize("regroup", ["0", "1"], ids=["in-place", "regrouped"])
def test_trajectory_word_equals_pair(monkeypatch, width, players, regroup):
    monkeypatch.setenv("COUP_REGROUP", regroup)
    n, T = 2000, 10
    pair, packed = _twins(n, width, seed=3, obs=False, num_players=players)
    for e in (pair, packed):
        e.rollout(30)
        e.clear_episode_stats()
        e.collect_trajectory(T)
    _check(pair, packed, width)


@pytest.mark.parametrize("width", [2, 4])
@pytest.mark.parametrize("players", [2, 6])
@pytest.mark.parametrize("regroup", ["0", "1"], ids=["in-place", "regrouped"])
def test_rollout_word_equals_pair(monkeypatch, width, players, regroup):
    """coup_rollout_stats.episode_word against its int32 pair."""
    monkeypatch.setenv("COUP_REGROUP", regroup)
    n = 2000
    K = 10 if players == 6 else 60
    a = BatchedCoupEnv(n, seed=9, obs=False, num_players=players)
    b = BatchedCoupEnv(n, seed=9, obs=False, num_players=players)
    sa, sb = a.new_stats(), b.new_stats(width)
    a.rollout(K, sa)
    b.rollout(K, sb)
    assert torch.equal(a.export_state(), b.export_state())
    assert torch.equal(sb["episode_word"].view(torch.int32) if width == 2 else sb["episode_word"],
                       bench.pack_episodes(sa["episodes"], sa["return_sum"], width))


def test_word_folds_past_its_capacity():
    """An int16 word holds 63 2-player steps: eager steps past that fold it
    into int32 totals first, and the totals stay exact."""
    n = 4096
    pair, packed = _twins(n, 2, seed=21, obs=False)
    assert packed.episode_capacity() == 63
    for _ in range(200):
        for e in (pair, packed):
            e.step()
    assert packed._ep_fold is not None
    _check(pair, packed, 2)
    with pytest.raises(ValueError):
        packed.episode_payload()  # the folded word is no longer the window's payload
    packed.clear_episode_stats()
    assert int(packed.episode_stats()[0].sum()) == 0


def test_word_arguments_are_checked():
    env = BatchedCoupEnv(64, seed=1, obs=False, episode_stats=True)
    word = torch.zeros(64, dtype=torch.int16, device="cuda")
    out = _native.StepOutputs(None, None, None, None, None, None, None, env.episodes.data_ptr(),
                              env.return_sum.data_ptr(), word.data_ptr(), 2)
    assert env.lib.coup_step(env._h, None, ctypes.byref(out)) == _native.COUP_E_INVALID  # both forms
    out = _native.StepOutputs(None, None, None, None, None, None, None, None, None, word.data_ptr(), 3)
    assert env.lib.coup_step(env._h, None, ctypes.byref(out)) == _native.COUP_E_INVALID  # bad width
    with pytest.raises(ValueError):
        BatchedCoupEnv(64, seed=1, obs=False, episode_stats=2, num_players=6).collect_trajectory(13)
