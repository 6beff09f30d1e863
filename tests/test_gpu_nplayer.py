"""GPU parity of the N-player extension (csrc/coup_nplayer.hip, N = 2..6)
with its CPU specification (oracle/coup_nplayer.c).

The reference is 2-player only, so N > 2 is "parity unpinned" with respect
to the reference: these tests pin the kernels to the written specification.
At N = 2 the N-player engine (COUP_FLAG_GENERIC) is also checked against
the 2-player engine and the 2-player oracle, which the reference's golden
vectors pin.  Bit-exact throughout (integers and small-integer floats)."""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv  # noqa: E402


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("regroup", ["1", "0"], ids=["regrouped", "in-place"])
@pytest.mark.parametrize("n_players", [2, 3, 4, 5, 6])
@pytest.mark.parametrize("auto_reset", [True, False])
def test_uniform_steps_match_spec(monkeypatch, n_players, auto_reset, regroup):
    """coup_step (uniform policy) == np_rollout: actions, rewards [B, N],
    step types, legal masks, ObservationTensor [B, N, 49N] at every step and
    the final 32-byte records; step kernel with the lanes regrouped by
    decision (coup_regroup.h, the default from 2^18 lanes) and in place."""
    monkeypatch.setenv("COUP_REGROUP", regroup)
    n, steps, seed, base = 512, 200, 40 + n_players, 7000
    ref = oracle.np_rollout(n_players, seed=seed, n=n, steps=steps, env_id_base=base, auto_reset=auto_reset,
                            want_obs=True)
    env = BatchedCoupEnv(n, seed=seed, env_id_base=base, auto_reset=auto_reset, obs=True, num_players=n_players,
                         generic=True)
    assert env.state_words == 8
    for t in range(steps):
        o = env.step()
        np.testing.assert_array_equal(_np(o["actions"]), ref["actions"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(_np(o["rewards"]), ref["rewards"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(_np(o["step_type"]), ref["step_type"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(_np(o["legal_mask"]).astype(np.uint32), ref["legal"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(_np(o["obs"]), ref["obs"][t], err_msg=f"step {t}")
    np.testing.assert_array_equal(_np(env.export_state()).astype(np.uint32), ref["final_state"])
    assert env.error_count() == 0


def test_generic_engine_equals_two_player_engine():
    """At N = 2 the N-player kernels reproduce the 2-player kernels (and so
    the reference): same per-step outputs for 300 steps of 4096 lanes."""
    n, steps, seed = 4096, 300, 77
    a = BatchedCoupEnv(n, seed=seed, obs=True)
    b = BatchedCoupEnv(n, seed=seed, obs=True, generic=True)
    for t in range(steps):
        oa, ob = a.step(), b.step()
        for k in ("actions", "rewards", "step_type", "legal_mask", "current_player", "obs"):
            assert torch.equal(oa[k], ob[k]), (t, k)
    assert a.error_count() == 0 and b.error_count() == 0


@pytest.mark.parametrize("regroup", ["1", "0"], ids=["regrouped", "in-place"])
@pytest.mark.parametrize("n_players", [3, 6])
def test_fused_rollout_matches_spec(monkeypatch, n_players, regroup):
    monkeypatch.setenv("COUP_REGROUP", regroup)
    n, steps, seed = 4096, 300, 5 + n_players
    ref = oracle.np_rollout(n_players, seed=seed, n=n, steps=steps, auto_reset=True)
    env = BatchedCoupEnv(n, seed=seed, obs=False, num_players=n_players)
    stats = env.new_stats()
    env.rollout(120, stats)
    env.rollout(180, stats)
    np.testing.assert_array_equal(_np(env.export_state()).astype(np.uint32), ref["final_state"])
    assert int(stats["episodes"].sum()) == int(ref["episodes_done"][0])
    assert int(stats["return_sum"].sum()) == int(ref["return_sum_p0"][0])
    assert env.error_count() == 0


@pytest.mark.parametrize("n_players", [3, 4, 6])
def test_state_api_against_spec(n_players):
    """coup_new_initial_state / coup_apply_action / coup_query per lane
    against NpState, with chance outcomes and decisions picked on the host
    (a different rng from the in-kernel one), until every game ends."""
    B = 48
    rng = np.random.default_rng(n_players)
    env = BatchedCoupEnv(B, seed=0, obs=False, num_players=n_players)
    env.new_initial_state()
    states = [oracle.NpState(n_players) for _ in range(B)]
    for _ in range(60 * n_players):
        q = env.query(obs=True)
        legal, cur, term = _np(q["legal_mask"]).astype(np.uint32), _np(q["current_player"]), _np(q["terminal"])
        rew, ret, obs = _np(q["rewards"]), _np(q["returns"]), _np(q["obs"])
        words = _np(env.export_state()).astype(np.uint32)
        acts = np.full(B, -1, np.int8)
        for i, s in enumerate(states):
            assert int(legal[i]) == s.legal_mask()
            assert int(cur[i]) == s.current_player() and bool(term[i]) == s.is_terminal()
            assert rew[i].tolist() == s.rewards() and ret[i].tolist() == s.returns()
            assert words[i].tolist() == s.pack(1)  # new_initial_state starts episode 1
            for p in range(n_players):
                np.testing.assert_array_equal(obs[i, p], s.observation_tensor(p))
            if not s.is_terminal():
                acts[i] = rng.choice(s.legal_actions())
                s.apply_action(int(acts[i]))
        if np.all(acts < 0):
            break
        env.apply_action(torch.from_numpy(acts))
    assert all(s.is_terminal() for s in states)
    assert env.error_count() == 0


def test_export_import_roundtrip_and_illegal():
    env = BatchedCoupEnv(256, seed=3, obs=False, num_players=5)
    env.rollout(37)
    w = env.export_state()
    other = BatchedCoupEnv(256, seed=3, obs=False, num_players=5)
    other.import_state(w)
    assert torch.equal(other.export_state(), w)
    env.rollout(20)
    other.rollout(20)
    assert torch.equal(other.export_state(), env.export_state())
    fresh = BatchedCoupEnv(4, seed=0, obs=False, num_players=4)
    before = fresh.export_state().clone()
    fresh.step(torch.tensor([9, 10, 7, 18], dtype=torch.int8))  # not legal at turn begin
    assert fresh.error_count() == 4
    assert torch.equal(fresh.export_state(), before)


def test_six_player_full_batch_properties():
    """B = 2^20 six-player lanes: zero-sum rewards, non-empty well-formed
    legal masks, deck + hands = 15 cards, no rules errors."""
    B = 1 << 20
    env = BatchedCoupEnv(B, seed=9, obs=False, num_players=6)
    for _ in range(60):
        o = env.step()
        assert int(o["rewards"].to(torch.int32).sum(1).abs().max()) == 0
    legal = _np(o["legal_mask"]).astype(np.uint32)
    assert np.all(legal != 0) and np.all(legal < (1 << 18))
    w = _np(env.export_state()).astype(np.uint32)
    cards = np.zeros(B, np.int64)
    for p in range(6):
        h = (w[:, p // 2] >> (16 * (p % 2))) & 0xFFFF
        for i in range(4):
            cards += ((h >> (4 * i)) & 0xF) != 0xF
    deck = sum((w[:, 5] >> (4 * t)) & 0xF for t in range(5))
    assert np.all(deck + cards == 15)
    assert not np.any(w[:, 3] >> 31)
    assert env.error_count() == 0


@pytest.mark.parametrize("n_players", [2, 4, 6])
@pytest.mark.parametrize("auto_reset", [True, False])
def test_regrouped_step_equals_in_place_step(monkeypatch, n_players, auto_reset, ahead="1"):
    """k_step_sorted (lanes counting-sorted by decision through LDS, resets
    dealt by the first threads) == k_step (lanes in place), ragged batch,
    both the uniform policy and caller actions (about 1 in 8 illegal, so
    the rejected-action path is in the sort too); with the next uniform
    decision drawn ahead and parked in the record (the default) and without.
    Exported records carry no parked decision."""
    monkeypatch.setenv("COUP_AHEAD", ahead)
    n, steps, seed = 1000, 150, 11 + n_players
    envs = {}
    for knob in ("0", "1"):
        monkeypatch.setenv("COUP_REGROUP", knob)
        envs[knob] = BatchedCoupEnv(n, seed=seed, env_id_base=3 << 20, auto_reset=auto_reset, obs=False,
                                    num_players=n_players, generic=True)
    g = torch.Generator().manual_seed(seed)
    for t in range(steps):
        acts = None
        if t % 3 == 2:
            legal = envs["0"].query(obs=False)["legal_mask"].cpu().to(torch.int64)
            acts = torch.randint(0, 18, (n,), generator=g, dtype=torch.int64)
            ok = ((legal >> acts) & 1) == 1
            keep = torch.rand(n, generator=g) < 0.875
            # pick a legal action where there is one, except for the kept illegal ones
            first = torch.where(legal != 0, (legal & -legal).float().log2().to(torch.int64), acts)
            acts = torch.where(ok | ~keep, acts, first).to(torch.int8)
        outs = {}
        for knob, env in envs.items():
            monkeypatch.setenv("COUP_REGROUP", knob)
            outs[knob] = {k: v.clone() for k, v in env.step(acts).items()}
        for k in ("actions", "rewards", "step_type", "legal_mask", "current_player"):
            assert torch.equal(outs["0"][k], outs["1"][k]), (t, k)
        assert torch.equal(envs["0"].export_state(), envs["1"].export_state()), t
    assert envs["0"].error_count() == envs["1"].error_count()


@pytest.mark.parametrize("n_players", [2, 5, 6])
def test_regrouped_rollout_equals_in_place_rollout(monkeypatch, n_players):
    """k_rollout_sorted (lanes re-sorted by their next decision every step,
    finished lanes reset together) == k_rollout: records and per-lane
    statistics, ragged batch, launches of 1, 7 and 150 steps, and a start
    from terminal records (auto_reset off) and mid-deal records."""
    n, seed = 1000, 21 + n_players
    envs, stats = {}, {}
    for knob in ("0", "1"):
        monkeypatch.setenv("COUP_REGROUP", knob)
        env = BatchedCoupEnv(n, seed=seed, auto_reset=False, obs=False, num_players=n_players, generic=True)
        for _ in range(40):
            env.step()  # some lanes end terminal (no auto-reset)
        envs[knob], stats[knob] = env, env.new_stats()
    assert torch.equal(envs["0"].export_state(), envs["1"].export_state())
    for k in (1, 7, 150):
        for knob, env in envs.items():
            monkeypatch.setenv("COUP_REGROUP", knob)
            env.rollout(k, stats[knob])
        assert torch.equal(envs["0"].export_state(), envs["1"].export_state()), k
        for key in ("episodes", "return_sum", "length_sum"):
            assert torch.equal(stats["0"][key], stats["1"][key]), (k, key)
    for knob, env in envs.items():  # records at the first chance node, deals pending
        monkeypatch.setenv("COUP_REGROUP", knob)
        env.new_initial_state()
        env.rollout(9, stats[knob])
    assert torch.equal(envs["0"].export_state(), envs["1"].export_state())
    assert envs["0"].error_count() == envs["1"].error_count() == 0


@pytest.mark.parametrize("fused", [False, True], ids=["step", "rollout"])
def test_six_player_full_batch_sampled_lanes_match_spec(fused):
    """B = 2^20 six-player lanes (the c4 / c4r kernels, regrouped by
    decision): three 256-lane slices after 80 steps == np_rollout on those
    env ids alone."""
    B, steps, seed = 1 << 20, 80, 17
    env = BatchedCoupEnv(B, seed=seed, obs=False, num_players=6)
    if fused:
        env.rollout(steps)
    else:
        for _ in range(steps):
            env.step()
    words = _np(env.export_state()).astype(np.uint32)
    for k in (0, 300_001, B - 256):
        ref = oracle.np_rollout(6, seed=seed, n=256, steps=steps, env_id_base=k, auto_reset=True)
        np.testing.assert_array_equal(words[k:k + 256], ref["final_state"], err_msg=f"slice {k}")
    assert env.error_count() == 0
