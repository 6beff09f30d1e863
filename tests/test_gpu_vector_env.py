"""coup_step's skipped lanes (actions[i] < 0) and the batched SyncVectorEnv
built on them (open_spiel/python/vector_env.py:17-78)."""
import numpy as np
import pytest
import torch

from oracle import oracle

# state_mode: host-resident envs (kept on the host by the vector env) and
# device-lane envs (adopted into one shared env) -- conftest.py
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("state_mode")]

from open_spiel_coup_amd import BatchedCoupEnv, pyspiel, rl_environment, vector_env  # noqa: E402

SKIPPED = 3  # COUP_STEP_SKIPPED


def _random_legal(mask, rng):
    """One uniformly chosen set bit of each 18-bit mask (0 where empty)."""
    out = np.zeros(len(mask), dtype=np.int64)
    for i, m in enumerate(mask):
        bits = [a for a in range(18) if (int(m) >> a) & 1]
        out[i] = rng.choice(bits) if bits else 0
    return out


@pytest.mark.parametrize("regroup", ["0", "1"], ids=["in-place", "regrouped"])
@pytest.mark.parametrize("players,generic", [(2, False), (2, True), (6, False)], ids=["2p", "2p-generic", "6p"])
def test_negative_action_skips_lane(monkeypatch, regroup, players, generic):
    """Every step, ~30% of the lanes get action -1.  Those lanes keep their
    record and episode statistics, count no error and report action -1,
    rewards 0, step type SKIPPED and their current legal mask / player /
    observations; every other lane equals a copy of the env stepped with the
    same actions on all lanes."""
    monkeypatch.setenv("COUP_REGROUP", regroup)
    n, seed = 700, 77
    kw = dict(seed=seed, env_id_base=5, auto_reset=False, obs=True, num_players=players, generic=generic,
              episode_stats=True)
    env = BatchedCoupEnv(n, **kw)
    twin = BatchedCoupEnv(n, **kw)
    rng = np.random.default_rng(seed)
    skipped_total = 0
    for t in range(100):
        before = env.export_state()
        q = env.query(obs=True)
        legal = q["legal_mask"].cpu().numpy() & 0x3FFFF
        acts = _random_legal(legal, rng)
        skip = rng.random(n) < 0.3
        skipped_total += int(skip.sum())
        twin.import_state(before)
        twin.episodes.copy_(env.episodes)
        twin.return_sum.copy_(env.return_sum)
        ep_before = env.episodes.clone(), env.return_sum.clone()
        a_env = torch.from_numpy(np.where(skip, -1, acts).astype(np.int8))
        out = {k: v.clone() for k, v in env.step(a_env).items()}
        ref = {k: v.clone() for k, v in twin.step(torch.from_numpy(acts.astype(np.int8))).items()}
        sk = torch.from_numpy(skip).to(env.device)
        after = env.export_state()
        assert torch.equal(after[sk], before[sk]), t
        assert torch.equal(after[~sk], twin.export_state()[~sk]), t
        assert (out["actions"][sk] == -1).all() and (out["rewards"][sk] == 0).all()
        assert (out["step_type"][sk] == SKIPPED).all()
        assert torch.equal(out["legal_mask"][sk], q["legal_mask"][sk])
        assert torch.equal(out["current_player"][sk], q["current_player"][sk])
        assert torch.equal(out["obs"][sk], q["obs"][sk])
        for k in ("actions", "rewards", "step_type", "legal_mask", "current_player", "obs"):
            assert torch.equal(out[k][~sk], ref[k][~sk]), (t, k)
        assert torch.equal(env.episodes[sk], ep_before[0][sk]) and torch.equal(env.return_sum[sk], ep_before[1][sk])
        assert torch.equal(env.episodes[~sk], twin.episodes[~sk])
        assert torch.equal(env.return_sum[~sk], twin.return_sum[~sk])
    assert env.error_count() == 0
    assert skipped_total > 0


def _loop_envs(n, seed, obs_type):
    """Environments stepped one by one whose lane i is keyed like lane i of a
    batched SyncVectorEnv (global env id i under `seed`)."""
    envs = [rl_environment.Environment("coup", seed=seed, observation_type=obs_type) for _ in range(n)]
    for i, e in enumerate(envs):
        e._key_stream(i)
    return envs


class _Out:
    def __init__(self, a):
        self.action = a


def _same_time_step(a, b):
    assert a.step_type == b.step_type
    assert a.rewards == b.rewards and a.discounts == b.discounts
    assert a.observations["current_player"] == b.observations["current_player"]
    assert a.observations["legal_actions"] == b.observations["legal_actions"]
    assert a.observations["info_state"] == b.observations["info_state"]


@pytest.mark.parametrize("obs_type", [rl_environment.ObservationType.INFORMATION_STATE,
                                      rl_environment.ObservationType.OBSERVATION], ids=["info", "obs"])
@pytest.mark.parametrize("n", [2, 24], ids=["lane-ops", "launch"])
def test_batched_sync_vector_env_equals_loop(obs_type, n):
    """The batched vector env (one shared env: one launch per step, or one
    lane op per env at most vector_env.LANE_OPS_UPTO envs) and the
    reference's loop over the same games give identical time steps, with
    and without reset_if_done."""
    assert (n <= vector_env.LANE_OPS_UPTO) == (n == 2)
    seed = 1234
    batched = vector_env.SyncVectorEnv([rl_environment.Environment("coup", seed=seed, observation_type=obs_type)
                                        for _ in range(n)])
    loop = vector_env.SyncVectorEnv(_loop_envs(n, seed, obs_type), batched=False)
    assert batched.batched and not loop.batched
    ta, tb = batched.reset(), loop.reset()
    for x, y in zip(ta, tb):
        _same_time_step(x, y)
    rng = np.random.default_rng(5)
    lasts = 0
    for t in range(90):
        outs = [_Out(0 if ts.last() else int(rng.choice(ts.observations["legal_actions"][ts.current_player()])))
                for ts in ta]
        rid = t % 3 != 0
        ta, ra, da, ua = batched.step(outs, reset_if_done=rid)
        tb, rb, db, ub = loop.step(outs, reset_if_done=rid)
        assert ra == rb and da == db
        lasts += sum(da)
        for x, y in zip(ta, tb):
            _same_time_step(x, y)
        for x, y in zip(ua, ub):
            _same_time_step(x, y)
    assert lasts > 2 * n  # episodes end (~15 decisions each) and restart


@pytest.mark.parametrize("host_upto", [None, 0], ids=["kept", "adopted"])
def test_adopted_envs_keep_their_games(host_upto, monkeypatch):
    """After adoption each Environment still plays its own lane: get_state
    replays through the oracle to the last time step; a single env's step,
    set_state and seed act on that lane only; an action DoApplyAction
    raises on (the reference's apply_action has no legality check) raises
    SpielError after the other envs' actions were applied."""
    monkeypatch.setattr(vector_env, "HOST_UPTO", host_upto)  # 0: host-resident games move to lanes too
    n = 6
    envs = [rl_environment.Environment("coup", seed=100 + i) for i in range(n)]
    envs[2].reset()
    pre = envs[2].get_state.history()
    venv = vector_env.SyncVectorEnv(envs)
    assert venv.batched
    assert envs[2].get_state.history() == pre  # the game moved into the shared env intact
    ts = venv.reset()
    rng = np.random.default_rng(9)

    def act(t):
        return 0 if t.last() else int(rng.choice(t.observations["legal_actions"][t.current_player()]))

    for _ in range(25):
        ts, _, _, _ = venv.step([_Out(act(t)) for t in ts], reset_if_done=True)
    for e, t in zip(envs, ts):
        ref = oracle.OracleState()
        for a in e.get_state.history():
            ref.apply_action(a)
        cur = t.observations["current_player"]
        assert cur == ref.current_player()
        assert t.observations["legal_actions"][cur] == ref.legal_actions()
        for p in (0, 1):
            assert t.observations["info_state"][p] == ref.information_state_tensor(p).tolist()
    # one env stepped on its own: the others do not move
    others = [e.get_state.history() for e in envs]
    t1 = envs[1].step([act(ts[1])])
    for j, e in enumerate(envs):
        if j != 1:
            assert e.get_state.history() == others[j]
    assert len(envs[1].get_state.history()) > len(others[1]) or t1.first()
    ts[1] = t1
    # set_state copies a game into one lane
    envs[0].set_state(envs[3].get_state)
    assert envs[0].get_state.history() == envs[3].get_state.history()
    ts[0] = envs[0].get_time_step()
    # an action the reference rejects: SpielError, the others applied
    hist = [e.get_state.history() for e in envs]
    bad = [act(t) for t in ts]
    if not ts[4].last():
        ref4 = oracle.OracleState()
        for p, a in envs[4].get_state.full_history():
            ref4.apply_action(a)

        def rejected(a):
            try:
                ref4.clone().apply_action_unchecked(a)
                return False
            except RuntimeError:
                return True
        bad[4] = next((a for a in range(18) if rejected(a)), 18)
        with pytest.raises(pyspiel.SpielError):
            venv.step([_Out(a) for a in bad])
        assert envs[4].get_state.history() == hist[4]
        assert any(len(envs[j].get_state.history()) > len(hist[j]) for j in range(n) if j != 4)
    # seed() of an adopted env re-keys the shared stream; that env restarts
    ts = [e.get_time_step() for e in envs]
    envs[5].seed(77)
    assert venv.batched and envs[5]._owner is venv
    ts, _, _, _ = venv.step([_Out(act(t)) for t in ts])
    assert ts[5].first()


def test_vector_env_falls_back_to_loop():
    """Envs with their own chance sampler keep the reference's loop."""
    envs = [rl_environment.Environment("coup", chance_event_sampler=rl_environment.ChanceEventSampler(seed=i))
            for i in range(2)]
    venv = vector_env.SyncVectorEnv(envs)
    assert not venv.batched
    ts = venv.reset()
    ts, _, _, _ = venv.step([_Out(t.observations["legal_actions"][t.current_player()][0]) for t in ts])
    assert all(t.mid() or t.last() for t in ts)


@pytest.mark.parametrize("players,obs,info", [(2, True, False), (2, False, True), (6, True, False), (3, False, False)],
                         ids=["2p-obs", "2p-info", "6p-obs", "3p"])
@pytest.mark.parametrize("uniform", [True, False])
def test_step_host_equals_step(players, obs, info, uniform):
    """coup_step_host (outputs written into mapped host memory, one launch)
    == coup_step on a twin env (device outputs, then queries), lane by lane,
    with skipped lanes among caller actions."""
    n, seed = 300, 41
    kw = dict(seed=seed, env_id_base=9, auto_reset=False, num_players=players, history=info)
    host = BatchedCoupEnv(n, obs=False, **kw)
    dev = BatchedCoupEnv(n, obs=obs, info_state=info, **kw)
    rng = np.random.default_rng(seed)
    for t in range(60):
        acts = None
        if not uniform:
            legal = dev.query(obs=False)["legal_mask"].cpu().numpy() & 0x3FFFF
            acts = np.where(rng.random(n) < 0.25, -1, _random_legal(legal, rng)).astype(np.int8)
        q = host.step_host(acts, obs=obs, info_state=info)
        o = dev.step(None if acts is None else torch.from_numpy(acts))
        assert np.array_equal(q["legal_mask"], o["legal_mask"].cpu().numpy()), t
        assert np.array_equal(q["current_player"], o["current_player"].cpu().numpy()), t
        assert np.array_equal(q["step_type"], o["step_type"].cpu().numpy()), t
        assert np.array_equal(q["rewards"], o["rewards"].cpu().numpy()), t
        assert np.array_equal(q["actions"], o["actions"].cpu().numpy()), t
        if obs:
            assert np.array_equal(q["obs"], o["obs"].cpu().numpy()), t
        if info:
            assert np.array_equal(q["info_state"], o["info_state"].cpu().numpy()), t
    assert torch.equal(host.export_state(), dev.export_state())
    assert host.error_count() == dev.error_count() == 0


@pytest.mark.parametrize("obs,info", [(True, False), (False, True), (True, True)], ids=["obs", "info", "both"])
def test_step_host_active_rows(obs, info):
    """coup_step_host with COUP_HOST_ACTIVE (an env of a shared SyncVectorEnv
    env stepping alone): the small outputs of every lane as without it, and
    the tensor rows of the stepped lanes only, in lane order -- equal to the
    full step's rows of those lanes."""
    n, seed = 64, 12
    kw = dict(seed=seed, env_id_base=3, auto_reset=False, obs=False, history=True)
    full, act = BatchedCoupEnv(n, **kw), BatchedCoupEnv(n, **kw)
    rng = np.random.default_rng(seed)
    for t in range(50):
        legal = full.query(obs=False)["legal_mask"].cpu().numpy() & 0x3FFFF
        keep = rng.random(n) < (0.05 if t % 2 else 0.5)
        keep[t % n] = True
        acts = np.where(keep, _random_legal(legal, rng), -1).astype(np.int8)
        q = full.step_host(acts, obs=obs, info_state=info)
        r = act.step_host(acts, obs=obs, info_state=info, active_only=True)
        for k in ("legal_mask", "current_player", "step_type", "rewards", "actions"):
            assert np.array_equal(q[k], r[k]), (t, k)
        for k in (("obs",) if obs else ()) + (("info_state",) if info else ()):
            assert np.array_equal(q[k][acts >= 0], r[k]), (t, k)
    assert torch.equal(full.export_state(), act.export_state())
    assert full.error_count() == act.error_count() == 0
