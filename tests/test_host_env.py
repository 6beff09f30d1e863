"""rl_environment.Environment and vector_env.SyncVectorEnv over host-resident
games (round 4: the game is a coup_slot_result stepped by
coup_host_state_step, the library's host build of the lane op), checked on
the CPU: every time step against the oracle replaying the env's own history
(current player, legal actions, both players' tensors as lists, rewards,
discounts, step types: rl_environment.py:243-254, 282-322), LAST then a
reset on the next step (rl_environment.py:310-311), seeds, get_state /
set_state, and a SyncVectorEnv that keeps its games on the host against the
reference's loop over envs keyed like its lanes (vector_env.py:40-78).

Host code only.  The facade binds the HIP device's lane pool even for host
games (it needs the device for snapshots and batched ops and says so at
once); here that lookup is replaced by a placeholder, since nothing in these
paths touches it.  The same paths run on the GPU in test_gpu_vector_env.py /
test_gpu_facade.py (state_mode "host")."""
import random

import numpy as np
import pytest

from oracle import oracle

from open_spiel_coup_amd import _native, pyspiel, rl_environment, vector_env


@pytest.fixture(autouse=True)
def host_games(monkeypatch):
    try:
        _native.load()
        pyspiel._host()
    except (ImportError, OSError) as e:
        pytest.skip(f"library / binding not built: {e}")
    monkeypatch.setattr(pyspiel, "DEVICE_STATES", False)
    monkeypatch.setattr(pyspiel, "_pool", lambda device=None: object())


def _replay(env):
    ref = oracle.OracleState()
    for _, a in env.get_state.full_history():
        ref.apply_action(a)
    return ref


def _check(env, ts, use_obs):
    ref = _replay(env)
    cur = ts.observations["current_player"]
    assert cur == ref.current_player()
    for p in (0, 1):
        want = ref.observation_tensor(p) if use_obs else ref.information_state_tensor(p)
        assert ts.observations["info_state"][p] == want.tolist()
        assert ts.observations["legal_actions"][p] == (ref.legal_actions() if p == cur else [])
    if ts.first():
        assert ts.rewards is None and ts.discounts is None
    else:
        assert ts.rewards == [float(r) for r in ref.rewards()]
        assert ts.discounts == ([0.0, 0.0] if ts.last() else [1.0, 1.0])
    assert ts.last() == ref.is_terminal()
    assert cur >= 0 or ref.is_terminal()  # chance is resolved inside the step


@pytest.mark.parametrize("use_obs", [False, True], ids=["info", "obs"])
def test_environment_time_steps_match_oracle(use_obs):
    otype = rl_environment.ObservationType.OBSERVATION if use_obs else None
    env = rl_environment.Environment("coup", seed=21, observation_type=otype)
    assert env._hq is not None  # host-resident
    rng = random.Random(4)
    ts = env.reset()
    _check(env, ts, use_obs)
    lasts = 0
    for _ in range(400):
        if ts.last():
            lasts += 1
            nxt = env.step([0])  # step after LAST starts a new episode (rl_environment.py:310-311)
            assert nxt.first()
        else:
            nxt = env.step([rng.choice(ts.observations["legal_actions"][ts.current_player()])])
        ts = nxt
        _check(env, ts, use_obs)
    assert lasts >= 5
    t2 = env.get_time_step()  # the same state, reported as MID (or LAST)
    assert t2.observations["info_state"] == ts.observations["info_state"] and not t2.first()


def test_environment_seeds_and_states():
    a = rl_environment.Environment("coup", seed=5)
    b = rl_environment.Environment("coup", seed=5)
    c = rl_environment.Environment("coup", seed=6)
    ta, tb, tc = a.reset(), b.reset(), c.reset()
    assert ta.observations == tb.observations
    hists = {tuple(e.get_state.full_history()) for e in (a, b, c)}
    assert len(hists) == 2  # seed 6 deals another game (the deals are in the history)
    # get_state is a snapshot; set_state copies a game in
    s = a.get_state
    s.apply_action(s.legal_actions()[0])
    assert a.get_state.history() != s.history()
    c.set_state(s)
    assert c.get_state.history() == s.history()
    t = c.get_time_step()
    _check(c, t, False)
    # an action DoApplyAction raises on: SpielError, the game unchanged
    st = c.get_state
    bad = next((x for x in range(18) if x not in t.observations["legal_actions"][t.current_player()]
                and _rejected(st, x)), None)
    if bad is not None:
        with pytest.raises(pyspiel.SpielError):
            c.step([bad])
        assert c.get_state.history() == st.history()
    with pytest.raises(pyspiel.SpielError):
        c.step([200])  # not an action id
    # an int8 id past the action space: DoApplyAction raises
    # (coup.cc:806), so SpielError -- a RuntimeError, not the binding's
    # ValueError -- and the game unchanged
    before = c.get_state.history()
    for x in (18, 20, 127):
        with pytest.raises(pyspiel.SpielError):
            c.step([x])
        assert c.get_state.history() == before
    q = pyspiel._host()._ext.step(c._hq._raw, 20, _native.SLOT_DEAL | _native.SLOT_UNCHECKED, 1, 0)
    assert not q["ok"]
    # seed() restarts the env on its own new stream: seed 6's first deal
    a.seed(6)
    assert a.step([0]).first()
    e6 = rl_environment.Environment("coup", seed=6)
    e6.reset()
    assert a.get_state.full_history() == e6.get_state.full_history()


def _rejected(state, a):
    ref = oracle.OracleState()
    for _, x in state.full_history():
        ref.apply_action(x)
    try:
        ref.apply_action_unchecked(a)
        return False
    except RuntimeError:
        return True


class _Out:
    def __init__(self, a):
        self.action = a


@pytest.mark.parametrize("use_obs", [False, True], ids=["info", "obs"])
def test_vector_env_kept_on_host_equals_loop(use_obs):
    """A SyncVectorEnv of host games keeps them on the host (up to
    vector_env.HOST_UPTO envs) and re-keys env i as global env id i under
    the first env's seed -- the deals of lane i of an adopting vector env;
    the reference's loop over envs keyed the same way gives equal time steps
    with and without reset_if_done."""
    otype = rl_environment.ObservationType.OBSERVATION if use_obs else None
    n, seed = 5, 77
    venv = vector_env.SyncVectorEnv([rl_environment.Environment("coup", seed=seed, observation_type=otype)
                                     for _ in range(n)])
    assert venv.batched and venv._host and venv._shared is None
    loop_envs = [rl_environment.Environment("coup", seed=seed, observation_type=otype) for _ in range(n)]
    for i, e in enumerate(loop_envs):
        e._key_stream(i)
    loop = vector_env.SyncVectorEnv(loop_envs, batched=False)
    assert not loop.batched
    ta, tb = venv.reset(), loop.reset()
    rng = np.random.default_rng(3)
    lasts = 0
    for t in range(120):
        for x, y in zip(ta, tb):
            assert x.observations == y.observations and x.step_type == y.step_type
            assert x.rewards == y.rewards and x.discounts == y.discounts
        outs = [_Out(0 if ts.last() else int(rng.choice(ts.observations["legal_actions"][ts.current_player()])))
                for ts in ta]
        rid = t % 3 != 0
        ta, ra, da, ua = venv.step(outs, reset_if_done=rid)
        tb, rb, db, ub = loop.step(outs, reset_if_done=rid)
        assert ra == rb and da == db
        for x, y in zip(ua, ub):
            assert x.observations == y.observations and x.step_type == y.step_type
        lasts += sum(da)
    assert lasts >= n
    for e, ts in zip(venv.envs, ta):
        _check(e, ts, use_obs)
    # seed() of a kept env re-keys the shared stream: every game is kept
    hist = [e.get_state.history() for e in venv.envs]
    venv.envs[2].seed(1234)
    assert [e.get_state.history() for e in venv.envs] == hist
    assert all(e._hseed == venv.envs[2]._seed and e._env_id == i for i, e in enumerate(venv.envs))
