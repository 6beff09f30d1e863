"""The pyspiel / rl_environment / vector_env facades over the GPU engine,
checked against the reference's golden data and the oracle."""
import numpy as np
import pytest

from oracle import oracle
from tests import golden_util as G

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("state_mode")]

from open_spiel_coup_amd import pyspiel, rl_environment, vector_env  # noqa: E402

PT = G.load_playthrough()["states"]
KATS = G.load_kats()


def test_pyspiel_playthrough():
    """Replay coup.txt through load_game('coup').new_initial_state() and
    check every recorded field, strings included."""
    game = pyspiel.load_game("coup")
    state = game.new_initial_state()
    hist = PT[-1]["history"]
    for k, rec in enumerate(PT):
        assert state.history() == rec["history"]
        if "to_string" in rec:
            assert G.rstrip_lines(str(state)) == rec["to_string"]
        if "current_player" in rec:
            assert state.current_player() == rec["current_player"]
            assert state.is_terminal() == rec["is_terminal"]
            assert state.is_chance_node() == rec["is_chance"]
            if not rec["is_terminal"]:
                assert state.legal_actions() == rec["legal_actions"]
            if rec["is_chance"]:
                assert state.chance_outcomes() == [tuple(x) for x in rec["chance_outcomes"]]
            else:
                assert state.rewards() == [float(x) for x in rec["rewards"]]
                assert state.returns() == [float(x) for x in rec["returns"]]
            for p in (0, 1):
                assert state.observation_tensor(p) == G.dense(rec["ObservationTensor"][str(p)], 98).tolist()
                assert state.information_state_tensor(p) == \
                    G.dense(rec["InformationStateTensor"][str(p)], 2492).tolist()
                assert state.observation_string(p) == rec["ObservationString"][str(p)]
                assert state.information_state_string(p) == rec["InformationStateString"][str(p)]
        if k < len(hist):
            state.apply_action(hist[k])


@pytest.mark.parametrize("scenario", KATS, ids=[s["name"] for s in KATS])
def test_pyspiel_kats(scenario):
    state = pyspiel.load_game("coup").new_initial_state()
    applied = 0

    def cards(p):
        from open_spiel_coup_amd import packed
        return packed.lane(state.packed_record().reshape(1, 4))["cards"][p]

    def coins(p):
        from open_spiel_coup_amd import packed
        return packed.lane(state.packed_record().reshape(1, 4))["coins"][p]

    def last(p):
        from open_spiel_coup_amd import packed
        return packed.lane(state.packed_record().reshape(1, 4))["last_action"][p]

    for chk in sorted(scenario["checks"], key=lambda c: c["after"]):
        while applied < chk["after"]:
            state.apply_action(scenario["actions"][applied])
            applied += 1
        G.check_kat(chk, cards, coins, last, state.current_player, state.legal_actions, state.is_terminal,
                    state.rewards, state.returns)


def test_pyspiel_clone_child_serialize_and_errors():
    game = pyspiel.load_game("coup")
    s = game.new_initial_state()
    for a in [4, 3, 2, 0, 1]:
        s.apply_action(a)
    c = s.clone()
    ch = s.child(10)
    assert c.history() == [4, 3, 2, 0, 1] and ch.history() == [4, 3, 2, 0, 1, 10]
    assert s.history() == [4, 3, 2, 0, 1]  # child() leaves the parent untouched
    assert ch.current_player() == 0 and ch.legal_actions() == [9, 11]
    text = pyspiel.serialize_game_and_state(game, ch)
    g2, s2 = pyspiel.deserialize_game_and_state(text)
    assert s2.history() == ch.history() and str(s2) == str(ch)
    assert ch.legal_actions_mask() == [1 if a in (9, 11) else 0 for a in range(18)]
    with pytest.raises(pyspiel.SpielError):
        ch.apply_action_with_legality_check(0)  # Income is not a response to a block
    assert ch.history() == [4, 3, 2, 0, 1, 10]
    # pyspiel's apply_action has no legality check (pyspiel.cc:266): Income
    # applies (coup.cc:531-534), as the oracle's unchecked apply does
    from oracle import oracle
    ref = oracle.OracleState()
    for a in [4, 3, 2, 0, 1, 10, 0]:
        ref.apply_action_unchecked(a)
    ch.apply_action(0)
    assert ch.history() == [4, 3, 2, 0, 1, 10, 0]
    assert ch.packed_record().tolist() == [int(x) for x in ref.pack(0)]


def test_rl_environment_matches_oracle():
    """Environment('coup') (INFORMATION_STATE default, in-kernel chance) on
    random legal actions; the oracle replays the same history and must give
    the same time steps."""
    rng = np.random.default_rng(3)
    env = rl_environment.Environment("coup", seed=9)
    assert env.observation_spec()["info_state"] == (2492,)
    episodes = 0
    ts = env.reset()
    ref = None
    while episodes < 6:
        state = env.get_state
        ref = oracle.OracleState()
        for a in state.history():
            ref.apply_action(a)
        cur = ts.observations["current_player"]
        if ts.last():
            assert ts.discounts == [0.0, 0.0]
            assert ts.rewards == [float(x) for x in ref.rewards()]
            assert sum(ref.returns()) == 0
            episodes += 1
        else:
            assert cur == ref.current_player()
            assert ts.observations["legal_actions"][cur] == ref.legal_actions()
            assert ts.observations["legal_actions"][1 - cur] == []
        for p in (0, 1):
            assert ts.observations["info_state"][p] == ref.information_state_tensor(p).tolist()
        if ts.first():
            assert ts.rewards is None and ts.discounts is None
        action = None if ts.last() else int(rng.choice(ts.observations["legal_actions"][cur]))
        ts = env.step([action if action is not None else 0])


def test_rl_environment_observation_type_and_custom_sampler():
    """OBSERVATION tensors and a caller-supplied chance sampler (the State API
    path) reproduce the oracle driven by the same sampler."""
    env = rl_environment.Environment("coup", observation_type=rl_environment.ObservationType.OBSERVATION,
                                     chance_event_sampler=rl_environment.ChanceEventSampler(seed=11))
    ref_sampler = rl_environment.ChanceEventSampler(seed=11)
    ref = oracle.OracleState()

    class _Probe:
        """Adapter so the reference sampler can read the oracle's outcomes."""

        def __init__(self, st):
            self.st = st

        def chance_outcomes(self):
            return self.st.chance_outcomes()

    ts = env.reset()
    while ref.is_chance_node():
        ref.apply_action(ref_sampler(_Probe(ref)))
    rng = np.random.default_rng(1)
    while not ts.last():
        for p in (0, 1):
            assert ts.observations["info_state"][p] == ref.observation_tensor(p).tolist()
        cur = ts.observations["current_player"]
        a = int(rng.choice(ts.observations["legal_actions"][cur]))
        ts = env.step([a])
        ref.apply_action(a)
        while ref.is_chance_node():
            ref.apply_action(ref_sampler(_Probe(ref)))
        assert env.get_state.history() == ref.history()
    assert ts.rewards == [float(x) for x in ref.rewards()]


def test_sync_vector_env():
    envs = [rl_environment.Environment("coup", seed=s) for s in range(3)]
    venv = vector_env.SyncVectorEnv(envs)
    ts = venv.reset()
    assert len(ts) == 3 and all(t.first() for t in ts)

    class Out:
        def __init__(self, a):
            self.action = a

    rng = np.random.default_rng(0)
    for _ in range(40):
        outs = [Out(int(rng.choice(t.observations["legal_actions"][t.current_player()]))) for t in ts]
        ts, reward, done, unreset = venv.step(outs, reset_if_done=True)
        for t, d, u in zip(ts, done, unreset):
            assert d == u.last()
            assert t.first() if d else t.mid()


def test_default_environments_deal_independent_games():
    """Environment('coup') without a seed draws its key from OS entropy, like
    the reference's RandomState(None) chance sampler (rl_environment.py:
    119-131): default-constructed environments do not replay one stream, and
    seed(None) re-keys."""
    envs = [rl_environment.Environment("coup") for _ in range(4)]
    for e in envs:
        e.reset()
    deals = {tuple(e.get_state.history()) for e in envs}
    keys = {e._seed for e in envs}
    assert len(keys) == 4
    # 4 initial deals from 15 cards: four identical deals by chance are ~impossible
    assert len(deals) > 1
    k = envs[0]._seed
    envs[0].seed(None)
    assert envs[0]._seed != k
    fixed = [rl_environment.Environment("coup", seed=5) for _ in range(2)]
    for e in fixed:
        e.reset()
    assert fixed[0].get_state.history() == fixed[1].get_state.history()
