"""The reference's own scripted game sequences: the policy tests of
coup_experiments/scripts/policy_analysis.py apply fixed action sequences to
game.new_initial_state() and query the bot at decision nodes whose player
(and, in coup_test, coin count) the script's log messages state.  Replayed
here on the oracle (CPU) and on the GPU engine through the pyspiel facade:
every query point must be a decision node of the stated player with the
stated coins.

The two bluff_seq_test sequences answer a Tax with Block, outside
LegalActions (coup.cc:867-871).  The reference script runs anyway: pyspiel's
apply_action is State::ApplyAction, which has no legality check (pyspiel.cc:
266, spiel.cc:322-331), so the Block is applied by DoApplyAction's Block
branch (coup.cc:631-633).  Both engines here replay the whole script that
way; apply_action_with_legality_check (spiel.cc:334-344) stops at the Block
('illegal_at')."""
import json
import os

import pytest

from oracle import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "policy_prefixes.json")) as _f:
    SEQS = json.load(_f)["sequences"]


def replay(seq, state, coins, apply):
    """Apply the whole sequence with `apply(state, a)`, checking every query
    point on the way."""
    queries = {q["after"]: q for q in seq["queries"]}
    for k in range(len(seq["actions"]) + 1):
        q = queries.get(k)
        if q is not None:
            assert not state.is_terminal() and not state.is_chance_node(), f"{seq['name']} query after {k}"
            assert state.current_player() == q["player"], f"{seq['name']} query after {k}"
            assert state.legal_actions(), f"{seq['name']} query after {k}"
            if "coins" in q:
                assert coins(state, q["player"]) == q["coins"], f"{seq['name']} query after {k}"
        if k == len(seq["actions"]):
            break
        a = seq["actions"][k]
        first_illegal = seq.get("illegal_at", len(seq["actions"]))
        if k <= first_illegal:  # legal up to 'illegal_at', which is not
            assert (a in state.legal_actions()) == (k < first_illegal), f"{seq['name']}: action {k} ({a})"
        apply(state, a)


def replay_checked(seq, state, apply_checked):
    """The legality-checked form: every action up to 'illegal_at' applies,
    that one raises and leaves the state as it was."""
    stop = seq.get("illegal_at", len(seq["actions"]))
    for a in seq["actions"][:stop]:
        apply_checked(state, a)
    if "illegal_at" in seq:
        a = seq["actions"][stop]
        assert a not in state.legal_actions()
        before = state.legal_actions(), state.current_player()
        with pytest.raises(RuntimeError):
            apply_checked(state, a)
        assert (state.legal_actions(), state.current_player()) == before


@pytest.mark.parametrize("seq", SEQS, ids=[s["name"] for s in SEQS])
def test_oracle_policy_sequence(seq):
    replay(seq, oracle.OracleState(), lambda st, p: st.coins(p), lambda st, a: st.apply_action_unchecked(a))
    replay_checked(seq, oracle.OracleState(), lambda st, a: st.apply_action(a))


@pytest.mark.gpu
@pytest.mark.parametrize("seq", SEQS, ids=[s["name"] for s in SEQS])
def test_gpu_policy_sequence(seq):
    """The facade replays the whole script with apply_action, equal to the
    oracle's unchecked apply at every state (records, legal actions, both
    observation tensors); apply_action_with_legality_check stops at the
    Block."""
    from open_spiel_coup_amd import packed, pyspiel

    def coins(st, p):
        return packed.lane(st.packed_record().reshape(1, 4))["coins"][p]

    game = pyspiel.load_game("coup")
    st, ref = game.new_initial_state(), oracle.OracleState()

    def apply(s, a):
        s.apply_action(a)
        ref.apply_action_unchecked(a)
        assert s.packed_record().tolist() == [int(x) for x in ref.pack(0)]
        assert s.history() == ref.history()
        for p in (0, 1):
            assert s.observation_tensor(p) == list(ref.observation_tensor(p))

    replay(seq, st, coins, apply)
    replay_checked(seq, game.new_initial_state(), lambda s, a: s.apply_action_with_legality_check(a))
