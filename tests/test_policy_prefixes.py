"""The reference's own scripted game sequences: the policy tests of
coup_experiments/scripts/policy_analysis.py apply fixed action prefixes to
game.new_initial_state() and query the bot at decision nodes whose player
(and, in coup_test, coin count) the script's log messages state.  Replayed
here on the oracle (CPU) and on the GPU engine through the pyspiel facade:
every action must be in LegalActions(), every query point a decision node of
the stated player with the stated coins.  The two bluff_seq_test prefixes
answer a Tax with Block, outside LegalActions (coup.cc:868-873); the
reference applies it unchecked, both engines here reject it (DESIGN.md
section 8), and the check stops there."""
import json
import os

import pytest

from oracle import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "policy_prefixes.json")) as _f:
    SEQS = json.load(_f)["sequences"]


def replay(seq, state, coins):
    queries = {q["after"]: q for q in seq["queries"]}
    stop = seq.get("illegal_at", len(seq["actions"]))
    for k in range(stop + 1):
        q = queries.get(k)
        if q is not None:
            assert not state.is_terminal() and not state.is_chance_node(), f"{seq['name']} query after {k}"
            assert state.current_player() == q["player"], f"{seq['name']} query after {k}"
            if "coins" in q:
                assert coins(state, q["player"]) == q["coins"], f"{seq['name']} query after {k}"
        if k == stop:
            break
        a = seq["actions"][k]
        assert a in state.legal_actions(), f"{seq['name']}: action {k} ({a}) not legal"
        state.apply_action(a)
    if "illegal_at" in seq:
        a = seq["actions"][stop]
        assert a not in state.legal_actions()
        with pytest.raises(RuntimeError):
            state.apply_action(a)


@pytest.mark.parametrize("seq", SEQS, ids=[s["name"] for s in SEQS])
def test_oracle_policy_prefix(seq):
    replay(seq, oracle.OracleState(), lambda st, p: st.coins(p))


@pytest.mark.gpu
@pytest.mark.parametrize("seq", SEQS, ids=[s["name"] for s in SEQS])
def test_gpu_policy_prefix(seq):
    from open_spiel_coup_amd import packed, pyspiel

    def coins(st, p):
        return packed.lane(st.packed_record().reshape(1, 4))["coins"][p]

    replay(seq, pyspiel.load_game("coup").new_initial_state(), coins)
