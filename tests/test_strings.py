"""Host-side strings (open_spiel_coup_amd.strings) from packed records +
history bytes: verbatim with the reference transcript and the oracle."""
import numpy as np
import pytest

from open_spiel_coup_amd import strings
from oracle import oracle
from tests import golden_util as G

PT = G.load_playthrough()["states"]


def _oracle_at(history):
    st = oracle.OracleState()
    for a in history:
        st.apply_action(a)
    return st


@pytest.mark.parametrize("rec", PT, ids=[f"state{s['index']}" for s in PT])
def test_strings_match_transcript(rec):
    st = _oracle_at(rec["history"])
    w = np.array([st.pack()], np.uint32)
    h = st.history_bytes()
    if "to_string" in rec:
        assert G.rstrip_lines(strings.to_string(w, h)) == rec["to_string"]
    if "ObservationString" in rec:
        for p in (0, 1):
            assert strings.observation_string(w, h, p) == rec["ObservationString"][str(p)]
            assert strings.information_state_string(w, h, p) == rec["InformationStateString"][str(p)]


def test_strings_match_oracle_on_random_games():
    rng = np.random.default_rng(5)
    checked = 0
    for g in range(60):
        st = oracle.OracleState()
        while not st.is_terminal():
            w = np.array([st.pack()], np.uint32)
            h = st.history_bytes()
            assert strings.to_string(w, h) == st.to_string()
            for p in (0, 1):
                assert strings.observation_string(w, h, p) == st.observation_string(p)
                assert strings.information_state_string(w, h, p) == st.information_state_string(p)
            checked += 1
            st.apply_action(int(rng.choice(st.legal_actions())))
    assert checked > 1000


def test_action_to_string():
    assert strings.action_to_string(-1, 4) == "Chance drawn card:Duke"
    assert strings.action_to_string(0, 16) == "ExchangeReturn24"
