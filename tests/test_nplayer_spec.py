"""The N-player extension's CPU specification (oracle/coup_nplayer.c).

At N = 2 it must be the reference game: pinned here against the reference's
KATs and transcript, and step for step against the 2-player oracle.  For
N > 2 (no reference semantics, parity unpinned) the tests check the
extension's invariants."""
import numpy as np
import pytest

from oracle import oracle
from tests import golden_util as G

KATS = G.load_kats()
PT = G.load_playthrough()["states"]


@pytest.mark.parametrize("scenario", KATS, ids=[s["name"] for s in KATS])
def test_n2_spec_kats(scenario):
    st = oracle.NpState(2)
    applied = 0
    for chk in sorted(scenario["checks"], key=lambda c: c["after"]):
        while applied < chk["after"]:
            st.apply_action(scenario["actions"][applied])
            applied += 1
        G.check_kat(chk, st.cards, st.coins, lambda p: st._s.pl[p].last_action, st.current_player,
                    st.legal_actions, st.is_terminal, st.rewards, st.returns)


def test_n2_spec_playthrough():
    st = oracle.NpState(2)
    hist = PT[-1]["history"]
    for k, rec in enumerate(PT):
        if "current_player" in rec:
            assert st.current_player() == rec["current_player"]
            if not rec["is_terminal"]:
                assert st.legal_actions() == rec["legal_actions"]
            if not rec["is_chance"]:
                assert st.rewards() == [int(x) for x in rec["rewards"]]
                assert st.returns() == [int(x) for x in rec["returns"]]
            for p in (0, 1):
                np.testing.assert_array_equal(st.observation_tensor(p), G.dense(rec["ObservationTensor"][str(p)], 98))
        if k < len(hist):
            st.apply_action(hist[k])


def _to_2p_record(w8):
    """N-player record at N = 2 -> the 2-player 16-byte record."""
    w = [int(x) for x in w8]
    coins, lost, begin, err = w[3] & 0xFFFFFF, (w[3] >> 24) & 0x3F, (w[3] >> 30) & 1, w[3] >> 31
    last, rcount = w[4] & 0x3FFFFFFF, w[4] >> 30
    deck, qlen, qp, T = w[5] & 0xFFFFF, (w[5] >> 24) & 3, (w[5] >> 26) & 7, w[5] >> 29
    move, turn, M, rloser = w[6] & 0x1FF, (w[6] >> 9) & 0x1FF, (w[6] >> 18) & 7, (w[6] >> 24) & 7
    ep = (w[7] & 0x1FFFFFF) | ((w[6] >> 27) << 25)  # 30-bit N-player episode
    r0 = -rcount if rloser == 0 else rcount
    qids = (1 << qlen) - 1 if qp == 1 else 0
    return [w[0],
            deck | ((coins & 0xF) << 20) | (((coins >> 4) & 0xF) << 24) | ((r0 + 2) << 28) | (err << 31),
            (last & 31) | (((last >> 5) & 31) << 5) | ((lost & 1) << 10) | (((lost >> 1) & 1) << 11) |
            (qlen << 12) | (qids << 15) | (T << 19) | (M << 20) | (begin << 21) | (move << 22) |
            (((ep >> 25) & 7) << 29),
            turn | ((ep & 0x1FFFFFF) << 7)]


@pytest.mark.parametrize("auto_reset", [True, False])
def test_n2_spec_equals_two_player_oracle(auto_reset):
    ref = oracle.rollout(seed=13, n=256, steps=200, auto_reset=auto_reset, want_obs=True)
    got = oracle.np_rollout(2, seed=13, n=256, steps=200, auto_reset=auto_reset, want_obs=True)
    for k in ("actions", "rewards", "step_type", "legal", "obs"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    assert int(got["episodes_done"][0]) == int(ref["episodes_done"][0])
    for lane in range(256):
        assert _to_2p_record(got["final_state"][lane]) == [int(x) for x in ref["final_state"][lane]]


@pytest.mark.parametrize("n", [3, 4, 5, 6])
def test_n_player_invariants(n):
    out = oracle.np_rollout(n, seed=n, n=64, steps=600, auto_reset=False, want_obs=True)
    st, rw, lg, obs = out["step_type"], out["rewards"].astype(np.int64), out["legal"], out["obs"]
    acc = np.zeros((64, n), np.int64)
    finished = 0
    for t in range(st.shape[0]):
        acc += rw[t]
        assert np.all(rw[t].sum(1) == 0)  # zero-sum every step
        for lane in np.nonzero(st[t] == 2)[0]:
            assert acc[lane].sum() == 0
            assert np.abs(acc[lane]).max() <= 2 * (n - 1)
            finished += 1
        acc[st[t] != 1] = 0
        acc[st[t] == 2] = 0
        assert np.all((lg[t] != 0) == (st[t] != 2))
        assert np.all(lg[t] < (1 << 18))
        o = obs[t]
        assert np.all(o[:, np.arange(n), np.arange(n)] == 1)  # observer one-hot
    assert finished > 20
    # every card is somewhere: deck + hands = 15; no lane hit an error
    w = out["final_state"]
    assert not np.any(w[:, 3] >> 31)
    for lane in range(64):
        hands = [int(w[lane, k // 2]) >> (16 * (k % 2)) & 0xFFFF for k in range(n)]
        cards = sum(sum(1 for i in range(4) if (h >> (4 * i)) & 0xF != 0xF) for h in hands)
        deck = sum((int(w[lane, 5]) >> (4 * t)) & 0xF for t in range(5))
        assert deck + cards == 15


def test_six_player_targets_and_responders():
    """Scripted 6-player opening: P1's Foreign Aid is answered by P2..P6 in
    seat order; P1's Steal targets P2 only."""
    st = oracle.NpState(6)
    for k in range(12):
        st.apply_action(k % 5)  # deal 12 cards
    assert st.current_player() == 0 and st.coins(0) == 2
    st.apply_action(1)  # P1 Foreign Aid
    for r in range(1, 6):
        assert st.current_player() == r and st.legal_actions() == [9, 10]
        st.apply_action(9)  # everybody passes
    assert st.coins(0) == 4 and st.current_player() == 1  # FA done, P2's turn
    st.apply_action(6)  # P2 steals from P3
    assert st.current_player() == 2 and st.legal_actions() == [9, 10, 11]
    st.apply_action(9)
    assert st.coins(1) == 4 and st.coins(2) == 0 and st.current_player() == 2
