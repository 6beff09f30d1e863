"""The oracle's unchecked ApplyAction (oc_apply_action_unchecked): pyspiel's
apply_action binds State::ApplyAction, which applies an action without a
LegalActions() check (pyspiel.cc:266, spiel.cc:322-331); DoApplyAction's own
checks decide (coup.cc:490-809).  The expectations below are read off
coup.cc's branches by hand, so they pin the restatement on the paths legal
play never takes; the GPU's lanes are compared with it in
tests/test_gpu_unchecked.py."""
import numpy as np
import pytest

from oracle import oracle

DEALS = [1, 1, 3, 3]  # queue P1, P2, P1, P2: each holds Ambassador + Contessa; coins 1 / 2 (coup.cc:407-427)


def start(*actions):
    st = oracle.OracleState()
    for a in DEALS + list(actions):
        st.apply_action_unchecked(a)
    return st


def rejects(st, a, code=None):
    before = (list(st.pack(0)), st.history())
    with pytest.raises(RuntimeError) as e:
        st.apply_action_unchecked(a)
    assert (list(st.pack(0)), st.history()) == before  # unchanged
    if code is not None:
        assert f"code {code}" in str(e.value)


def test_tax_answered_by_block_then_pass():
    """policy_analysis.py:290-299: Block (coup.cc:631-633) answers a Tax; the
    Tax player's LegalActions are then {Pass, Challenge} (coup.cc:930-933),
    and the Pass ends the turn with no coins (coup.cc:622-624)."""
    st = start(3)
    assert st.current_player() == 1 and 10 not in st.legal_actions()
    st.apply_action_unchecked(10)
    assert st.current_player() == 0 and st.legal_actions() == [9, 11]
    assert st.last_action(1) == 10
    st.apply_action_unchecked(9)
    assert st.current_player() == 1 and st.coins(0) == 1 and st.coins(1) == 2
    assert st.legal_actions() == [0, 1, 3, 5, 6]  # P2's turn begins


def test_claim_second_half_off_turn_begin():
    """A claim applied when is_turn_begin_ is false runs its second half for
    the mover (coup.cc:543-545 FA, 562-564 Tax, 582-586 Exchange, 598-602
    Steal) and NextPlayerTurn from there."""
    st = start(3, 1)  # P1 Tax, P2 answers with Foreign Aid
    assert st.coins(1) == 4 and st.coins(0) == 1
    assert st.current_player() == 1 and st.legal_actions() == [0, 1, 3, 4, 5, 6]  # T ^= 1 -> P2, 4 coins
    st = start(3, 3)  # ... with Tax: +3
    assert st.coins(1) == 5
    st = start(3, 6)  # ... with Steal: takes k = min(2, coins of P1) = 1
    assert (st.coins(0), st.coins(1)) == (0, 3)
    st = start(3, 5)  # ... with Exchange: two deals to P2, still P2's move
    assert st.is_chance_node()
    st.apply_action_unchecked(0)
    st.apply_action_unchecked(4)
    assert st.current_player() == 1 and len(st.cards(1)) == 4


def test_pass_completes_whatever_came_last():
    """Pass recurses into DoApplyAction(op.last) for the opponent (coup.cc:
    625-628): after P1's Income and an illegal Pass by P2, P1's Income runs
    again (+1, NextPlayerTurn)."""
    st = start(0)  # P1 Income: coins 2, P2's turn
    st.apply_action_unchecked(9)
    assert st.coins(0) == 3 and st.last_action(1) == 9


def test_rejections_where_the_reference_raises():
    rejects(start(), 9)            # Pass -> DoApplyAction(kNone): "Invalid player action" (coup.cc:806)
    rejects(start(), 2)            # Coup with 1 coin: SPIEL_CHECK_GE (coup.cc:549)
    rejects(start(), 4)            # Assassinate with 1 coin (coup.cc:568)
    rejects(start(), 11)           # Challenge of nothing (coup.cc:770)
    rejects(start(), 12)           # ExchangeReturn with 2 cards (coup.cc:787-796)
    st = start(6, 9, 10)           # P1 steals P2's 2 coins (P2 passes), P2 Blocks at its turn begin
    assert st.coins(1) == 0 and st.current_player() == 0
    rejects(st, 6)                 # P1 Steal from 0 coins: SPIEL_CHECK_GE (coup.cc:590)
    st = start(3, 9)               # P1 Tax, P2 passes: P2's turn
    st.apply_action_unchecked(0)   # P2 Income
    st.apply_action_unchecked(10)  # P1 Block (of nothing blockable)
    st.apply_action_unchecked(9)   # P2 Pass: the "block" ends P1's turn (coup.cc:622-624)
    assert st.current_player() == 1 and st.legal_actions() == [0, 1, 3, 4, 5, 6]  # P2: 3 coins
    rejects(oracle.OracleState(), 9)  # a chance node takes card types 0..4 only (coup.cc:493)


def test_lose_card_face_up_and_pass_after_pass():
    st = start(3, 11)  # P2 challenges P1's Tax; P1 holds no Duke: P1 lost
    assert st.current_player() == 0 and st.legal_actions() == [7, 8]
    st.apply_action_unchecked(7)
    assert st.cards(0) == [(1, 1), (3, 0)]  # the Ambassador in slot 0 is face up
    # P2's turn; P2 loses a card without having lost anything: allowed
    st.apply_action_unchecked(7)
    assert st.cards(1) == [(1, 1), (3, 0)] and st.current_player() == 0
    rejects(st, 7)  # P1's slot 0 is face up: SPIEL_CHECK_EQ face down (coup.cc:608)
    st.apply_action_unchecked(10)  # P1 Block at its own turn begin
    st.apply_action_unchecked(9)   # P2 Pass -> P1's Block: NextPlayerTurn
    st2 = start(3, 9)              # P1's Tax completes: 4 coins, P2's turn
    st2.apply_action_unchecked(9)  # P2 passes at its own turn begin: the pending
    assert st2.coins(0) == 7       # claim is P1's Tax, which completes again (coup.cc:625-628)
    assert st2.current_player() == 0 and st2.last_action(1) == 9
    rejects(st2, 9)                # a Pass answering a Pass: the recursion never ends (coup.cc:628)


def test_field_widths_are_enforced():
    """Coins past 15 are valid in the reference but not in the packed record:
    code 4 (OC_ERR_UNREPRESENTABLE), state unchanged."""
    st = start()
    while st.coins(1) < 15:
        st.apply_action_unchecked(0)  # Income, legal or not (coup.cc:531-534)
        st.apply_action_unchecked(0)
    st.apply_action_unchecked(0)
    assert st.coins(0) == st.coins(1) == 15 and st.current_player() == 1
    rejects(st, 0, code=4)


def test_unchecked_equals_checked_on_legal_actions():
    """On legal actions the unchecked apply is the checked one."""
    rng = np.random.default_rng(7)
    for g in range(200):
        a_st, b_st = oracle.OracleState(), oracle.OracleState()
        while not a_st.is_terminal():
            a = int(rng.choice(a_st.legal_actions()))
            a_st.apply_action(a)
            b_st.apply_action_unchecked(a)
            assert list(a_st.pack(0)) == list(b_st.pack(0))
        assert a_st.history() == b_st.history()
        rejects(b_st, 0, code=3)  # terminal
