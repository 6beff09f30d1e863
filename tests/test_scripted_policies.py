"""Deterministic scripted policies that drive games into corners uniform play
rarely reaches: truncation at move_number_ > 90 (coup.cc:989-992) through an
exchange loop -- including truncation in the middle of a turn's deals -- and
always-min / always-max / always-challenge play with chosen chance outcomes
(deck counts above 3 through the ExchangeReturn slot quirk, coup.cc:790-795).

CPU: the oracle reaches the truncation corner.  GPU: the same policies on
the State API of the batched engine (coup_new_initial_state with no deals,
then coup_apply_action for every decision and chance outcome), every lane
compared with an oracle game after every action."""
import numpy as np
import pytest

from oracle import oracle

CHANCE_FLAG = 1 << 31
N_POLICIES = 4


def bits(mask):
    return [a for a in range(18) if (mask >> a) & 1]


def choose(policy, mask, chance):
    """Action of scripted policy `policy` given the current legal mask."""
    acts = bits(mask & 0x3FFFF)
    if chance:
        return acts[0] if policy in (0, 2) else acts[-1]
    if policy == 0:  # always the smallest legal action
        return acts[0]
    if policy == 1:  # always the largest
        return acts[-1]
    if policy == 2:  # exchange loop: Exchange, Pass, return the highest pair
        for a in (5, 9):
            if a in acts:
                return a
        return acts[-1]
    for a in (11, 10):  # challenge / block whenever offered
        if a in acts:
            return a
    return acts[-1]


def oracle_mask(st):
    if st.is_terminal():
        return 0
    m = 0
    for a in st.legal_actions():
        m |= 1 << a
    return m | (CHANCE_FLAG if st.is_chance_node() else 0)


def test_oracle_exchange_loop_truncates():
    """Policy 2 never loses a card: the game ends by truncation, with
    move_number_ = 91 (possibly in the middle of an Exchange's deals)."""
    st = oracle.OracleState()
    n = 0
    while not st.is_terminal():
        st.apply_action(choose(2, oracle_mask(st), st.is_chance_node()))
        n += 1
        assert n < 200
    assert len(st.history()) == 91
    assert st.returns() == [0, 0]
    # the slot-index credit of ExchangeReturn pushed some deck count past 3
    assert max(st.deck()) > 3


@pytest.mark.gpu
def test_gpu_scripted_policies_match_oracle():
    import torch

    from open_spiel_coup_amd import BatchedCoupEnv
    n = 64
    env = BatchedCoupEnv(n, seed=5, auto_reset=False, obs=True, history=True)
    env.new_initial_state()  # chance node, no deals yet
    games = [oracle.OracleState() for _ in range(n)]
    policy = [i % N_POLICIES for i in range(n)]
    for step in range(260):
        q = env.query(obs=True, info_state=True)
        mask = q["legal_mask"].cpu().numpy().astype(np.uint32)
        term = q["terminal"].cpu().numpy()
        obs = q["obs"].cpu().numpy()
        info = q["info_state"].cpu().numpy()
        ret = q["returns"].cpu().numpy()
        rew = q["rewards"].cpu().numpy()
        actions = np.full(n, -1, np.int8)
        for i, g in enumerate(games):
            assert int(mask[i]) == oracle_mask(g), f"lane {i} step {step}"
            assert bool(term[i]) == g.is_terminal(), f"lane {i} step {step}"
            assert list(ret[i]) == g.returns(), f"lane {i} step {step}"
            if not g.is_chance_node():
                assert list(rew[i]) == g.rewards(), f"lane {i} step {step}"
            for p in (0, 1):
                np.testing.assert_array_equal(obs[i, p], g.observation_tensor(p), err_msg=f"lane {i} step {step}")
                np.testing.assert_array_equal(info[i, p], g.information_state_tensor(p),
                                              err_msg=f"lane {i} step {step}")
            if not g.is_terminal():
                a = choose(policy[i], oracle_mask(g), g.is_chance_node())
                g.apply_action(a)
                actions[i] = a
        if (actions < 0).all():
            break
        env.apply_action(torch.from_numpy(actions))
    assert all(g.is_terminal() for g in games), "scripted games did not finish"
    assert any(len(g.history()) == 91 for g in games), "no lane reached truncation"
    packed = env.export_state().cpu().numpy().astype(np.uint32)
    for i, g in enumerate(games):
        # coup_new_initial_state starts episode 1 (the env was created at episode 0)
        np.testing.assert_array_equal(packed[i], np.array(g.pack(episode=1), np.uint32), err_msg=f"lane {i}")
    assert env.error_count() == 0


def contract_deal(g, seed, env_id, episode):
    """Resolve pending deals of oracle game g by the sampling contract
    (DESIGN.md section 4): the draw of slot move_number_, r = u * total >> 32,
    the first card type whose cumulative deck count exceeds r."""
    while g.is_chance_node() and not g.is_terminal():
        u = oracle.draw(seed, env_id, episode, len(g.history()))
        deck = g.deck()
        r = (u * sum(deck)) >> 32
        cum = 0
        for t in range(5):
            cum += deck[t]
            if cum > r:
                break
        g.apply_action(t)


@pytest.mark.gpu
def test_gpu_step_kernel_scripted_actions_truncate():
    """The same policies through coup_step with external actions: the
    kernel resolves the deals from its Philox stream (including a deal run
    cut short by truncation), and a lane that finished is reset on its next
    step (rl_environment semantics, no auto-reset).  Every lane is mirrored
    by an oracle game dealt by the same contract."""
    import torch

    from open_spiel_coup_amd import BatchedCoupEnv
    n, seed = 128, 77
    env = BatchedCoupEnv(n, seed=seed, auto_reset=False, obs=True)
    games, episode = [], [0] * n
    for i in range(n):
        g = oracle.OracleState()
        contract_deal(g, seed, i, 0)
        games.append(g)
    policy = [i % N_POLICIES for i in range(n)]
    truncated = 0
    for step in range(300):
        actions = np.zeros(n, np.int8)
        for i, g in enumerate(games):
            if g.is_terminal():
                truncated += len(g.history()) == 91
                episode[i] += 1
                g = games[i] = oracle.OracleState()  # step() after LAST resets
                contract_deal(g, seed, i, episode[i])
            else:
                a = choose(policy[i], oracle_mask(g), False)
                g.apply_action(a)
                contract_deal(g, seed, i, episode[i])
                actions[i] = a
        o = env.step(torch.from_numpy(actions))
        mask = o["legal_mask"].cpu().numpy().astype(np.uint32)
        obs = o["obs"].cpu().numpy()
        for i, g in enumerate(games):
            assert int(mask[i]) == oracle_mask(g), f"lane {i} step {step}"
            for p in (0, 1):
                np.testing.assert_array_equal(obs[i, p], g.observation_tensor(p), err_msg=f"lane {i} step {step}")
    assert truncated > 0, "no game reached truncation"
    packed = env.export_state().cpu().numpy().astype(np.uint32)
    for i, g in enumerate(games):
        np.testing.assert_array_equal(packed[i], np.array(g.pack(episode=episode[i]), np.uint32), err_msg=f"lane {i}")
    assert env.error_count() == 0
