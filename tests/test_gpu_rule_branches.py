"""Directed playouts through the rule branches that no reference-held vector
reaches ("What's weak" 1): the lost Exchange challenge and
its recursion (coup.cc:708-720), lost Tax / Steal challenges (:696-701,
:753-761), the Assassinate refund (:743-748), and a challenged Steal block
held up by an Ambassador (:677-680), plus every other challenge, block and
pass case.

512 games run on the GPU through the State API (coup_apply_action, one lane
per game) and on the oracle side by side.  Chance outcomes are drawn from
the oracle's ChanceOutcomes; decisions prefer Challenge and Block, so the
rare branches come up hundreds of times.  After every action the GPU
records (all fields but the episode counter), legal masks, rewards and
returns equal the oracle's, and the ObservationTensors every 8th action.
The test asserts that every targeted branch was exercised."""
import collections

import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv  # noqa: E402

FA, TAX, ASSASSINATE, EXCHANGE, STEAL, PASS, BLOCK, CHALLENGE = 1, 3, 4, 5, 6, 9, 10, 11
ASSASSIN, AMBASSADOR, CAPTAIN, CONTESSA, DUKE = 0, 1, 2, 3, 4
NAMES = {FA: "foreign_aid", TAX: "tax", ASSASSINATE: "assassinate", EXCHANGE: "exchange", STEAL: "steal", 2: "coup",
         BLOCK: "block"}
CLAIMED = {TAX: DUKE, EXCHANGE: AMBASSADOR, ASSASSINATE: ASSASSIN, STEAL: CAPTAIN}
# record bits that hold the episode counter (w2 [31:29], w3 [31:7]): NewInitialState's
# episode is the env's, the oracle packs episode 0
EPISODE_MASK = np.array([0xFFFFFFFF, 0xFFFFFFFF, 0x1FFFFFFF, 0x7F], dtype=np.uint32)

TARGETS = ("challenge_exchange_holds", "challenge_tax_holds", "challenge_steal_holds", "challenge_assassinate_bluff",
           "challenge_steal_block_ambassador")


def _face_down(hand16):
    out = set()
    for i in range(4):
        k = (hand16 >> (4 * i)) & 0xF
        if k != 0xF and not k & 1:
            out.add(k >> 1)
    return out


def classify(words, a):
    """Branch of DoApplyAction that decision `a` takes at packed record `words`."""
    x, z = int(words[0]), int(words[2])
    M = (z >> 20) & 1
    O = 1 - M
    last = [z & 0x1F, (z >> 5) & 0x1F]
    op_last, cp_last = last[O], last[M]
    down = _face_down((x >> (16 * O)) & 0xFFFF)
    if a == CHALLENGE:
        if op_last == BLOCK:
            if cp_last == FA:
                return "challenge_foreign_aid_block_" + ("duke" if DUKE in down else "bluff")
            if cp_last == ASSASSINATE:
                return "challenge_assassinate_block_" + ("contessa" if CONTESSA in down else "bluff")
            return "challenge_steal_block_" + ("captain" if CAPTAIN in down else
                                               "ambassador" if AMBASSADOR in down else "bluff")
        return f"challenge_{NAMES[op_last]}_" + ("holds" if CLAIMED[op_last] in down else "bluff")
    if a == PASS:
        return "pass_" + NAMES.get(op_last, str(op_last))
    if a == BLOCK:
        return "block_" + NAMES.get(op_last, str(op_last))
    return None


def _np(t):
    return t.detach().cpu().numpy()


def test_directed_playouts_cover_rare_branches():
    B, iters = 512, 400
    rng = np.random.default_rng(2024)
    env = BatchedCoupEnv(B, seed=0, obs=True, auto_reset=False)
    env.new_initial_state()
    states = [oracle.OracleState() for _ in range(B)]
    seen = collections.Counter()
    games = 0
    for it in range(iters):
        acts = np.full(B, -1, np.int8)
        restart = np.zeros(B, np.uint8)
        for i, s in enumerate(states):
            if s.is_terminal():
                restart[i] = 1
                continue
            if s.is_chance_node():
                outs = s.chance_outcomes()
                a = int(rng.choice([o for o, _ in outs], p=[p for _, p in outs]))
            else:
                legal = s.legal_actions()
                if CHALLENGE in legal and rng.random() < 0.6:
                    a = CHALLENGE
                elif BLOCK in legal and rng.random() < 0.5:
                    a = BLOCK
                else:
                    a = int(rng.choice(legal))
                cat = classify(s.pack(0), a)
                if cat:
                    seen[cat] += 1
            s.apply_action(a)
            acts[i] = a
        env.apply_action(torch.from_numpy(acts))  # -1: lane left as it is
        if restart.any():  # finished games start over on both sides
            games += int(restart.sum())
            env.new_initial_state(torch.from_numpy(restart))
            for i in np.nonzero(restart)[0]:
                states[i] = oracle.OracleState()
        words = _np(env.export_state()).astype(np.uint32).reshape(B, 4)
        want = np.array([s.pack(0) for s in states], dtype=np.uint32).reshape(B, 4)
        np.testing.assert_array_equal(words & EPISODE_MASK, want & EPISODE_MASK, err_msg=f"iteration {it}")
        q = env.query(obs=it % 8 == 0)
        # chance nodes carry the flag bit 31 beside the card types (coup_mi355x.h)
        np.testing.assert_array_equal(_np(q["legal_mask"]).astype(np.uint32) & 0x7FFFFFFF,
                                      np.array([s.legal_mask() for s in states], dtype=np.uint32))
        np.testing.assert_array_equal(_np(q["current_player"]), np.array([s.current_player() for s in states]))
        np.testing.assert_array_equal(_np(q["rewards"]), np.array([s.rewards() for s in states], dtype=np.int8))
        np.testing.assert_array_equal(_np(q["returns"]), np.array([s.returns() for s in states], dtype=np.int8))
        if it % 8 == 0:
            obs = _np(q["obs"])
            for i in range(0, B, 37):
                for p in (0, 1):
                    np.testing.assert_array_equal(obs[i, p], states[i].observation_tensor(p))
    assert env.error_count() == 0
    assert games > 100
    print("\nbranch counts:", dict(sorted(seen.items())))
    for t in TARGETS:
        assert seen[t] >= 5, (t, dict(seen))
    # every challenge case the rules distinguish came up
    challenge_cases = [k for k in seen if k.startswith("challenge_")]
    assert len(challenge_cases) >= 14, sorted(challenge_cases)
