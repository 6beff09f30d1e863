"""The host-resident per-game State ops of libcoup_mi355x.so
(coup_host_state_init / _apply / _tensors, csrc/coup_host.cpp: the product's
rules header coup_lane.h and tensor decoders coup_tensor.h built for the
host) against the oracle: random games mixing legal actions, chance outcomes
and arbitrary action ids through the unchecked apply (pyspiel's apply_action,
spiel.cc:322-331), every record, history, legal mask, player, reward,
return and both players' tensors compared after every action.  Host code
only: no device call, so this runs in the CPU suite; the facade tests
(-m gpu) run the same functions through pyspiel."""
import ctypes

import numpy as np
import pytest

from oracle import oracle

from open_spiel_coup_amd import _native

RESULT = 128


def _lib():
    try:
        return _native.load()
    except (ImportError, OSError) as e:  # the library is not built in this checkout
        pytest.skip(f"libcoup_mi355x.so not loadable: {e}")


def _fields(raw):
    rec = np.frombuffer(raw, np.uint32, 4, 0)
    hist = np.frombuffer(raw, np.uint8, 96, 16)
    lm, cp, term, ok, unrep = np.frombuffer(raw, np.uint32, 1, 112)[0], *np.frombuffer(raw, np.int8, 1, 116), \
        raw[117], raw[118], raw[119]
    rew = np.frombuffer(raw, np.int8, 2, 120)
    ret = np.frombuffer(raw, np.int8, 2, 122)
    return rec, hist, int(lm), int(cp), term, ok, unrep, rew, ret


def _check(lib, raw, ref, what):
    rec, hist, lm, cp, term, _, _, rew, ret = _fields(raw)
    assert rec.tolist() == [int(x) for x in ref.pack(0)], what
    n = len(ref.history())
    assert bytes(hist[:min(n, 96)]) == ref.history_bytes()[:min(n, 96)], what
    assert cp == ref.current_player(), what
    assert bool(term) == ref.is_terminal(), what
    if not ref.is_terminal():
        assert lm & 0x7FFFFFFF == ref.legal_mask(), what  # bit 31 marks a chance node
    assert rew.tolist() == ref.rewards() and ret.tolist() == ref.returns(), what
    obs = np.zeros((2, 98), np.float32)
    info = np.zeros((2, 2492), np.float32)
    assert lib.coup_host_state_tensors(raw, obs.ctypes.data, info.ctypes.data) == 0
    for p in (0, 1):
        np.testing.assert_array_equal(obs[p], ref.observation_tensor(p), err_msg=what)
        np.testing.assert_array_equal(info[p], ref.information_state_tensor(p), err_msg=what)


def test_host_states_walk_matches_oracle():
    lib = _lib()
    rng = np.random.default_rng(17)
    out = ctypes.create_string_buffer(RESULT)
    accepted = rejected = unrep_seen = 0
    for g in range(60):
        assert lib.coup_host_state_init(out) == 0
        raw = out.raw
        ref = oracle.OracleState()
        _check(lib, raw, ref, f"game {g} start")
        for k in range(150):
            if ref.is_terminal():
                break
            legal = ref.legal_actions()
            a = int(rng.choice(legal)) if legal and (ref.is_chance_node() or rng.random() < 0.7) else int(rng.integers(18))
            assert lib.coup_host_state_apply(raw, a, _native.SLOT_UNCHECKED, out) == 0
            new = out.raw
            r2 = ref.clone()
            try:
                r2.apply_action_unchecked(a)
                code = 0
            except RuntimeError as e:
                code = int(str(e).rsplit(" ", 1)[1])
            ok, unrep = new[118], new[119]
            what = f"game {g} step {k} action {a}"
            assert ok == (code == 0), what
            assert unrep == (code == 4), what
            if ok:
                accepted += 1
                ref = r2
                raw = new
            else:
                rejected += 1
                unrep_seen += unrep
                assert new[:112] == raw[:112], what  # record and history unchanged
            _check(lib, new, ref, what)
    assert accepted > 1000 and rejected > 50


def test_host_checked_apply_refuses_illegal_actions():
    """Without COUP_SLOT_UNCHECKED the legality check applies
    (State::ApplyActionWithLegalityCheck's effect): legal actions as the
    oracle's apply_action, any other id rejected, the state unchanged."""
    lib = _lib()
    rng = np.random.default_rng(3)
    out = ctypes.create_string_buffer(RESULT)
    for g in range(20):
        lib.coup_host_state_init(out)
        raw, ref = out.raw, oracle.OracleState()
        while not ref.is_terminal():
            legal = ref.legal_actions()
            bad = [a for a in range(18) if a not in legal]
            if bad:
                b = int(rng.choice(bad))
                assert lib.coup_host_state_apply(raw, b, 0, out) == 0
                assert out.raw[118] == 0 and out.raw[:112] == raw[:112]
            a = int(rng.choice(legal))
            assert lib.coup_host_state_apply(raw, a, 0, out) == 0
            assert out.raw[118] == 1
            ref.apply_action(a)
            raw = out.raw
            _check(lib, raw, ref, f"game {g}")


def test_host_apply_argument_checks():
    lib = _lib()
    out = ctypes.create_string_buffer(RESULT)
    lib.coup_host_state_init(out)
    raw = out.raw
    # ids 18..127: a rejected action (ok = 0, record and history unchanged), as
    # coup_host_state_step reports it; -1 and 128 are invalid arguments
    for a in (18, 127):
        for flags in (0, _native.SLOT_UNCHECKED):
            assert lib.coup_host_state_apply(raw, a, flags, out) == 0
            assert out.raw[118] == 0 and out.raw[:112] == raw[:112], (a, flags)
    assert lib.coup_host_state_apply(raw, 128, 0, out) == _native.COUP_E_INVALID
    assert lib.coup_host_state_apply(raw, -1, 0, out) == _native.COUP_E_INVALID
    assert lib.coup_host_state_apply(None, 0, 0, out) == _native.COUP_E_INVALID
    assert lib.coup_host_state_tensors(None, None, None) == _native.COUP_E_INVALID


def _host_string(lib, raw, kind, player):
    buf = ctypes.create_string_buffer(64)
    n = lib.coup_host_state_string(raw, kind, player, buf, 64)
    assert n >= 0
    if n >= 64:
        buf = ctypes.create_string_buffer(n + 1)
        assert lib.coup_host_state_string(raw, kind, player, buf, n + 1) == n
    return buf.value.decode()


def test_host_strings_match_oracle_and_python_forms():
    """coup_host_state_string (ObservationString / InformationStateString /
    ToString, coup.cc:290-373 and 945-987) against the oracle's strings and
    the facade's Python formatter (strings.py) on random states, legal and
    unchecked play, both observers."""
    from open_spiel_coup_amd import strings
    lib = _lib()
    rng = np.random.default_rng(5)
    out = ctypes.create_string_buffer(RESULT)
    seen = 0
    for g in range(40):
        lib.coup_host_state_init(out)
        raw, ref = out.raw, oracle.OracleState()
        for k in range(120):
            words = np.frombuffer(raw, np.uint32, 4, 0).reshape(1, 4)
            hist = np.frombuffer(raw, np.uint8, 96, 16)
            for p in (0, 1):
                o = _host_string(lib, raw, 0, p)
                i = _host_string(lib, raw, 1, p)
                assert o == ref.observation_string(p) == strings.observation_string(words, hist, p)
                assert i == ref.information_state_string(p) == strings.information_state_string(words, hist, p)
            assert _host_string(lib, raw, 2, 0) == ref.to_string() == strings.to_string(words, hist)
            seen += 1
            if ref.is_terminal():
                break
            legal = ref.legal_actions()
            a = int(rng.choice(legal)) if legal and rng.random() < 0.85 else int(rng.integers(18))
            lib.coup_host_state_apply(raw, a, _native.SLOT_UNCHECKED, out)
            if out.raw[118]:
                ref.apply_action_unchecked(a)
                raw = out.raw
    assert seen > 500
    assert lib.coup_host_state_string(raw, 3, 0, None, 0) == -1
    assert lib.coup_host_state_string(raw, 0, 2, None, 0) == -1


def test_host_env_steps_replay_the_oracle_rollout():
    """coup_host_state_step (rl_environment's reset / step on a host state,
    the device lane ops' COUP_SLOT_RESET / COUP_SLOT_DEAL): driven with the
    oracle rollout's own decisions, lanes of several env ids, no auto-reset
    (LAST, then the next step starts the next episode), the host lanes deal
    the same cards -- every record equal to the oracle's at the end, and
    every step type, reward and legal mask on the way."""
    import ctypes as C
    lib = _lib()
    seed, K = 0x1234_5678_9ABC_DEF0, 400
    out = C.create_string_buffer(RESULT)
    for env_id in (0, 1, 77, 4096):
        ref = oracle.rollout(seed=seed, n=1, steps=K, env_id_base=env_id, auto_reset=False)
        assert lib.coup_host_state_step(None, -1, _native.SLOT_INIT | _native.SLOT_DEAL, seed, env_id, out) == 0
        raw = out.raw
        for t in range(K):
            st = int(ref["step_type"][t][0])
            if st == 0:  # FIRST: the step after LAST started the next episode
                mode, a = _native.SLOT_RESET | _native.SLOT_DEAL, -1
            else:
                mode, a = _native.SLOT_DEAL | _native.SLOT_UNCHECKED, int(ref["actions"][t][0])
            assert lib.coup_host_state_step(raw, a, mode, seed, env_id, out) == 0
            raw = out.raw
            assert raw[118] == 1, (env_id, t)
            rec, hist, lm, cp, term, _, _, rew, ret = _fields(raw)
            assert (2 if term else (0 if st == 0 else 1)) == st, (env_id, t)
            assert rew[0] == ref["rewards"][t][0][0], (env_id, t)
            assert (lm & 0xFFFFFFFF) == int(ref["legal"][t][0]), (env_id, t)
        rec = np.frombuffer(raw, np.uint32, 4, 0)
        assert rec.tolist() == ref["final_state"][0].tolist(), env_id
