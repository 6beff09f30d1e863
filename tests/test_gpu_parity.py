"""Parity of the HIP path (through the C ABI) with the oracle and with the
reference's golden vectors.  Bit-exact everywhere: integer state, legal
masks, rewards, step types and the fp32 observation tensors (whose values
are exact small integers)."""
import numpy as np
import pytest
import torch

from oracle import oracle
from tests import golden_util as G

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv, packed  # noqa: E402


def _np(t):
    return t.detach().cpu().numpy()


def _mask_to_list(m):
    m = int(m) & 0x3FFFF
    return [a for a in range(18) if (m >> a) & 1]


# ------------------------------------------------------------------ goldens

def test_kat_scenarios_batched():
    """All 14 coup_test.cc scenarios at once, one lane each, through
    coup_apply_action / coup_query / coup_export_state."""
    kats = G.load_kats()
    B = len(kats)
    env = BatchedCoupEnv(B, seed=0, obs=False)
    env.new_initial_state()
    maxlen = max(len(s["actions"]) for s in kats)
    checks = {(i, c["after"]): c for i, s in enumerate(kats) for c in s["checks"]}
    for k in range(maxlen + 1):
        if k > 0:
            acts = torch.tensor([s["actions"][k - 1] if k - 1 < len(s["actions"]) else -1 for s in kats],
                                dtype=torch.int8)
            env.apply_action(acts)
        q = env.query(obs=False)
        words = _np(env.export_state())
        legal, cur, term = _np(q["legal_mask"]), _np(q["current_player"]), _np(q["terminal"])
        rew, ret = _np(q["rewards"]), _np(q["returns"])
        for i in range(B):
            c = checks.get((i, k))
            if c is None:
                continue
            r = packed.lane(words, i)
            G.check_kat(c, lambda p: r["cards"][p], lambda p: r["coins"][p], lambda p: r["last_action"][p],
                        lambda: int(cur[i]), lambda: _mask_to_list(legal[i]), lambda: bool(term[i]),
                        lambda: rew[i].tolist(), lambda: ret[i].tolist())
    assert env.error_count() == 0


def test_playthrough_transcript():
    """Replay coup.txt's history; compare every recorded field (legal sets,
    chance probabilities, current player, rewards, returns, obs tensors)."""
    pt = G.load_playthrough()["states"]
    env = BatchedCoupEnv(1, seed=0, obs=False)
    env.new_initial_state()
    hist = pt[-1]["history"]
    for k in range(len(hist) + 1):
        if k > 0:
            env.apply_action(torch.tensor([hist[k - 1]], dtype=torch.int8))
        rec = pt[k]
        assert rec["history"] == hist[:k]
        q = env.query()
        r = packed.lane(_np(env.export_state()), 0)
        assert r["move_number"] == k
        if "current_player" not in rec:
            continue
        cur, term = int(_np(q["current_player"])[0]), bool(_np(q["terminal"])[0])
        assert cur == rec["current_player"] and term == rec["is_terminal"]
        mask = int(_np(q["legal_mask"])[0]) & 0xFFFFFFFF
        if rec["is_chance"]:
            assert mask & (1 << 31)
            assert _mask_to_list(mask & 0x1F) == rec["legal_actions"]
            total = float(sum(r["deck"]))
            got = [(t, r["deck"][t] / total) for t in range(5) if r["deck"][t] > 0]
            assert got == [tuple(x) for x in rec["chance_outcomes"]]
        else:
            if not term:
                assert _mask_to_list(mask) == rec["legal_actions"]
            assert _np(q["rewards"])[0].tolist() == [int(x) for x in rec["rewards"]]
            assert _np(q["returns"])[0].tolist() == [int(x) for x in rec["returns"]]
        obs = _np(q["obs"])[0]
        for p in (0, 1):
            np.testing.assert_array_equal(obs[p], G.dense(rec["ObservationTensor"][str(p)], 98))


# --------------------------------------------------------- oracle rollouts

@pytest.mark.parametrize("auto_reset", [True, False])
def test_uniform_rollout_matches_oracle(auto_reset):
    """coup_step with the in-kernel uniform policy == the oracle's rollout
    under the same sampling contract: actions, rewards, step types, legal
    masks and obs at every step, final packed state bit for bit."""
    n, steps, seed, base = 2048, 160, 11, 1000
    ref = oracle.rollout(seed=seed, n=n, steps=steps, env_id_base=base, auto_reset=auto_reset, want_obs=True)
    env = BatchedCoupEnv(n, seed=seed, env_id_base=base, auto_reset=auto_reset, obs=True)
    for t in range(steps):
        o = env.step()
        np.testing.assert_array_equal(_np(o["actions"]), ref["actions"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(_np(o["rewards"]), ref["rewards"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(_np(o["step_type"]), ref["step_type"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(_np(o["legal_mask"]).astype(np.uint32), ref["legal"][t],
                                      err_msg=f"step {t}")
        np.testing.assert_array_equal(_np(o["obs"]), ref["obs"][t], err_msg=f"step {t}")
    np.testing.assert_array_equal(_np(env.export_state()).astype(np.uint32), ref["final_state"])
    assert env.error_count() == 0


@pytest.mark.parametrize("n", [1000, 8 * 256 * 3 + 1000])
def test_obs_writer_matches_oracle(n):
    """The fused step's observation writer (the wave-cooperative bitmap, sc1
    buffer stores) gives the oracle's tensors, including a ragged last wave
    (1000 lanes = 15 full waves + 40) and, at 7144 lanes (27 full blocks +
    232 lanes), the XCD-aware block -> group remap with blocks past the last
    round of 8.  The rejected writers: tests/ab_variants/test_ab_parity.py."""
    steps, seed = 40, 17
    ref = oracle.rollout(seed=seed, n=n, steps=steps, want_obs=True)
    env = BatchedCoupEnv(n, seed=seed, obs=True)
    guard = torch.full((n + 64, 2, 98), -7.0, device="cuda")
    env.set_output("obs", guard[:n])
    for t in range(steps):
        o = env.step()
        np.testing.assert_array_equal(_np(o["obs"]), ref["obs"][t], err_msg=f"step {t}")
    assert torch.all(guard[n:] == -7.0), "writer touched memory past the last lane"


def test_playthrough_information_state():
    """InformationStateTensor (perfect recall, history block) of both players
    at every recorded state of coup.txt, via coup_query on an env keeping
    histories."""
    pt = G.load_playthrough()["states"]
    env = BatchedCoupEnv(1, seed=0, obs=False, history=True)
    env.new_initial_state()
    hist = pt[-1]["history"]
    for k in range(len(hist) + 1):
        if k > 0:
            env.apply_action(torch.tensor([hist[k - 1]], dtype=torch.int8))
        rec = pt[k]
        if "InformationStateTensor" not in rec:
            continue
        info = _np(env.query(obs=False, info_state=True)["info_state"])[0]
        for p in (0, 1):
            np.testing.assert_array_equal(info[p], G.dense(rec["InformationStateTensor"][str(p)], 2492),
                                          err_msg=f"state {k} player {p}")


@pytest.mark.parametrize("auto_reset", [True, False])
def test_info_state_rollout_matches_oracle(auto_reset):
    """coup_step writing InformationStateTensor x2 every step (ragged batch of
    200 lanes) == the oracle; histories match byte for byte."""
    n, steps, seed = 200, 48, 31
    ref = oracle.rollout(seed=seed, n=n, steps=steps, auto_reset=auto_reset, want_obs=True, want_info=True)
    env = BatchedCoupEnv(n, seed=seed, auto_reset=auto_reset, obs=True, info_state=True)
    for t in range(steps):
        o = env.step()
        np.testing.assert_array_equal(_np(o["actions"]), ref["actions"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(_np(o["obs"]), ref["obs"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(_np(o["info_state"]), ref["info"][t], err_msg=f"step {t}")
    np.testing.assert_array_equal(_np(env.export_state()).astype(np.uint32), ref["final_state"])
    h = _np(env.export_history())
    moves = packed.decode(ref["final_state"])["move_number"]
    for lane in range(n):
        m = int(moves[lane])
        assert bytes(h[lane, :m]) == bytes(ref["final_hist"][lane, :m]), lane
    assert env.error_count() == 0


def test_history_kept_by_apply_and_step():
    """History bytes recorded by coup_apply_action (State API) equal the
    oracle's for the KAT action sequences."""
    kats = G.load_kats()
    env = BatchedCoupEnv(len(kats), seed=0, obs=False, history=True)
    env.new_initial_state()
    maxlen = max(len(s["actions"]) for s in kats)
    for k in range(maxlen):
        env.apply_action(torch.tensor([s["actions"][k] if k < len(s["actions"]) else -1 for s in kats],
                                      dtype=torch.int8))
    h = _np(env.export_history())
    for i, s in enumerate(kats):
        st = oracle.OracleState()
        for a in s["actions"]:
            st.apply_action(a)
        m = len(s["actions"])
        assert bytes(h[i, :m]) == st.history_bytes()[:m], s["name"]


def test_c2_eager_step_matches_oracle_every_step():
    """BASELINE config 2's batch with EAGER per-step launches: 65,536 lanes,
    in-kernel uniform policy (random_agent.py:29-42), no observations, one
    coup_step per step (the group-Philox step k_step_group<1, true>;
    regrouping starts at 2^18 lanes) -- what a learner passing actions each
    step runs, and bench.py's c2 warm-up.  bench.py's timed c2 steps are ONE
    coup_step_many trajectory launch instead (k_step_trajectory, output
    stride 0): tests/test_gpu_every_lane.py checks that form on every lane.
    Every lane's action, rewards, step type and post-step legal mask
    (LegalActions, coup.cc:824-938) equal the oracle's at each of 160 steps;
    so do the per-lane episode accumulators and the final records."""
    from open_spiel_coup_amd import _native  # noqa: F401
    n, steps, seed = 65536, 160, 1
    assert n < (1 << 18)  # the in-place kernel, not k_step_sorted
    ref = oracle.rollout(seed=seed, n=n, steps=steps)
    env = BatchedCoupEnv(n, seed=seed, obs=False, episode_stats=True)
    for t in range(steps):
        o = env.step()
        np.testing.assert_array_equal(_np(o["actions"]), ref["actions"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(_np(o["rewards"]), ref["rewards"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(_np(o["step_type"]), ref["step_type"][t], err_msg=f"step {t}")
        np.testing.assert_array_equal(_np(o["legal_mask"]).astype(np.uint32), ref["legal"][t], err_msg=f"step {t}")
    np.testing.assert_array_equal(_np(env.export_state()).astype(np.uint32), ref["final_state"])
    eps, ret = env.episode_stats()
    np.testing.assert_array_equal(_np(eps), ref["lane_episodes"])
    np.testing.assert_array_equal(_np(ret), ref["lane_return_sum"])
    assert env.error_count() == 0


@pytest.mark.parametrize("regroup", ["1", "0"], ids=["regrouped", "in-place"])
@pytest.mark.parametrize("auto_reset", [True, False])
def test_episode_stats_match_oracle(monkeypatch, regroup, auto_reset):
    """coup_step's per-episode accumulators (episodes, player-0 return sum
    per lane) == the oracle's, with the obs writer on and off, in place and
    regrouped by decision."""
    monkeypatch.setenv("COUP_REGROUP", regroup)
    n, steps, seed = 3000, 120, 8
    ref = oracle.rollout(seed=seed, n=n, steps=steps, auto_reset=auto_reset, want_trajectory=False)
    for obs in (False, True):
        env = BatchedCoupEnv(n, seed=seed, auto_reset=auto_reset, obs=obs, episode_stats=True)
        for _ in range(steps):
            env.step()
        eps, ret = env.episode_stats()
        np.testing.assert_array_equal(_np(eps), ref["lane_episodes"], err_msg=f"obs={obs}")
        np.testing.assert_array_equal(_np(ret), ref["lane_return_sum"], err_msg=f"obs={obs}")
        env.clear_episode_stats()
        assert int(env.episode_stats()[0].sum()) == 0


def test_traffic_ceiling_kernel_leaves_records():
    """coup_measure_step_traffic (bench.py's in-process store ceiling) stores
    every record back unchanged and writes the full obs buffer, ragged
    batch included, nothing past it."""
    import ctypes
    from open_spiel_coup_amd import _native
    n = 1000
    env = BatchedCoupEnv(n, seed=3, obs=True)
    for _ in range(5):
        env.step()
    rec = env.export_state()
    before = rec.clone()
    guard = torch.full((n + 64, 2, 98), -7.0, device="cuda")
    out = _native.StepOutputs(None, None, None, None, None, guard.data_ptr())
    _native.check(env.lib.coup_measure_step_traffic(n, ctypes.c_void_p(rec.data_ptr()), ctypes.byref(out),
                                                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    assert torch.equal(rec, before)
    assert torch.all(guard[n:] == -7.0) and not torch.any(guard[:n] == -7.0)


def test_external_actions_replay():
    """Feeding the oracle's chosen actions back through coup_step(actions)
    reproduces the same trajectory (chance deals depend only on the env's
    stream, not on who chose the decision)."""
    n, steps, seed = 1024, 120, 5
    ref = oracle.rollout(seed=seed, n=n, steps=steps, auto_reset=True)
    env = BatchedCoupEnv(n, seed=seed, auto_reset=True, obs=False)
    for t in range(steps):
        o = env.step(torch.from_numpy(ref["actions"][t]).cuda())
        np.testing.assert_array_equal(_np(o["rewards"]), ref["rewards"][t])
        np.testing.assert_array_equal(_np(o["legal_mask"]).astype(np.uint32), ref["legal"][t])
    np.testing.assert_array_equal(_np(env.export_state()).astype(np.uint32), ref["final_state"])
    assert env.error_count() == 0


@pytest.mark.parametrize("regroup", ["1", "0"], ids=["regrouped", "in-place"])
def test_fused_rollout_matches_oracle(monkeypatch, regroup):
    """coup_rollout (K steps per launch) lands on the same states and episode
    statistics as the oracle, with the lanes regrouped by decision every
    step (coup_regroup.h, the default from 2^18 lanes) and in place.
    Ragged batch."""
    monkeypatch.setenv("COUP_REGROUP", regroup)
    n, steps, seed = 4000, 300, 21
    ref = oracle.rollout(seed=seed, n=n, steps=steps, auto_reset=True, want_trajectory=False)
    env = BatchedCoupEnv(n, seed=seed, auto_reset=True, obs=False)
    stats = env.new_stats()
    env.rollout(100, stats)
    env.rollout(200, stats)
    np.testing.assert_array_equal(_np(env.export_state()).astype(np.uint32), ref["final_state"])
    assert int(stats["episodes"].sum()) == int(ref["episodes_done"][0])
    assert int(stats["return_sum"].sum()) == int(ref["return_sum_p0"][0])
    assert env.error_count() == 0


def test_regrouped_rollout_equals_in_place_rollout(monkeypatch):
    """k_rollout_sorted == k_rollout lane by lane (records and per-lane
    statistics), starting from terminal records (auto_reset off) and from
    records at the first chance node, launches of 1, 5 and 120 steps."""
    n, seed = 1500, 31
    envs, stats = {}, {}
    for knob in ("0", "1"):
        monkeypatch.setenv("COUP_REGROUP", knob)
        env = BatchedCoupEnv(n, seed=seed, auto_reset=False, obs=False)
        for _ in range(30):
            env.step()
        envs[knob], stats[knob] = env, env.new_stats()
    for k in (1, 5, 120, -7):
        for knob, env in envs.items():
            monkeypatch.setenv("COUP_REGROUP", knob)
            if k < 0:
                env.new_initial_state()
            env.rollout(abs(k), stats[knob])
        assert torch.equal(envs["0"].export_state(), envs["1"].export_state()), k
        for key in ("episodes", "return_sum", "length_sum"):
            assert torch.equal(stats["0"][key], stats["1"][key]), (k, key)
    assert envs["0"].error_count() == envs["1"].error_count() == 0


@pytest.mark.parametrize("auto_reset", [True, False])
def test_regrouped_step_equals_in_place_step(monkeypatch, auto_reset):
    """k_step_sorted (the bare step with lanes counting-sorted by decision,
    resets dealt by the first threads; default from 2^18 lanes) == k_step,
    ragged batch, uniform policy and caller actions (about 1 in 8 illegal)."""
    n, steps, seed = 1000, 150, 41
    envs = {}
    for knob in ("0", "1"):
        monkeypatch.setenv("COUP_REGROUP", knob)
        envs[knob] = BatchedCoupEnv(n, seed=seed, env_id_base=123_457, auto_reset=auto_reset, obs=False)
    g = torch.Generator().manual_seed(seed)
    for t in range(steps):
        acts = None
        if t % 3 == 2:
            legal = envs["0"].query(obs=False)["legal_mask"].cpu().to(torch.int64)
            acts = torch.randint(0, 18, (n,), generator=g, dtype=torch.int64)
            ok = ((legal >> acts) & 1) == 1
            keep = torch.rand(n, generator=g) < 0.875
            first = torch.where(legal != 0, (legal & -legal).float().log2().to(torch.int64), acts)
            acts = torch.where(ok | ~keep, acts, first).to(torch.int8)
        outs = {}
        for knob, env in envs.items():
            monkeypatch.setenv("COUP_REGROUP", knob)
            outs[knob] = {k: v.clone() for k, v in env.step(acts).items()}
        for k in ("actions", "rewards", "step_type", "legal_mask", "current_player"):
            assert torch.equal(outs["0"][k], outs["1"][k]), (t, k)
        assert torch.equal(envs["0"].export_state(), envs["1"].export_state()), t
    assert envs["0"].error_count() == envs["1"].error_count()
