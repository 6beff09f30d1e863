"""Measurement build (tests/ab_variants/conftest.py): the N-player
kernels' rejected schedules and block sizes against the shipped ones --
the next decision drawn in the step instead of ahead (COUP_AHEAD=0),
256 / 512 / 1024-lane regrouping blocks (COUP_NP_SORT_THREADS), one thread
per reset or resets dealt where the game ends (COUP_NP_RESET_GROUP /
_INLINE), the rollout's per-lane bin prefix (COUP_NP_SCAN=0).  Parity
unpinned w.r.t. the 2-player reference for N > 2 (coup.h:42); every form
must give the same lanes."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv  # noqa: E402


@pytest.mark.parametrize("ahead", ["0"], ids=["drawn-in-step"])
@pytest.mark.parametrize("n_players", [2, 4, 6])
@pytest.mark.parametrize("auto_reset", [True, False])
def test_regrouped_step_equals_in_place_step(monkeypatch, n_players, auto_reset, ahead):
    """k_step_sorted (lanes counting-sorted by decision through LDS, resets
    dealt by the first threads) == k_step (lanes in place), ragged batch,
    both the uniform policy and caller actions (about 1 in 8 illegal, so
    the rejected-action path is in the sort too); with the next uniform
    decision drawn ahead and parked in the record (the default) and without.
    Exported records carry no parked decision."""
    monkeypatch.setenv("COUP_AHEAD", ahead)
    n, steps, seed = 1000, 150, 11 + n_players
    envs = {}
    for knob in ("0", "1"):
        monkeypatch.setenv("COUP_REGROUP", knob)
        envs[knob] = BatchedCoupEnv(n, seed=seed, env_id_base=3 << 20, auto_reset=auto_reset, obs=False,
                                    num_players=n_players, generic=True)
    g = torch.Generator().manual_seed(seed)
    for t in range(steps):
        acts = None
        if t % 3 == 2:
            legal = envs["0"].query(obs=False)["legal_mask"].cpu().to(torch.int64)
            acts = torch.randint(0, 18, (n,), generator=g, dtype=torch.int64)
            ok = ((legal >> acts) & 1) == 1
            keep = torch.rand(n, generator=g) < 0.875
            # pick a legal action where there is one, except for the kept illegal ones
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

@pytest.mark.parametrize("n_players", [3, 6])
def test_regrouped_step_block_size_invariant(monkeypatch, n_players):
    """The uniform regrouped step sorting 256-, 512- or 1024-lane blocks
    (COUP_NP_SORT_THREADS, A/B variants) == the default 256-lane blocks: the
    sort only changes which wave runs a lane, never its result.  Ragged
    batch, auto-reset, episode accumulators."""
    n, steps, seed = 1000, 150, 5 + n_players
    knobs = ("256", "512", "1024")
    envs = {}
    monkeypatch.setenv("COUP_REGROUP", "1")
    for knob in knobs:
        monkeypatch.setenv("COUP_NP_SORT_THREADS", knob)
        envs[knob] = BatchedCoupEnv(n, seed=seed, env_id_base=7 << 20, auto_reset=True, obs=False,
                                    num_players=n_players, generic=True, episode_stats=True)
    for t in range(steps):
        outs = {}
        for knob, env in envs.items():
            monkeypatch.setenv("COUP_NP_SORT_THREADS", knob)
            outs[knob] = {k: v.clone() for k, v in env.step().items()}
        for knob in knobs[1:]:
            for k in ("actions", "rewards", "step_type", "legal_mask", "current_player"):
                assert torch.equal(outs["256"][k], outs[knob][k]), (knob, t, k)
            assert torch.equal(envs["256"].export_state(), envs[knob].export_state()), (knob, t)
    for knob in knobs[1:]:
        for a, b in zip(envs["256"].episode_stats(), envs[knob].episode_stats()):
            assert torch.equal(a, b), knob
        assert envs[knob].error_count() == 0
    assert int(envs["256"].episode_stats()[0].sum()) > 0
    assert envs["256"].error_count() == 0

@pytest.mark.parametrize("n_players", [2, 6])
def test_regrouped_rollout_block_size_invariant(monkeypatch, n_players):
    """k_rollout_sorted over 256-, 512- and 1024-lane blocks (1024 the
    default) agree: records and per-lane statistics, ragged batch, launches of 1, 9
    and 140 steps, starting mid-game."""
    n, seed = 3000, 61 + n_players
    knobs = ("256", "512", "1024")
    monkeypatch.setenv("COUP_REGROUP", "1")
    envs, stats = {}, {}
    for knob in knobs:
        monkeypatch.setenv("COUP_NP_SORT_THREADS", knob)
        env = BatchedCoupEnv(n, seed=seed, auto_reset=True, obs=False, num_players=n_players, generic=True)
        for _ in range(25):
            env.step()
        envs[knob], stats[knob] = env, env.new_stats()
    for k in (1, 9, 140):
        for knob, env in envs.items():
            monkeypatch.setenv("COUP_NP_SORT_THREADS", knob)
            env.rollout(k, stats[knob])
        for knob in knobs[1:]:
            assert torch.equal(envs["256"].export_state(), envs[knob].export_state()), (knob, k)
            for key in ("episodes", "return_sum", "length_sum"):
                assert torch.equal(stats["256"][key], stats[knob][key]), (knob, k, key)
    assert int(stats["256"]["episodes"].sum()) > 0
    assert all(env.error_count() == 0 for env in envs.values())


@pytest.mark.parametrize("n_players", [3, 6])
@pytest.mark.parametrize("lanes", ["256", "1024"])
def test_regrouped_step_reset_schedule_invariant(monkeypatch, n_players, lanes):
    """The regrouped uniform step's auto-reset schedules agree lane by lane:
    the block's resets in a phase of their own, each dealt by a group of 4
    threads sharing the Philox blocks (the default), or by one thread
    (COUP_NP_RESET_GROUP=1); and resets dealt where the game ends
    (COUP_NP_RESET_INLINE=1, decisions that end a game drawn ahead as
    kKeyEnding).  So does an env alternating the kernels, where a decision
    parked by one is played by another.  Outputs, records, accumulators."""
    n, steps, seed = 3000, 200, 40 + n_players
    monkeypatch.setenv("COUP_REGROUP", "1")
    monkeypatch.setenv("COUP_NP_SORT_THREADS", lanes)
    forms = {"phase": ("0", "4"), "single": ("0", "1"), "inline": ("1", "4")}
    envs = {}
    for knob in ("phase", "single", "inline", "alt"):  # the knobs are read at coup_create
        inline, group = forms[knob if knob != "alt" else "phase"]
        monkeypatch.setenv("COUP_NP_RESET_INLINE", inline)
        monkeypatch.setenv("COUP_NP_RESET_GROUP", group)
        envs[knob] = BatchedCoupEnv(n, seed=seed, env_id_base=9 << 20, auto_reset=True, obs=False,
                                    num_players=n_players, generic=True, episode_stats=True)
    cycle = ("phase", "inline", "single")
    for t in range(steps):
        outs = {}
        for knob, env in envs.items():
            inline, group = forms[knob if knob != "alt" else cycle[t % 3]]
            monkeypatch.setenv("COUP_NP_RESET_INLINE", inline)
            monkeypatch.setenv("COUP_NP_RESET_GROUP", group)
            env.reload_knobs()  # the knobs are read at coup_create; "alt" switches its kernel every step
            outs[knob] = {k: v.clone() for k, v in env.step().items()}
        for knob in ("single", "inline", "alt"):
            for k in ("actions", "rewards", "step_type", "legal_mask", "current_player"):
                assert torch.equal(outs["phase"][k], outs[knob][k]), (knob, t, k)
            assert torch.equal(envs["phase"].export_state(), envs[knob].export_state()), (knob, t)
    for knob in ("single", "inline", "alt"):
        for x, y in zip(envs["phase"].episode_stats(), envs[knob].episode_stats()):
            assert torch.equal(x, y), knob
    assert int(envs["phase"].episode_stats()[0].sum()) > 100
    assert all(env.error_count() == 0 for env in envs.values())


@pytest.mark.parametrize("n_players", [3, 6])
def test_regrouped_rollout_scan_forms_equal(monkeypatch, n_players):
    """The sorted rollout's bin prefix computed by every wave for itself
    (wave_bins_below, the default) == its round-2 per-lane sums
    (COUP_NP_SCAN=0), 1024-lane blocks, ragged batch, starting mid-game:
    records and statistics after launches of 1, 9 and 60 steps."""
    n, seed = 2500, 71 + n_players
    monkeypatch.setenv("COUP_REGROUP", "1")
    monkeypatch.setenv("COUP_NP_SORT_THREADS", "1024")
    envs = {}
    for knob in ("1", "0"):  # the knobs are read at coup_create
        monkeypatch.setenv("COUP_NP_SCAN", knob)
        envs[knob] = BatchedCoupEnv(n, seed=seed, env_id_base=3 << 20, auto_reset=True, obs=False,
                                    num_players=n_players, generic=True)
    for env in envs.values():
        for _ in range(20):
            env.step()
    stats = {knob: env.new_stats() for knob, env in envs.items()}
    for k in (1, 9, 60):
        for knob, env in envs.items():
            monkeypatch.setenv("COUP_NP_SCAN", knob)
            env.rollout(k, stats[knob])
        assert torch.equal(envs["1"].export_state(), envs["0"].export_state()), k
        for key in ("episodes", "return_sum", "length_sum"):
            assert torch.equal(stats["1"][key], stats["0"][key]), (k, key)
    assert int(stats["1"]["episodes"].sum()) > 0
    assert all(env.error_count() == 0 for env in envs.values())
