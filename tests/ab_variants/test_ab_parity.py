"""Measurement build (tests/ab_variants/conftest.py): the fused step's
rejected observation writers (COUP_OBS_MODE 1..8, the XCD remap off) against
the oracle, and the 2-player regrouped kernels' block sizes
(COUP_SORT_THREADS 256 / 512 / 1024) against each other.  Reference
semantics: coup.cc:248-287 (ObservationTensor), :522-808."""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv  # noqa: E402


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("mode", ["1", "2", "3", "4", "5", "6", "7", "8", "9"])
@pytest.mark.parametrize("n,remap", [(1000, "1"), (8 * 256 * 3 + 1000, "1"), (8 * 256 * 3 + 1000, "0")])
def test_obs_writers_match_oracle(mode, n, remap, monkeypatch):
    """Every observation writer (per-lane rows, wave-cooperative from keys,
    bitmap, block-cooperative; plain / nt stores) gives
    the oracle's tensors, including a ragged last wave (1000 lanes = 15 full
    waves + 40) and, at 7144 lanes (27 full blocks + 232 lanes), the
    XCD-aware block -> group remap with blocks past the last round of 8."""
    monkeypatch.setenv("COUP_OBS_MODE", mode)
    monkeypatch.setenv("COUP_XCD_REMAP", remap)
    steps, seed = 40, 17
    ref = oracle.rollout(seed=seed, n=n, steps=steps, want_obs=True)
    env = BatchedCoupEnv(n, seed=seed, obs=True)
    guard = torch.full((n + 64, 2, 98), -7.0, device="cuda")
    env.set_output("obs", guard[:n])
    for t in range(steps):
        o = env.step()
        np.testing.assert_array_equal(_np(o["obs"]), ref["obs"][t], err_msg=f"mode {mode} step {t}")
    assert torch.all(guard[n:] == -7.0), "writer touched memory past the last lane"


def test_regrouped_block_size_invariant(monkeypatch):
    """2-player k_step_sorted (uniform and caller actions) and
    k_rollout_sorted over 256-, 512- and 1024-lane blocks
    (COUP_SORT_THREADS) agree lane by lane: records, outputs, statistics."""
    n, seed = 3000, 53
    knobs = ("256", "512", "1024")
    monkeypatch.setenv("COUP_REGROUP", "1")
    envs, stats = {}, {}
    for knob in knobs:
        monkeypatch.setenv("COUP_SORT_THREADS", knob)
        envs[knob] = BatchedCoupEnv(n, seed=seed, env_id_base=99, auto_reset=True, obs=False, episode_stats=True)
        stats[knob] = envs[knob].new_stats()
    g = torch.Generator().manual_seed(seed)
    for t in range(90):
        acts = None
        if t % 4 == 3:
            legal = envs["256"].query(obs=False)["legal_mask"].cpu().to(torch.int64)
            first = torch.where(legal != 0, (legal & -legal).float().log2().to(torch.int64), torch.zeros_like(legal))
            acts = first.to(torch.int8)
        outs = {}
        for knob, env in envs.items():
            monkeypatch.setenv("COUP_SORT_THREADS", knob)
            outs[knob] = {k: v.clone() for k, v in env.step(acts).items()}
        for knob in knobs[1:]:
            for k in outs["256"]:
                assert torch.equal(outs["256"][k], outs[knob][k]), (knob, t, k)
            assert torch.equal(envs["256"].export_state(), envs[knob].export_state()), (knob, t)
    for steps in (1, 40):
        for knob, env in envs.items():
            monkeypatch.setenv("COUP_SORT_THREADS", knob)
            env.rollout(steps, stats[knob])
        for knob in knobs[1:]:
            assert torch.equal(envs["256"].export_state(), envs[knob].export_state()), (knob, steps)
            for key in stats["256"]:
                assert torch.equal(stats["256"][key], stats[knob][key]), (knob, key)
    for knob in knobs[1:]:
        for a, b in zip(envs["256"].episode_stats(), envs[knob].episode_stats()):
            assert torch.equal(a, b)
    assert int(stats["256"]["episodes"].sum()) > 0
    assert all(env.error_count() == 0 for env in envs.values())
