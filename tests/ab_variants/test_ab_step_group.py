"""Measurement build (tests/ab_variants/conftest.py).

coup::k_step_group (COUP_STEP_TPL = 1 / 2 / 4): the rules-bound step with
the Philox blocks one step can need computed ahead by the lane's thread
group (PrefRng) and traded by DPP (TPL 1, the default, computes them in
one thread with ILP), against the plain k_step (COUP_STEP_TPL=0) and the
oracle.  Same sampling contract, so the same games: every
output of every step, the records and the episode accumulators are equal,
at c2's batch (65,536 lanes: one wave per SIMD) and ragged batches whose
last group is partial.  Caller actions (legal, illegal: counted once per
lane) and rl_environment semantics (auto_reset off, LAST then reset) too.
Reference semantics: coup.cc:490-809 (the transition), random_agent.py:29-42
with spiel.cc:258-294 (the draws)."""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv  # noqa: E402

KEYS = ("actions", "rewards", "step_type", "legal_mask", "current_player")


def _run(monkeypatch, tpl, B, steps, seed=3, auto_reset=True, actions_fn=None, env_id_base=0):
    monkeypatch.setenv("COUP_STEP_TPL", str(tpl))  # 0: k_step
    env = BatchedCoupEnv(B, seed=seed, auto_reset=auto_reset, obs=False, device="cuda", episode_stats=True,
                         env_id_base=env_id_base)
    outs = []
    for t in range(steps):
        a = actions_fn(env, t) if actions_fn else None
        o = env.step(a)
        outs.append({k: o[k].cpu().numpy().copy() for k in KEYS})
    eps, ret = env.episode_stats()
    res = (outs, env.export_state().cpu().numpy(), eps.cpu().numpy(), ret.cpu().numpy(), env.error_count())
    env.close()
    return res


def _same(a, b, what):
    outs_a, rec_a, eps_a, ret_a, err_a = a
    outs_b, rec_b, eps_b, ret_b, err_b = b
    for t, (x, y) in enumerate(zip(outs_a, outs_b)):
        for k in KEYS:
            np.testing.assert_array_equal(x[k], y[k], err_msg=f"{what}: {k} at step {t}")
    np.testing.assert_array_equal(rec_a, rec_b, err_msg=f"{what}: records")
    np.testing.assert_array_equal(eps_a, eps_b, err_msg=f"{what}: episodes")
    np.testing.assert_array_equal(ret_a, ret_b, err_msg=f"{what}: return sums")
    assert err_a == err_b, what


@pytest.mark.parametrize("B", [65536, 65536 + 77, 1000, 3])
def test_group_step_equals_k_step_uniform(monkeypatch, B):
    ref = _run(monkeypatch, 0, B, 80)
    for tpl in (1, 2, 4):
        _same(_run(monkeypatch, tpl, B, 80), ref, f"TPL {tpl} B {B}")


@pytest.mark.parametrize("tpl", [1, 4])
def test_group_step_equals_oracle_slices(monkeypatch, tpl):
    """k_step_group at c2's batch (TPL 1: the default c2 kernel) against the
    oracle directly, on three 256-lane slices at every step."""
    B, K = 65536, 60
    outs, rec, _, _, err = _run(monkeypatch, tpl, B, K, seed=11)
    assert err == 0
    for k in (0, B // 2 + 77, B - 256):
        ref = oracle.rollout(seed=11, n=256, steps=K, env_id_base=k)
        for t in range(K):
            sl = slice(k, k + 256)
            np.testing.assert_array_equal(outs[t]["actions"][sl], ref["actions"][t], err_msg=f"{k} {t}")
            np.testing.assert_array_equal(outs[t]["rewards"][sl], ref["rewards"][t], err_msg=f"{k} {t}")
            np.testing.assert_array_equal(outs[t]["step_type"][sl], ref["step_type"][t], err_msg=f"{k} {t}")
            np.testing.assert_array_equal(outs[t]["legal_mask"][sl].astype(np.uint32), ref["legal"][t],
                                          err_msg=f"{k} {t}")
        np.testing.assert_array_equal(rec[k:k + 256].view(np.uint32), ref["final_state"], err_msg=f"records {k}")


def test_group_step_caller_actions_and_errors(monkeypatch):
    """Caller actions: a legal pick per lane from the last legal mask, with
    some lanes given an illegal action (left unchanged, counted once per
    lane even though four threads play it) and some skipped (-1); no auto
    reset (rl_environment: LAST, then a reset on the next step)."""
    B = 4099

    def actions(env, t):
        g = torch.Generator().manual_seed(t)
        m = env.legal_mask.cpu().to(torch.int64) & 0x3FFFF
        u = torch.randint(0, 1 << 30, (B,), generator=g)
        acts = torch.zeros(B, dtype=torch.int64)
        for lane in range(B):
            bits = [a for a in range(18) if (int(m[lane]) >> a) & 1]
            acts[lane] = bits[int(u[lane]) % len(bits)] if bits else 0
        if t % 5 == 3:
            acts[::97] = 17  # mostly illegal (ExchangeReturn34 outside an exchange)
        acts[5::211] = -1
        return acts

    ref = _run(monkeypatch, 0, B, 24, auto_reset=False, actions_fn=actions)
    assert ref[4] > 0
    for tpl in (1, 2, 4):
        _same(_run(monkeypatch, tpl, B, 24, auto_reset=False, actions_fn=actions), ref, f"caller TPL {tpl}")


def test_group_step_env_id_base_and_default_kernel(monkeypatch):
    """Lanes keyed by env_id_base + i (a rank's shard), and an out-of-range
    value selects k_step."""
    ref = _run(monkeypatch, 0, 2048, 30, env_id_base=123457)
    _same(_run(monkeypatch, 4, 2048, 30, env_id_base=123457), ref, "env_id_base")
    monkeypatch.setenv("COUP_STEP_TPL", "3")
    env = BatchedCoupEnv(64, seed=3, obs=False, device="cuda")
    env.step()
    assert env.error_count() == 0
