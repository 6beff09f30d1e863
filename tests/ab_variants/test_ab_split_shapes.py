"""Measurement build (tests/ab_variants/conftest.py): every writer shape the
split steps were measured with (COUP_OBS_SPLIT 1..17, COUP_INFO_SPLIT 1..5).

The split observation step (COUP_OBS_SPLIT, the default from 2^20 lanes):
the rules step without tensors, then coup::k_obs_sweep writing every lane's
ObservationTensor pair from the post-step records in address order.  It must
equal the fused step (k_step<*, kObsWaveBitsSc1>, COUP_OBS_SPLIT=0) bit for
bit: observations, records, every small output and the episode
accumulators, at every step -- uniform policy and caller actions (skipped
lanes, rejected actions, the unchecked env), ragged batches whose last 4 KiB
chunk is partial, and the headline size.  The oracle side of the same
observations is tests/test_gpu_headline.py (c3 at 2^20 lanes, now split).
Reference semantics: ObservationTensor coup.cc:1051-1056, 248-287."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv  # noqa: E402

KEYS = ("actions", "rewards", "step_type", "legal_mask", "current_player", "obs")


def _run(monkeypatch, split, B, steps, seed=5, actions_fn=None, unchecked=False, auto_reset=True):
    monkeypatch.setenv("COUP_OBS_SPLIT", str(split))
    env = BatchedCoupEnv(B, seed=seed, auto_reset=auto_reset, obs=True, device="cuda", episode_stats=True,
                         unchecked=unchecked)
    outs = []
    for t in range(steps):
        o = env.step(actions_fn(env, t) if actions_fn else None)
        outs.append({k: o[k].cpu().numpy().copy() for k in KEYS})
    eps, ret = env.episode_stats()
    res = (outs, env.export_state().cpu().numpy(), eps.cpu().numpy(), ret.cpu().numpy(), env.error_count())
    env.close()
    return res


def _same(a, b, what):
    for t, (x, y) in enumerate(zip(a[0], b[0])):
        for k in KEYS:
            np.testing.assert_array_equal(x[k], y[k], err_msg=f"{what}: {k} at step {t}")
    np.testing.assert_array_equal(a[1], b[1], err_msg=f"{what}: records")
    np.testing.assert_array_equal(a[2], b[2], err_msg=f"{what}: episodes")
    np.testing.assert_array_equal(a[3], b[3], err_msg=f"{what}: return sums")
    assert a[4] == b[4], what


@pytest.mark.parametrize("B", [3, 1000, 65536 + 77, 1 << 18])
def test_split_equals_fused_uniform(monkeypatch, B):
    steps = 40 if B <= 65613 else 12
    ref = _run(monkeypatch, 0, B, steps)
    # 1: k_obs_sweep (NT stores), 2: plain stores, 3-7 and 9-17:
    # k_obs_sweep_rows shapes (11 the default from 2^20 lanes)
    for split in [v for v in range(1, 18) if v != 8]:
        _same(_run(monkeypatch, split, B, steps), ref, f"split {split} B {B}")


INFO_KEYS = ("actions", "rewards", "step_type", "legal_mask", "current_player", "info_state")


def _run_info(monkeypatch, split, B, steps, seed=7, actions_fn=None):
    monkeypatch.setenv("COUP_INFO_SPLIT", str(split))
    env = BatchedCoupEnv(B, seed=seed, auto_reset=True, obs=False, info_state=True, history=True, device="cuda",
                         episode_stats=True)
    outs = []
    for t in range(steps):
        o = env.step(actions_fn(env, t) if actions_fn else None)
        outs.append({k: o[k].cpu().numpy().copy() for k in INFO_KEYS})
    eps, ret = env.episode_stats()
    res = (outs, env.export_state().cpu().numpy(), env.export_history().cpu().numpy(), eps.cpu().numpy(),
           ret.cpu().numpy(), env.error_count())
    env.close()
    return res


@pytest.mark.parametrize("B", [3, 1000, 4099, 1 << 18])
def test_info_split_equals_fused(monkeypatch, B):
    """COUP_INFO_SPLIT: the history-keeping rules step, then k_info_sweep
    writing the InformationStateTensor (coup.cc:1044-1049) in address order
    -- every shape equal to the fused writer (k_step<*, 0, 256, kInfoWrite>)
    bit for bit, with the histories, records and episode words."""
    steps = 30 if B < (1 << 18) else 4
    ref = _run_info(monkeypatch, 0, B, steps)
    for split in (1, 2, 3, 4, 5):
        got = _run_info(monkeypatch, split, B, steps)
        for t, (x, y) in enumerate(zip(got[0], ref[0])):
            for k in INFO_KEYS:
                np.testing.assert_array_equal(x[k], y[k], err_msg=f"info split {split} B {B}: {k} at step {t}")
        for i in range(1, 5):
            np.testing.assert_array_equal(got[i], ref[i], err_msg=f"info split {split} B {B}: part {i}")
        assert got[5] == ref[5]


@pytest.mark.parametrize("pol", ["1", "2", "3"])
@pytest.mark.parametrize("B", [1000, 4099])
def test_info_writer_store_policies(monkeypatch, B, pol):
    """COUP_WRITER_POL: k_info_sweep<1024, 2>'s stores plain, sc1 or sc1 nt
    buffer stores (through the block's own resource, whose range drops the
    stores past the batch) instead of non-temporal ones: the same tensors."""
    steps = 12
    ref = _run_info(monkeypatch, 0, B, steps)
    monkeypatch.setenv("COUP_WRITER_POL", pol)
    got = _run_info(monkeypatch, 3, B, steps)
    monkeypatch.delenv("COUP_WRITER_POL")
    for t, (x, y) in enumerate(zip(got[0], ref[0])):
        for k in INFO_KEYS:
            np.testing.assert_array_equal(x[k], y[k], err_msg=f"pol {pol} B {B}: {k} at step {t}")
