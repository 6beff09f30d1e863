"""Measurement build (tests/ab_variants/conftest.py): the merged pipelined
split observation step (coup_step_many COUP_PIPE=2, k_step_obs_pipe;
DESIGN.md section 5, measured slower than the serial and rules-trajectory
forms): one launch runs the rules of step t + 1 beside the
observation writer of step t, the records alternating between two buffers.
It must equal coup_step launched once per step (COUP_PIPE=0: the split
step's two kernels per step) bit for bit -- the last step's outputs, the
records, the episode accumulators and the error count -- for odd and even
step counts (the first rules launch runs in place when the count is odd),
ragged batches (the last writer block partial), any spread of the rules
blocks over the launch (COUP_PIPE_SPAN), graph capture, and as a
trajectory with every step's observations in [T][B][2][98] slices.  The
oracle side at the bench size is tests/test_gpu_headline.py.  Reference
semantics: ObservationTensor coup.cc:1051-1056, 248-287; the transition
coup.cc:522-808; rl_environment.py:243-248 (both players' tensors every
step)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv, _native  # noqa: E402

KEYS = ("actions", "rewards", "step_type", "legal_mask", "current_player", "obs")


def _env(monkeypatch, B, pipe, seed, span=None, word=False):
    monkeypatch.setenv("COUP_OBS_SPLIT", "11")  # the shipped writer at every size (the default from 2^20)
    monkeypatch.setenv("COUP_PIPE", "2" if pipe else "0")
    if span is None:
        monkeypatch.delenv("COUP_PIPE_SPAN", raising=False)
    else:
        monkeypatch.setenv("COUP_PIPE_SPAN", str(span))
    return BatchedCoupEnv(B, seed=seed, auto_reset=True, obs=True, episode_stats=2 if word else True)


def _state(env):
    out = {k: v.cpu().numpy().copy() for k, v in
           (("actions", env.actions), ("rewards", env.rewards), ("step_type", env.step_type),
            ("legal_mask", env.legal_mask), ("current_player", env.cur_player), ("obs", env.obs))}
    eps, ret = env.episode_stats()
    return out, env.export_state().cpu().numpy(), eps.cpu().numpy(), ret.cpu().numpy()


def _same(a, b, what):
    for k in KEYS:
        np.testing.assert_array_equal(a[0][k], b[0][k], err_msg=f"{what}: {k}")
    np.testing.assert_array_equal(a[1], b[1], err_msg=f"{what}: records")
    np.testing.assert_array_equal(a[2], b[2], err_msg=f"{what}: episodes")
    np.testing.assert_array_equal(a[3], b[3], err_msg=f"{what}: return sums")


@pytest.mark.parametrize("B", [3, 65536 + 77, (1 << 18) + 5])
def test_step_many_equals_stepping(monkeypatch, B):
    seed = 11
    pipe, ref = _env(monkeypatch, B, True, seed), _env(monkeypatch, B, False, seed)
    for K in (1, 2, 5, 8, 3):  # odd and even counts, one after the other on the same env
        pipe.step_many(K)
        for _ in range(K):
            ref.step()
        _same(_state(pipe), _state(ref), f"B {B} after K={K}")
    assert pipe.error_count() == ref.error_count() == 0


@pytest.mark.parametrize("span", [0.01, 0.5, 1.0])
def test_rules_block_spread_invariant(monkeypatch, span):
    """Where the rules blocks sit among the writer blocks changes no result."""
    B, seed = 70001, 3
    pipe, ref = _env(monkeypatch, B, True, seed, span=span), _env(monkeypatch, B, False, seed)
    pipe.step_many(7)
    for _ in range(7):
        ref.step()
    _same(_state(pipe), _state(ref), f"span {span}")


def test_graph_capture_and_packed_word(monkeypatch):
    """capture_steps records coup_step_many (bench.py's timed region); two
    replays equal 2 K eager steps, the packed int16 episode word included."""
    B, seed, K = 50000, 21, 9
    pipe, ref = _env(monkeypatch, B, True, seed, word=True), _env(monkeypatch, B, False, seed, word=True)
    for _ in range(3):
        pipe.step()
        ref.step()
    pipe.clear_episode_stats()
    ref.clear_episode_stats()
    g = pipe.capture_steps(K)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    for _ in range(2 * K):
        ref.step()
    assert torch.equal(pipe.episode_word, ref.episode_word)
    _same(_state(pipe), _state(ref), "graph")


@pytest.mark.parametrize("B", [1000])
def test_trajectory_slices_every_step(monkeypatch, B):
    """coup_step_trajectory with observations through the pipeline: every
    step's outputs in its slice, equal to one coup_step per slice."""
    T, seed = (12 if B < (1 << 20) else 5), 17
    pipe, ref = _env(monkeypatch, B, True, seed), _env(monkeypatch, B, False, seed)
    for env in (pipe, ref):
        env.rollout(30)
    bp = pipe.collect_trajectory(T)
    br = ref.trajectory_buffers(T)
    ref._bind_stream()
    for t in range(T):
        _native.check(ref.lib.coup_step(ref._h, None, ctypes.byref(ref._slice_outputs(br, t))))
    for k in KEYS:
        assert torch.equal(bp[k], br[k]), k
    assert torch.equal(pipe.export_state(), ref.export_state())
    for a, b in zip(pipe.episode_stats(), ref.episode_stats()):
        assert torch.equal(a, b)

