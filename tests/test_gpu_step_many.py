"""coup_step_many / coup_step_trajectory with observations in the
rules-trajectory form (COUP_PIPE=1, the default):
chunks of up to COUP_TRAJ_CHUNK steps run as ONE regrouped rules-trajectory
launch (k_trajectory_sorted<1024, true>) that also stores every step's
post-step records, then one k_obs_sweep_rows<512, 2> launch per step reading
them.  It must equal coup_step launched once per step (COUP_PIPE=0: the
split step's two kernels per step) bit for bit -- the last step's outputs,
the records, the episode accumulators and the error count -- for every
chunk length (a chunk ending mid-call, episodes ending on a chunk's last
step), ragged batches, graph capture, and as a trajectory with every step's
observations in [T][B][2][98] slices.  The oracle side at the bench size is
tests/test_gpu_headline.py.  Reference semantics: ObservationTensor
coup.cc:1051-1056, 248-287; the transition coup.cc:522-808;
rl_environment.py:243-248 (both players' tensors every step)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv, _native  # noqa: E402

KEYS = ("actions", "rewards", "step_type", "legal_mask", "current_player", "obs")


# COUP_PIPE: the rules trajectory on the env's stream (the measurement
# build's overlapped form, "3", runs these tests from
# tests/ab_variants/test_ab_overlap.py)
FORMS = ["1"]


def _env(monkeypatch, B, traj, seed, chunk=None, word=False, stage=None):
    """traj: a COUP_PIPE form ("1" / "3"), or False for per-step coup_step;
    stage: COUP_MANY_STAGE."""
    if stage is None:
        monkeypatch.delenv("COUP_MANY_STAGE", raising=False)
    else:
        monkeypatch.setenv("COUP_MANY_STAGE", stage)
    monkeypatch.setenv("COUP_OBS_SPLIT", "11")  # the shipped writer at every size (the default from 2^20)
    monkeypatch.setenv("COUP_REGROUP", "1")     # the regrouped rules at every size (the default from 2^18)
    monkeypatch.setenv("COUP_PIPE", traj if traj else "0")
    if chunk is None:
        monkeypatch.delenv("COUP_TRAJ_CHUNK", raising=False)
    else:
        monkeypatch.setenv("COUP_TRAJ_CHUNK", str(chunk))
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


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("B", [3, 1000, 65536 + 77, (1 << 18) + 5])
def test_step_many_equals_stepping(monkeypatch, B, form):
    seed = 11
    many, ref = _env(monkeypatch, B, form, seed), _env(monkeypatch, B, False, seed)
    for K in (1, 2, 5, 8, 3, 17):  # below, at and above one chunk, one call after the other on the same env
        many.step_many(K)
        for _ in range(K):
            ref.step()
        _same(_state(many), _state(ref), f"B {B} after K={K}")
    assert many.error_count() == ref.error_count() == 0


@pytest.mark.parametrize("stage", [None])  # "1" (COUP_MANY_STAGE): tests/ab_variants/test_ab_overlap.py
@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("chunk", [1, 3, 8, 32])
def test_chunk_length_invariant(monkeypatch, chunk, form, stage):
    """How the steps split into rules-trajectory launches changes no result
    (episodes that end on a chunk's last step reset in the next launch), nor
    whether the outputs are staged by lane (COUP_MANY_STAGE)."""
    B, seed = 70001, 3
    many = _env(monkeypatch, B, form, seed, chunk=chunk, stage=stage)
    ref = _env(monkeypatch, B, False, seed)
    many.step_many(23)
    for _ in range(23):
        ref.step()
    _same(_state(many), _state(ref), f"chunk {chunk}")


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("chunk", [2, 8])
def test_graph_capture_and_packed_word(monkeypatch, form, chunk):
    """capture_steps records coup_step_many (bench.py's timed region); two
    replays equal 2 K eager steps, the packed int16 episode word included.
    The overlapped form's second stream joins the capture (its resources
    made by the eager steps before it)."""
    B, seed, K = 50000, 21, 9
    many = _env(monkeypatch, B, form, seed, chunk=chunk, word=True)
    ref = _env(monkeypatch, B, False, seed, word=True)
    for _ in range(3):
        many.step()
        ref.step()
    many.step_many(1)  # makes the overlapped form's stream and buffers outside the capture
    ref.step()
    many.clear_episode_stats()
    ref.clear_episode_stats()
    g = many.capture_steps(K)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    for _ in range(2 * K):
        ref.step()
    assert torch.equal(many.episode_word, ref.episode_word)
    _same(_state(many), _state(ref), "graph")


@pytest.mark.parametrize("stage", [None])  # "1" (COUP_MANY_STAGE): tests/ab_variants/test_ab_overlap.py
@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("B,T", [(1000, 12), (1 << 20, 10), (1 << 20, 21)])
def test_trajectory_slices_every_step(monkeypatch, B, T, form, stage):
    """coup_step_trajectory with observations through the rules-trajectory
    forms: every step's outputs in its slice, equal to one coup_step per
    slice (outputs stored from the playing threads, or staged by lane)."""
    seed = 17
    many, ref = _env(monkeypatch, B, form, seed, stage=stage), _env(monkeypatch, B, False, seed)
    for env in (many, ref):
        env.rollout(30)
    bp = many.collect_trajectory(T)
    br = ref.trajectory_buffers(T)
    ref._bind_stream()
    for t in range(T):
        _native.check(ref.lib.coup_step(ref._h, None, ctypes.byref(ref._slice_outputs(br, t))))
    for k in KEYS:
        assert torch.equal(bp[k], br[k]), k
    assert torch.equal(many.export_state(), ref.export_state())
    for a, b in zip(many.episode_stats(), ref.episode_stats()):
        assert torch.equal(a, b)


def test_default_form_by_batch(monkeypatch):
    """Without COUP_OBS_SPLIT / COUP_REGROUP the rules-trajectory form
    applies from 2^20 lanes (the split step's size); below it coup_step_many
    loops over the fused step."""
    for k in ("COUP_OBS_SPLIT", "COUP_REGROUP", "COUP_PIPE", "COUP_TRAJ_CHUNK"):
        monkeypatch.delenv(k, raising=False)
    lib = _native.load()
    assert lib.coup_obs_split_variant(1 << 20) == 11
    assert lib.coup_obs_split_variant((1 << 20) - 1) == 0
    a = BatchedCoupEnv(4096, seed=2, obs=True)
    b = BatchedCoupEnv(4096, seed=2, obs=True)
    a.step_many(4)
    for _ in range(4):
        b.step()
    assert torch.equal(a.obs, b.obs) and torch.equal(a.export_state(), b.export_state())



def _bare_state(env):
    out = {k: v.cpu().numpy().copy() for k, v in
           (("actions", env.actions), ("rewards", env.rewards), ("step_type", env.step_type),
            ("legal_mask", env.legal_mask), ("current_player", env.cur_player))}
    eps, ret = env.episode_stats()
    return out, env.export_state().cpu().numpy(), eps.cpu().numpy(), ret.cpu().numpy()


@pytest.mark.parametrize("players", [2, 3, 6])
@pytest.mark.parametrize("B", [1000, (1 << 18) + 5])
def test_bare_step_many_equals_stepping(monkeypatch, players, B):
    """coup_step_many without tensors: ONE trajectory launch (in place below
    2^18 lanes, regrouped from it; 2 and N players) whose every step's
    outputs overwrite the [B] buffers -- equal to coup_step launched once
    per step (COUP_PIPE=0): the last step's outputs, the records, the
    accumulators and the error count, eager and captured in a graph."""
    seed = 5 + players
    monkeypatch.delenv("COUP_OBS_SPLIT", raising=False)
    monkeypatch.delenv("COUP_REGROUP", raising=False)
    kw = dict(seed=seed, auto_reset=True, obs=False, num_players=players, episode_stats=True)
    monkeypatch.setenv("COUP_PIPE", "1")
    many = BatchedCoupEnv(B, **kw)
    monkeypatch.setenv("COUP_PIPE", "0")
    ref = BatchedCoupEnv(B, **kw)
    for K in (1, 7, 20):
        many.step_many(K)
        for _ in range(K):
            ref.step()
        a, b = _bare_state(many), _bare_state(ref)
        for k in a[0]:
            np.testing.assert_array_equal(a[0][k], b[0][k], err_msg=f"{players}p B {B} K {K}: {k}")
        for x, y, what in zip(a[1:], b[1:], ("records", "episodes", "return sums")):
            np.testing.assert_array_equal(x, y, err_msg=f"{players}p B {B} K {K}: {what}")
    g = many.capture_steps(9)
    g.replay()
    torch.cuda.synchronize()
    for _ in range(9):
        ref.step()
    np.testing.assert_array_equal(many.export_state().cpu().numpy(), ref.export_state().cpu().numpy())
    assert torch.equal(many.legal_mask, ref.legal_mask) and torch.equal(many.actions, ref.actions)
    assert many.error_count() == ref.error_count() == 0


@pytest.mark.parametrize("obs", [True, False])
def test_step_many_without_auto_reset(monkeypatch, obs):
    """Without auto-reset a finished lane reports LAST (terminal record, no
    legal actions) and restarts at the next step (FIRST), in both
    coup_step_many forms (rules trajectory + writers with observations; one
    trajectory launch without): equal to per-step coup_step."""
    B, seed = 5000, 31
    monkeypatch.setenv("COUP_OBS_SPLIT", "11")
    monkeypatch.setenv("COUP_REGROUP", "1")
    kw = dict(seed=seed, auto_reset=False, obs=obs, episode_stats=True)
    monkeypatch.setenv("COUP_PIPE", "1")
    many = BatchedCoupEnv(B, **kw)
    monkeypatch.setenv("COUP_PIPE", "0")
    ref = BatchedCoupEnv(B, **kw)
    for K in (9, 30, 17):
        many.step_many(K)
        for _ in range(K):
            ref.step()
        a, b = (_state(many), _state(ref)) if obs else (_bare_state(many), _bare_state(ref))
        for k in a[0]:
            np.testing.assert_array_equal(a[0][k], b[0][k], err_msg=f"K {K}: {k}")
        for x, y in zip(a[1:], b[1:]):
            np.testing.assert_array_equal(x, y)
    assert many.error_count() == ref.error_count() == 0
