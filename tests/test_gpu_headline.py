"""The bench's own kernels at the bench's own sizes, against the oracle.

bench.py's c3 line (the BASELINE metric) runs the split observation step
over 2^20 lanes: settle through the fused rollout, W warm-up steps, then K
steps replayed from one HIP graph (BatchedCoupEnv.capture_steps), which
records coup_step_many -- the rules-trajectory form: chunks of up to 8
steps as one regrouped rules-trajectory launch (k_trajectory_sorted<1024,
true>, the branch-form transition apply_decision_v1) storing every step's
records, then the address-order observation writer k_obs_sweep_rows<512, 2>
once per step.  Its timed region keeps only the last
step's tensors, so the same launches also run as a trajectory whose every
step lands in its own [T][B][2][98] slice, checked step by step.  c3i runs
the history-keeping rules step and k_info_sweep<1024, 2> over 2^18 lanes
with eager launches.  The oracle cannot afford 2^20 lanes per step, but
lanes are independent and keyed by their global env id (DESIGN.md section
4), so three 256-lane slices -- the start, an odd offset in the middle, the
end -- are checked against the oracle run on those env ids alone, at every
timed step: actions, rewards, step types, legal masks, current players,
both tensors of every lane, and the full 16-byte records (word 3:
turn_number_ and episode bits, the word the code-generation hazard of
DESIGN.md section 12 corrupted) and per-episode accumulators at the phase
boundaries.  Reference semantics: coup.cc:248-287 (ObservationTensor),
:230-245 (InformationStateTensor), :522-808 (the transition)."""
import numpy as np
import pytest
import torch

import bench
from oracle import oracle

pytestmark = pytest.mark.gpu

from open_spiel_coup_amd import BatchedCoupEnv  # noqa: E402


def _np(t):
    return t.detach().cpu().numpy()


def _slices(B):
    return (0, B // 2 + 77, B - 256)


def _cur_player_of_records(words):
    """CurrentPlayer of packed 2-player records: the
    bench's lanes are never at a chance node or terminal after an
    auto-reset step, so it is cur_player_move_ (w2 bit 20)."""
    return ((words[:, 2] >> 20) & 1).astype(np.int8)


def _check_step(o, ref, t, k, obs_key):
    sl = slice(k, k + 256)
    msg = f"slice {k} step {t}"
    np.testing.assert_array_equal(_np(o["actions"][sl]), ref["actions"][t], err_msg=msg)
    np.testing.assert_array_equal(_np(o["rewards"][sl]), ref["rewards"][t], err_msg=msg)
    np.testing.assert_array_equal(_np(o["step_type"][sl]), ref["step_type"][t], err_msg=msg)
    np.testing.assert_array_equal(_np(o["legal_mask"][sl]).astype(np.uint32), ref["legal"][t], err_msg=msg)
    if obs_key == "obs":
        np.testing.assert_array_equal(_np(o["obs"][sl]), ref["obs"][t], err_msg=msg)
    elif obs_key == "info":
        np.testing.assert_array_equal(_np(o["info_state"][sl]), ref["info"][t], err_msg=msg)


def _check_records(env, B, seed, steps, stats_from=None, cur_player=None):
    """Full records (and, with stats_from, the per-episode accumulators since
    step `stats_from`) of the three slices after `steps` steps; cur_player:
    the last step's current players (default: the env's output buffer)."""
    words = _np(env.export_state()).astype(np.uint32)
    cur = _np(env.cur_player if cur_player is None else cur_player)
    hist = _np(env.export_history()) if env.history else None
    for k in _slices(B):
        ref = oracle.rollout(seed=seed, n=256, steps=steps, env_id_base=k, auto_reset=True, want_trajectory=False)
        np.testing.assert_array_equal(words[k:k + 256], ref["final_state"], err_msg=f"records, slice {k}")
        np.testing.assert_array_equal(cur[k:k + 256], _cur_player_of_records(ref["final_state"]),
                                      err_msg=f"current player, slice {k}")
        if hist is not None:
            # entries past move_number_ are stale in both
            mv = (ref["final_state"][:, 2] >> 22) & 0x7F
            for j in range(256):
                np.testing.assert_array_equal(hist[k + j, :mv[j]], ref["final_hist"][j, :mv[j]],
                                              err_msg=f"history, lane {k + j}")
        if stats_from is not None:
            base = oracle.rollout(seed=seed, n=256, steps=stats_from, env_id_base=k, auto_reset=True,
                                  want_trajectory=False)
            eps, ret = env.episode_stats()
            np.testing.assert_array_equal(_np(eps[k:k + 256]), ref["lane_episodes"] - base["lane_episodes"],
                                          err_msg=f"episodes, slice {k}")
            np.testing.assert_array_equal(_np(ret[k:k + 256]), ref["lane_return_sum"] - base["lane_return_sum"],
                                          err_msg=f"return sums, slice {k}")


def test_c3_headline_kernel_full_batch_slices_match_oracle():
    """bench.py --config c3 at its size: 2^20 lanes, obs x2, settle 256 +
    warm-up 5, then K = 20 eager coup_step launches, K = 20 replays of a
    1-step graph (each step checked), one replay of a K = 20-step graph
    (bench.py's timed region, coup_step_many's rules-trajectory form; its last
    step and the records checked), and the same form as a TK-step trajectory with
    every step's observations in their own slice (each step checked)."""
    B, seed, settle, warm, K, TK = 1 << 20, 1, 256, 5, 20, 10
    # the bench's accumulators: the packed int16 word at K = 20 (bench.payload_width)
    env = BatchedCoupEnv(B, seed=seed, env_id_base=0, auto_reset=True, obs=True,
                         episode_stats=bench.episode_stats_mode(bench.payload_width(2, K, B)))
    assert env.episode_word_bytes == 2
    total = settle + warm + 3 * K + TK
    refs = {k: oracle.rollout(seed=seed, n=256, steps=total, env_id_base=k, auto_reset=True, want_obs=True)
            for k in _slices(B)}
    env.rollout(settle)
    for _ in range(warm):
        env.step()
    env.clear_episode_stats()
    t = settle + warm
    for _ in range(K):  # eager launches
        o = env.step()
        for k, ref in refs.items():
            _check_step(o, ref, t, k, "obs")
        t += 1
    _check_records(env, B, seed, t, stats_from=settle + warm)
    g1 = env.capture_steps(1)  # graph replays, one step each
    o = {"actions": env.actions, "rewards": env.rewards, "step_type": env.step_type, "legal_mask": env.legal_mask,
         "obs": env.obs}
    for _ in range(K):
        g1.replay()
        torch.cuda.synchronize()
        for k, ref in refs.items():
            _check_step(o, ref, t, k, "obs")
        t += 1
    gK = env.capture_steps(K)  # bench.py's timed region: K steps, one replay
    gK.replay()
    torch.cuda.synchronize()
    t += K
    for k, ref in refs.items():
        _check_step(o, ref, t - 1, k, "obs")
    _check_records(env, B, seed, t, stats_from=settle + warm)
    # the rules-trajectory form with a slice per step (coup_step_trajectory):
    # every step's tensors, not only the last (the packed word has taken 60
    # steps of replays its reserve count did not see: fold it first)
    env.fold_episode_stats()
    buf = env.collect_trajectory(TK)
    torch.cuda.synchronize()
    for s in range(TK):
        o_s = {name: buf[name][s] for name in ("actions", "rewards", "step_type", "legal_mask", "obs")}
        for k, ref in refs.items():
            _check_step(o_s, ref, t, k, "obs")
        t += 1
    last_cur = buf["current_player"][TK - 1].clone()
    del buf
    _check_records(env, B, seed, t, stats_from=settle + warm, cur_player=last_cur)
    assert t == total
    assert env.error_count() == 0


def test_c3i_info_state_kernel_full_batch_slices_match_oracle():
    """bench.py --config c3i at its size: 2^18 lanes with history and the
    InformationStateTensor of both players, warm-up 5 then K = 20 eager
    coup_step launches; every step's tensors of the three slices, then the
    records, history bytes and accumulators."""
    B, seed, warm, K = 1 << 18, 1, 5, 20
    env = BatchedCoupEnv(B, seed=seed, env_id_base=0, auto_reset=True, obs=False, info_state=True,
                         episode_stats=bench.episode_stats_mode(bench.payload_width(2, K, B)))
    total = warm + K
    for _ in range(warm):
        env.step()
    env.clear_episode_stats()
    # the slices' info rows of every step on the host (3 x 25 x 256 x 19,936 B)
    refs = {k: oracle.rollout(seed=seed, n=256, steps=total, env_id_base=k, auto_reset=True, want_info=True)
            for k in _slices(B)}
    for t in range(warm, total):
        o = env.step()
        for k, ref in refs.items():
            _check_step(o, ref, t, k, "info")
    _check_records(env, B, seed, total, stats_from=warm)
    assert env.error_count() == 0


def test_c4_eager_step_full_batch_slices_match_oracle():
    """c4's batch with EAGER per-step launches: 6
    players, 2^20 lanes, settle 256 through the regrouped fused rollout, 5
    warm-up and 20 eager coup_step launches of np::k_step_sorted<6, true,
    true, 1024> (the decision drawn ahead, resets dealt by 4-thread groups)
    -- bench.py's c4 warm-up form; its timed steps are ONE coup_step_many
    launch of np::k_trajectory_sorted<6, 1024>, checked on every lane by
    tests/test_gpu_every_lane.py.  At every step the actions, rewards, step
    types, legal masks and current players of three 256-lane slices against
    the written N-player spec (oracle/coup_nplayer.c, parity unpinned w.r.t.
    the 2-player reference: coup.h:42); then the full records and the
    per-episode accumulators."""
    B, seed, settle, warm, K, P = 1 << 20, 1, 256, 5, 20, 6
    env = BatchedCoupEnv(B, seed=seed, env_id_base=0, auto_reset=True, obs=False, num_players=P,
                         episode_stats=bench.episode_stats_mode(bench.payload_width(P, K, B)))
    total = settle + warm + K
    refs = {k: oracle.np_rollout(P, seed=seed, n=256, steps=total, env_id_base=k) for k in _slices(B)}
    env.rollout(settle)
    for _ in range(warm):
        env.step()
    env.clear_episode_stats()
    for t in range(settle + warm, total):
        o = env.step()
        for k, ref in refs.items():
            sl, msg = slice(k, k + 256), f"slice {k} step {t}"
            np.testing.assert_array_equal(_np(o["actions"][sl]), ref["actions"][t], err_msg=msg)
            np.testing.assert_array_equal(_np(o["rewards"][sl]), ref["rewards"][t], err_msg=msg)
            np.testing.assert_array_equal(_np(o["step_type"][sl]), ref["step_type"][t], err_msg=msg)
            np.testing.assert_array_equal(_np(o["legal_mask"][sl]).astype(np.uint32), ref["legal"][t], err_msg=msg)
            np.testing.assert_array_equal(_np(o["current_player"][sl]), ref["cur_player"][t], err_msg=msg)
    words = _np(env.export_state()).astype(np.uint32)
    eps, ret = env.episode_stats()
    for k, ref in refs.items():
        np.testing.assert_array_equal(words[k:k + 256], ref["final_state"], err_msg=f"records, slice {k}")
        pre = oracle.np_rollout(P, seed=seed, n=256, steps=settle + warm, env_id_base=k)
        np.testing.assert_array_equal(_np(eps[k:k + 256]), ref["lane_episodes"] - pre["lane_episodes"],
                                      err_msg=f"episodes, slice {k}")
        np.testing.assert_array_equal(_np(ret[k:k + 256]), ref["lane_return_sum"] - pre["lane_return_sum"],
                                      err_msg=f"return sums, slice {k}")
    assert int(eps.sum()) > 0
    assert env.error_count() == 0
