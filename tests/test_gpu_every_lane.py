"""Every lane, every checked step: the bench's exact forms at the bench's
sizes against the oracle.

bench.py's lines run these forms (the driver's command is `bench.py --gpus 1
--steps 20 --warmup 5`):
  c3   2^20 lanes, ObservationTensor x2: settle 256 through the fused
       rollout, 5 eager warm-up steps, then K = 20 steps replayed from one
       HIP graph of coup_step_many -- the rules-trajectory form
       (k_trajectory_sorted<1024, true, false, 8, 0, true>, balanced chunks of up to 10 steps,
       then k_obs_sweep_rows<512, 2> once per step);
  c2   65,536 lanes, no tensors: the same settle and warm-up, then the K = 20
       steps as ONE coup_step_many launch (k_step_trajectory, outputs stored
       with stride 0) replayed from a graph;
  c4   6 players, 2^20 lanes: the same with np::k_trajectory_sorted<6, 1024>;
  c3i  2^18 lanes with the InformationStateTensor x2: 5 warm-up and K = 20
       eager split steps (the history-keeping rules step, k_info_sweep<1024, 2>).
Each test records the library's launch log (coup_launch_log) of the calls it
makes and asserts it equals bench.expected_kernel -- what the bench line
reports as roofline.kernel -- so the test runs the kernels the line names.

The graph replays leave only the last step's outputs, so each replay's last
step is checked (and replayed more than once, as the bench's power warm-up
does); then the same kernels run as a trajectory with every step's outputs
in its own [T][B] slice (coup_step_trajectory: the c3 rules-trajectory form
writing each step's observations to its slice; c2 / c4 the same trajectory
kernel with a non-zero output stride), and every step is checked.

Checked on EVERY lane: actions, rewards, step types, legal masks, current
players, the observation / information-state rows (two 64-bit linear hashes
per lane and step, computed on the GPU by tests/lane_digest.py and by the
oracle's window driver on the host: any single wrong float changes both),
the full 16-byte records (32-byte for 6 players) and the per-lane episode
counts and player-0 return sums.  The oracle runs over env-id chunks on all
of the job's host threads (oracle.window).  Reference semantics: coup.cc:248-287
(ObservationTensor), :230-245 (InformationStateTensor), :522-808 (the
transition), :824-938 (LegalActions); rl_environment.py:243-248."""
import numpy as np
import pytest
import torch

import bench
from oracle import oracle
from open_spiel_coup_amd import BatchedCoupEnv, _native
from tests.lane_digest import assert_lanes_equal, tensor_hash

pytestmark = pytest.mark.gpu


def _np(t):
    return t.detach().cpu().numpy()


def _check_outputs(o, ref, r, msg, tensor=None):
    """Outputs `o` (a dict of [B, ...] device tensors) against row r of the
    oracle window `ref`."""
    assert_lanes_equal(_np(o["actions"]), ref["actions"][r], f"{msg}: actions")
    assert_lanes_equal(_np(o["rewards"]), ref["rewards"][r], f"{msg}: rewards")
    assert_lanes_equal(_np(o["step_type"]), ref["step_type"][r], f"{msg}: step types")
    assert_lanes_equal(_np(o["legal_mask"]).astype(np.uint32), ref["legal"][r], f"{msg}: legal masks")
    assert_lanes_equal(_np(o["current_player"]), ref["cur_player"][r], f"{msg}: current players")
    if tensor == "obs":
        assert_lanes_equal(tensor_hash(o["obs"]), ref["obs_hash"][r], f"{msg}: ObservationTensor rows")
    elif tensor == "info":
        assert_lanes_equal(tensor_hash(o["info_state"]), ref["info_hash"][r], f"{msg}: InformationStateTensor rows")


def _check_snapshot(env, ref, t, msg):
    assert_lanes_equal(_np(env.export_state()).astype(np.uint32), ref["snap_state"][t], f"{msg}: records")
    eps, ret = env.episode_stats()
    assert_lanes_equal(_np(eps), ref["snap_eps"][t], f"{msg}: episode counts")
    assert_lanes_equal(_np(ret), ref["snap_ret"][t], f"{msg}: return sums")


def _env_outputs(env):
    o = {"actions": env.actions, "rewards": env.rewards, "step_type": env.step_type,
         "legal_mask": env.legal_mask, "current_player": env.cur_player}
    if env.obs is not None:
        o["obs"] = env.obs
    return o


def _graph_then_trajectory(cfg, players, tensor):
    """The c2 / c3 / c4 flow: settle, warm-up, two replays of the bench's
    K-step graph (each replay's last step, records and accumulators on every
    lane), then the same kernels as a K-step trajectory (every step)."""
    B0, with_obs, _, _, _, _, P = bench.CONFIGS[cfg]
    assert P == players
    B, seed, settle, warm, K, replays = B0, 1, 256, 5, 20, 2
    t0 = settle + warm
    total = t0 + (replays + 1) * K
    snaps = tuple(t0 + (r + 1) * K for r in range(replays)) + (total,)
    ref = oracle.window(players, seed, B, total, t0, obs_hash=tensor == "obs", snaps=snaps, stats_from=t0)
    env = BatchedCoupEnv(B, seed=seed, env_id_base=0, auto_reset=True, obs=with_obs, num_players=players,
                         episode_stats=bench.episode_stats_mode(bench.payload_width(players, K, B)))
    env.rollout(settle)
    for _ in range(warm):
        env.step()
    env.clear_episode_stats()
    want = bench.expected_kernel(cfg, B, True)
    _native.launch_log()
    g = env.capture_steps(K)
    assert _native.launch_log() == want
    o = _env_outputs(env)
    for r in range(replays):
        if r:
            env.fold_episode_stats()  # the packed word holds one replay's K steps
        g.replay()
        torch.cuda.synchronize()
        t = t0 + (r + 1) * K
        _check_outputs(o, ref, t - 1 - t0, f"{cfg} replay {r} (step {t - 1})", tensor)
        _check_snapshot(env, ref, t, f"{cfg} after replay {r}")
    del g
    env.fold_episode_stats()
    _native.launch_log()
    buf = env.collect_trajectory(K)
    torch.cuda.synchronize()
    assert _native.launch_log() == want
    for s in range(K):
        r = replays * K + s
        o_s = {k: buf[k][s] for k in buf}
        _check_outputs(o_s, ref, r, f"{cfg} trajectory step {t0 + r}", tensor)
    _check_snapshot(env, ref, total, f"{cfg} after the trajectory")
    assert env.error_count() == 0
    # the accumulators saw episodes end
    assert int(ref["snap_eps"][total].sum()) > 0


def test_c3_every_lane_matches_oracle():
    """c3 (the headline): 2^20 lanes, every lane, 60 checked steps."""
    _graph_then_trajectory("c3", 2, "obs")


def test_c2_every_lane_matches_oracle():
    """c2: 65,536 lanes, ONE k_step_trajectory launch per K steps."""
    _graph_then_trajectory("c2", 2, None)


def test_c4_every_lane_matches_oracle():
    """c4: 6 players, 2^20 lanes, np::k_trajectory_sorted<6, 1024> (parity
    against the written N-player spec, oracle/coup_nplayer.c: unpinned
    w.r.t. the 2-player reference, coup.h:42)."""
    _graph_then_trajectory("c4", 6, None)


def test_c3i_every_lane_matches_oracle():
    """c3i: 2^18 lanes with history, 5 warm-up then K = 20 eager split
    steps (bench.py's c3i form), every step's InformationStateTensor rows
    hashed on every lane."""
    B, seed, warm, K = bench.CONFIGS["c3i"][0], 1, 5, 20
    total = warm + K
    ref = oracle.window(2, seed, B, total, warm, info_hash=True, snaps=(total,), stats_from=warm)
    env = BatchedCoupEnv(B, seed=seed, env_id_base=0, auto_reset=True, obs=False, info_state=True,
                         episode_stats=bench.episode_stats_mode(bench.payload_width(2, K, B)))
    for _ in range(warm):
        env.step()
    env.clear_episode_stats()
    want = bench.expected_kernel("c3i", B, False)
    for r in range(K):
        _native.launch_log()
        o = env.step()
        assert _native.launch_log() == want
        _check_outputs(o, ref, r, f"c3i step {warm + r}", "info")
    _check_snapshot(env, ref, total, "c3i")
    assert env.error_count() == 0
