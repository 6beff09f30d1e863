"""Same-process A/B of the fused trajectory launch (coup_step_trajectory)
against itself with no output buffers bound, against its round-2 store form
(outputs stored where each lane is played instead of staged by lane in LDS,
COUP_TRAJ_STAGE=0) and against the fused rollout (statistics only; also with
its round-2 bin prefix, COUP_NP_SCAN=0): the cost of storing every step's
outputs.  Measurement tool only.

    python tools/traj_ab.py [--players 6] [--batch 2^20] [--steps 50] [--rounds 7]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--players", type=int, default=6)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    import torch
    from open_spiel_coup_amd import BatchedCoupEnv, _native
    env = BatchedCoupEnv(a.batch, seed=1, auto_reset=True, obs=False, num_players=a.players, episode_stats=True)
    env.rollout(256)
    buf = env.trajectory_buffers(a.steps)
    full = env.step_trajectory_launcher(a.steps, buf)
    none_out = _native.StepOutputs(None, None, None, None, None, None, None, None, None)

    def bare():
        _native.check(env.lib.coup_step_trajectory(env._h, a.steps, ctypes.byref(none_out)))
    stats = env.new_stats()
    roll = env.rollout_launcher(a.steps, stats)
    def knob(var, val, fn):  # another form of the regrouped kernel, chosen at launch
        def launch():
            os.environ[var] = val
            try:
                fn()
            finally:
                os.environ.pop(var, None)
        return launch
    variants = {"trajectory": full, "trajectory_unstaged": knob("COUP_TRAJ_STAGE", "0", full),
                "trajectory_no_outputs": bare,
                "rollout_stats": roll, "rollout_lane_scan": knob("COUP_NP_SCAN", "0", roll)}
    times = {k: [] for k in variants}
    s = torch.cuda.current_stream()
    for _ in range(a.rounds):
        for k, fn in variants.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            env.rollout(8)  # keeps the GPU busy while the timed launch is enqueued
            e0.record(s)
            fn()
            e1.record(s)
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3 / a.steps)
    for k, v in times.items():
        print(json.dumps({"variant": k, "players": a.players, "batch": a.batch, "steps": a.steps,
                          "median_us_per_step": round(statistics.median(v), 2), "min_us_per_step": round(min(v), 2)}))


if __name__ == "__main__":
    main()
