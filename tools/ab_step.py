"""Interleaved A/B timing of step-kernel variants in ONE process (box-to-box
HBM variance is larger than the differences being measured).

    COUP_LIB_PATH=build/variants/libcoup_mi355x.so \
    python tools/ab_step.py [--batch B] [--obs 0|1] [--info 0|1] [--players N] [--rounds R] [--steps K] VAR=VAL[,...] ...

Each positional argument is one variant: a comma-separated list of
environment settings read by coup_create (csrc/coup_knobs.h: COUP_OBS_SPLIT,
COUP_INFO_SPLIT, COUP_REGROUP, COUP_PIPE, COUP_PIPE_SPAN; with the
measurement build also COUP_OBS_MODE, COUP_XCD_REMAP, COUP_STEP_DYN_LDS,
COUP_STEP_TPL, COUP_SORT_THREADS, COUP_NP_SORT_THREADS, COUP_AHEAD,
COUP_NP_RESET_INLINE, COUP_NP_RESET_GROUP, COUP_TRAJ_STAGE, COUP_NP_SCAN),
plus STATS=0/1 (bind the per-episode accumulators, coup_step_outputs.
episodes / return_sum; default 1, as bench.py) and CEIL=1 (time
coup_measure_step_traffic -- the step's traffic with no rules -- instead of
the step).  Each variant gets its own env, created with its settings and
settled the same way (same seed: the same games); the variants then run
round-robin `rounds` times.  Prints one JSON line per variant with the
median and min per-step kernel time (HIP events on the launch stream).
Measurement tool only.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KNOBS = ("COUP_OBS_MODE", "COUP_XCD_REMAP", "COUP_STEP_DYN_LDS", "COUP_REGROUP", "COUP_AHEAD",
         "COUP_NP_SORT_THREADS", "COUP_SORT_THREADS", "COUP_NP_RESET_INLINE", "COUP_TRAJ_STAGE",
         "COUP_NP_RESET_GROUP", "COUP_STEP_TPL", "COUP_OBS_SPLIT", "COUP_INFO_SPLIT", "COUP_NP_SCAN",
         "COUP_PIPE", "COUP_PIPE_SPAN", "COUP_WRITER_POL", "COUP_TRAJ_CHUNK", "COUP_MANY_SHAPE")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--obs", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--players", type=int, default=2)
    ap.add_argument("--info", type=int, default=0, help="write the InformationStateTensor (c3i) instead")
    ap.add_argument("--fused", type=int, default=0, help="time coup_rollout launches of this many steps instead")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import torch

    import ctypes

    from open_spiel_coup_amd import BatchedCoupEnv, _native
    stream = torch.cuda.current_stream()
    envs, opts_of = {}, {}
    for v in a.variants:
        for k in KNOBS:
            os.environ.pop(k, None)
        opts = {"STATS": "1", "CEIL": "0"}
        for kv in v.split(","):
            if kv:
                k, val = kv.split("=")
                if k in opts:
                    opts[k] = val
                else:
                    os.environ[k] = val
        env = BatchedCoupEnv(a.batch, seed=1, auto_reset=True, obs=bool(a.obs) and not a.info,
                             info_state=bool(a.info), device="cuda:0", num_players=a.players, episode_stats=True)
        if opts["STATS"] != "1":
            env._out.episodes, env._out.return_sum = None, None
        if a.info:
            for _ in range(32):  # histories: no fused rollout
                env.step()
        else:
            env.rollout(256)
        envs[v], opts_of[v] = env, opts
    for k in KNOBS:
        os.environ.pop(k, None)

    def ceiling_launcher(env):
        rec = env.export_state()
        out = _native.StepOutputs(*[t.data_ptr() if t is not None else None for t in
                                    (env.actions, env.rewards, env.step_type, env.legal_mask, env.cur_player,
                                     env.obs)])

        def launch():
            _native.check(env.lib.coup_measure_step_traffic(a.batch, ctypes.c_void_p(rec.data_ptr()),
                                                             ctypes.byref(out),
                                                             ctypes.c_void_p(stream.cuda_stream)))
        launch.keep = (rec, out)
        return launch

    steppers = {v: (ceiling_launcher(envs[v]) if opts_of[v]["CEIL"] == "1" else envs[v].step) for v in a.variants}
    times = {v: [] for v in a.variants}
    for _ in range(a.rounds):
        for v in a.variants:
            env, step = envs[v], steppers[v]
            if a.fused:
                env.rollout(a.fused)
            else:
                for _ in range(3):
                    step()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            if a.fused:
                env.rollout(a.fused * a.steps)
            else:
                for _ in range(a.steps):
                    step()
            e1.record(stream)
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) * 1e3 / (a.steps * max(a.fused, 1)))  # us per env step
    for v in a.variants:
        assert envs[v].error_count() == 0, v
    for v in a.variants:
        t = times[v]
        print(json.dumps({"variant": v, "median_us": round(statistics.median(t), 2), "min_us": round(min(t), 2),
                          "all_us": [round(x, 2) for x in t]}), flush=True)


if __name__ == "__main__":
    main()
