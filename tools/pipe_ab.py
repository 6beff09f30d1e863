"""Same-process A/B of the c3 step forms in the driver's own form (a HIP
graph of K uniform steps, the packed int16 episode word, 2^20 lanes after
the settle), variants interleaved round-robin.

    python tools/pipe_ab.py [--batch B] [--steps K] [--rounds R] NAME:VAR=VAL[,...] ...

Each positional argument is one env created with those environment settings
(knobs read at coup_create, e.g. COUP_PIPE, COUP_TRAJ_CHUNK, COUP_PIPE_SPAN)
and captured with BatchedCoupEnv.capture_steps(K).  Default variants: the
serial split step (COUP_PIPE=0), the rules-trajectory form (COUP_PIPE=1)
at chunks of 8 / 4 steps, and with the measurement build
(COUP_LIB_PATH=build/variants/libcoup_mi355x.so) the merged pipelined step
(COUP_PIPE=2) and the rules trajectories on a second stream beside the
writers (COUP_PIPE=3; the CU-masked form was deleted in round 6).  --eager:
time eager coup_step_many calls instead of graph replays.  Prints one JSON line per variant:
median / min us per env step.  Measurement tool only.
"""
import argparse
import json
import os
import statistics
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT = ["serial:COUP_PIPE=0", "traj8:COUP_PIPE=1", "traj10:COUP_TRAJ_CHUNK=10"]
AB_ONLY = ["t512w8:COUP_MANY_SHAPE=1", "t512w6:COUP_MANY_SHAPE=2", "t256w8:COUP_MANY_SHAPE=3",
           "t1024w4:COUP_MANY_SHAPE=4", "traj8s:COUP_MANY_STAGE=1", "fused:COUP_PIPE=4", "fused512w4:COUP_PIPE=4,COUP_FUSED_SHAPE=1", "fused1024w8:COUP_PIPE=4,COUP_FUSED_SHAPE=2",
           "fused512w8:COUP_PIPE=4,COUP_FUSED_SHAPE=3", "pipe85:COUP_PIPE=2,COUP_PIPE_SPAN=0.85",
           "over4:COUP_PIPE=3,COUP_TRAJ_CHUNK=4"]
KNOBS = ("COUP_PIPE", "COUP_PIPE_SPAN", "COUP_TRAJ_CHUNK", "COUP_MANY_STAGE", "COUP_MANY_SHAPE", "COUP_WRITER_POL",
         "COUP_WRITER_PRIO", "COUP_OVERLAP_LDS", "COUP_FUSED_SHAPE", "COUP_OBS_SPLIT", "COUP_OBS_MODE", "COUP_WRITER_FORM",
         "COUP_WRITER_DYN_LDS")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--settle", type=int, default=256)
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    import torch

    import bench
    from open_spiel_coup_amd import BatchedCoupEnv, _native
    ab = bool(_native.load().coup_build_flags() & _native.BUILD_AB_VARIANTS)
    variants = a.variants or (DEFAULT + (AB_ONLY if ab else []))
    envs, graphs = {}, {}
    for v in variants:
        name, _, kvs = v.partition(":")
        for k in KNOBS:
            os.environ.pop(k, None)
        for kv in kvs.split(","):
            if kv:
                k, val = kv.split("=")
                os.environ[k] = val
        env = BatchedCoupEnv(a.batch, seed=1, auto_reset=True, obs=True, device="cuda:0",
                             episode_stats=bench.episode_stats_mode(bench.payload_width(2, a.steps, a.batch)))
        env.rollout(a.settle)
        for _ in range(5):
            env.step()
        env.clear_episode_stats()
        if a.eager:
            graphs[name] = types.SimpleNamespace(replay=lambda e=env: e.step_many(a.steps))
        else:
            graphs[name] = env.capture_steps(a.steps)
        envs[name] = env
    for k in KNOBS:
        os.environ.pop(k, None)
    stream = torch.cuda.current_stream()
    times = {n: [] for n in graphs}
    for _ in range(a.rounds):
        for name, g in graphs.items():
            envs[name].clear_episode_stats()
            g.replay()  # warm
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            envs[name].clear_episode_stats()
            e0.record(stream)
            g.replay()
            e1.record(stream)
            e1.synchronize()
            times[name].append(e0.elapsed_time(e1) * 1e3 / a.steps)
    for name, env in envs.items():
        assert env.error_count() == 0, name
    bytes_step = 824 * a.batch
    for name, t in times.items():
        med = statistics.median(t)
        print(json.dumps({"variant": name, "median_us": round(med, 2), "min_us": round(min(t), 2),
                          "frac_of_spec": round(bytes_step / (med * 1e-6) / 8e12, 4),
                          "all_us": [round(x, 2) for x in t]}), flush=True)


if __name__ == "__main__":
    main()
