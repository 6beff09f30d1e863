"""Interleaved A/B timing of step-kernel variants in ONE process (box-to-box
HBM variance is larger than the differences being measured).

    python tools/ab_step.py [--batch B] [--obs 0|1] [--info 0|1] [--players N] [--rounds R] [--steps K] VAR=VAL[,...] ...

Each positional argument is one variant: a comma-separated list of
environment settings read by coup_step at launch (COUP_OBS_MODE,
COUP_XCD_REMAP, COUP_STEP_DYN_LDS).  The variants run
round-robin `rounds` times over the same settled batch; prints one JSON line
per variant with the median and min per-step kernel time (HIP events on the
launch stream).  Measurement tool only.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KNOBS = ("COUP_OBS_MODE", "COUP_XCD_REMAP", "COUP_STEP_DYN_LDS", "COUP_REGROUP", "COUP_AHEAD")


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

    from open_spiel_coup_amd import BatchedCoupEnv
    env = BatchedCoupEnv(a.batch, seed=1, auto_reset=True, obs=bool(a.obs) and not a.info, info_state=bool(a.info),
                         device="cuda:0", num_players=a.players)
    if a.info:
        for _ in range(32):  # histories: no fused rollout
            env.step()
    else:
        env.rollout(256)
    stream = torch.cuda.current_stream()
    times = {v: [] for v in a.variants}
    for _ in range(a.rounds):
        for v in a.variants:
            for k in KNOBS:
                os.environ.pop(k, None)
            for kv in v.split(","):
                if kv:
                    k, val = kv.split("=")
                    os.environ[k] = val
            if a.fused:
                env.rollout(a.fused)
            else:
                for _ in range(3):
                    env.step()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            if a.fused:
                env.rollout(a.fused * a.steps)
            else:
                for _ in range(a.steps):
                    env.step()
            e1.record(stream)
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) * 1e3 / (a.steps * max(a.fused, 1)))  # us per env step
    assert env.error_count() == 0
    for v in a.variants:
        t = times[v]
        print(json.dumps({"variant": v, "median_us": round(statistics.median(t), 2), "min_us": round(min(t), 2),
                          "all_us": [round(x, 2) for x in t]}), flush=True)


if __name__ == "__main__":
    main()
