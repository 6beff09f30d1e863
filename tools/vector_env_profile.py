"""Where a SyncVectorEnv step's time goes at 8 / 64 / 256 envs
(INFORMATION_STATE, the reference's default observation type): cProfile of
the batched step(reset_if_done=True) loop, plus the step's phases timed
alone (the launch + copy-out of coup_step_host, the per-env time steps).
Measurement tool only.

    python tools/vector_env_profile.py [--steps 40] [--top 25]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Out:
    def __init__(self, a):
        self.action = a


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--obs", type=int, default=0, help="1: OBSERVATION instead of INFORMATION_STATE")
    a = ap.parse_args()
    from open_spiel_coup_amd import rl_environment, vector_env
    otype = rl_environment.ObservationType.OBSERVATION if a.obs else rl_environment.ObservationType.INFORMATION_STATE
    rng = random.Random(1)
    result = {}
    for k in (8, 64, 256):
        envs = [rl_environment.Environment("coup", seed=k, observation_type=otype) for _ in range(k)]
        venv = vector_env.SyncVectorEnv(envs)
        ts = venv.reset()

        def run(m, ts):
            for _ in range(m):
                outs = [_Out(rng.choice(t.observations["legal_actions"][t.current_player()])) for t in ts]
                ts, _, _, _ = venv.step(outs, reset_if_done=True)
            return ts
        ts = run(3, ts)
        t0 = time.perf_counter()
        ts = run(a.steps, ts)
        us = 1e6 * (time.perf_counter() - t0) / (a.steps * k)
        # phases alone: the host step (launch, sync, copy-out) and the time steps
        sh = venv._shared
        acts = [-1] * k
        t1 = time.perf_counter()
        for _ in range(a.steps):
            q = sh.step_host(acts, obs=bool(a.obs), info_state=not a.obs)
        host_us = 1e6 * (time.perf_counter() - t1) / (a.steps * k)
        t2 = time.perf_counter()
        for _ in range(a.steps):
            venv._time_steps(q, [False] * k)
        ts_us = 1e6 * (time.perf_counter() - t2) / (a.steps * k)
        pr = cProfile.Profile()
        pr.enable()
        ts = run(a.steps, ts)
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(a.top)
        result[k] = {"us_per_env_step": round(us, 2), "step_host_us_per_env": round(host_us, 2),
                     "time_steps_us_per_env": round(ts_us, 2)}
        print(f"=== {k} envs: {json.dumps(result[k])}")
        print(s.getvalue())
    print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
