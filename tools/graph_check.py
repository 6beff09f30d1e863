"""Eager vs HIP-graph replay of the c3 step at full size, in one process:
per-step time of each (alternating), and the final records and obs of K
graph steps against K eager steps from the same starting records
(measurement tool).

    python tools/graph_check.py [--steps 20] [--rounds 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch

    from open_spiel_coup_amd import BatchedCoupEnv
    env = BatchedCoupEnv(a.batch, seed=1, auto_reset=True, obs=True, device="cuda:0")
    env.rollout(256)
    g = env.capture_steps(a.steps)
    stream = torch.cuda.current_stream()

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.steps

    def eager():
        for _ in range(a.steps):
            env.step()

    for r in range(a.rounds):
        start = env.export_state().clone()
        te = timed(eager)
        after_eager = env.export_state().clone()
        obs_eager = env.obs.clone()
        env.import_state(start)
        tg = timed(g.replay)
        after_graph = env.export_state().clone()
        same = bool(torch.equal(after_eager, after_graph)) and bool(torch.equal(obs_eager, env.obs))
        print(json.dumps({"round": r, "eager_us": round(te, 1), "graph_us": round(tg, 1), "identical": same}),
              flush=True)


if __name__ == "__main__":
    main()
