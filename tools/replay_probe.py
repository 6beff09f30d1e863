"""Why the bench's timed c3 replay runs slower than the same graph in
tools/pipe_ab.py: bench.py's sequence (settle rollout, W eager warm-up
steps, capture K steps) then replays of the K-step graph timed one by one
-- back to back, and after an idle gap -- so the first (timed) replay can be
compared with later ones on the same env.  Measurement tool only.

    python tools/replay_probe.py [--batch B] [--steps K] [--replays R] [--idle-ms MS]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--replays", type=int, default=6)
    ap.add_argument("--idle-ms", type=float, default=20.0)
    ap.add_argument("--settle", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    import torch

    import bench
    from open_spiel_coup_amd import BatchedCoupEnv
    env = BatchedCoupEnv(a.batch, seed=1, auto_reset=True, obs=True, device="cuda:0",
                         episode_stats=bench.episode_stats_mode(bench.payload_width(2, a.steps, a.batch)))
    stream = torch.cuda.current_stream()
    env.rollout(a.settle)
    for _ in range(a.warmup):
        env.step()
    env.clear_episode_stats()
    g = env.capture_steps(a.steps)
    torch.cuda.synchronize()
    for mode in ("first+back_to_back", "idle_gap"):
        for r in range(a.replays):
            if mode == "idle_gap":
                time.sleep(a.idle_ms * 1e-3)
            env.clear_episode_stats()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            g.replay()
            e1.record(stream)
            if mode == "idle_gap":
                e1.synchronize()
            ev = (e0, e1)
            if mode != "idle_gap":
                torch.cuda.synchronize()
            print(json.dumps({"mode": mode, "replay": r, "us_per_step": round(ev[0].elapsed_time(ev[1]) * 1e3 / a.steps, 2)}),
                  flush=True)
    assert env.error_count() == 0


if __name__ == "__main__":
    main()
