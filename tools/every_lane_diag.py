"""Diagnostic (measurement tool): where the c3 graph form's every-lane check
first differs from the oracle.  Prints one JSON line per probe: mismatching
lanes of the records / actions after settle + warm-up, after K eager
coup_step_many steps, after a graph replay (captured first thing, as
bench.py does), and after a graph replay captured behind a 1-step capture."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from oracle import oracle  # noqa: E402
from open_spiel_coup_amd import BatchedCoupEnv  # noqa: E402

B, seed, settle, warm, K = 1 << 20, 1, 256, 5, 20
t0 = settle + warm
ref = oracle.window(2, seed, B, t0 + 2 * K, t0, snaps=(t0, t0 + K, t0 + 2 * K))


def env_at_t0():
    env = BatchedCoupEnv(B, seed=seed, obs=True, episode_stats=2)
    env.rollout(settle)
    for _ in range(warm):
        env.step()
    env.clear_episode_stats()
    return env


def probe(name, env, t, acts_row=None):
    rec = env.export_state().cpu().numpy().astype(np.uint32)
    bad = int((rec != ref["snap_state"][t]).any(1).sum())
    out = {"probe": name, "step": t, "record_lanes_wrong": bad}
    if acts_row is not None:
        out["action_lanes_wrong"] = int((env.actions.cpu().numpy() != ref["actions"][acts_row]).sum())
    print(json.dumps(out), flush=True)


e = env_at_t0()
probe("after settle + warm-up", e, t0)
e.step_many(K)
torch.cuda.synchronize()
probe("eager coup_step_many(K)", e, t0 + K, K - 1)
del e
e = env_at_t0()
g = e.capture_steps(K)
probe("after capture, before replay", e, t0)
g.replay()
torch.cuda.synchronize()
probe("graph replay (first capture)", e, t0 + K, K - 1)
e.fold_episode_stats()
g.replay()
torch.cuda.synchronize()
probe("graph replay 2", e, t0 + 2 * K, 2 * K - 1)
del g, e
e = env_at_t0()
g1 = e.capture_steps(1)
del g1
g = e.capture_steps(K)
g.replay()
torch.cuda.synchronize()
probe("graph replay behind a 1-step capture", e, t0 + K, K - 1)
