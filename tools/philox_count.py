"""Philox evaluations per wave and step (measurement build only).

    python -m open_spiel_coup_amd.build --out ab/count.so --define COUP_COUNT_PHILOX
    COUP_LIB_PATH=ab/count.so python tools/philox_count.py [--players N] [--batch B]

Each wave-level evaluation of philox4x32_10 (one pass of the wave through
it, whatever its active lanes) is counted with the lanes active in it.
Prints evaluations per wave per env step and the mean active lanes, for the
step kernel, the fused rollout, coup_step_many without tensors (one
trajectory launch) and (2 players) coup_step_many's c3 form --
the rules trajectory with every step's records, from 2^20 lanes with
observations (its writers draw nothing).  Measurement tool only.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--players", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch

    from open_spiel_coup_amd import BatchedCoupEnv
    from open_spiel_coup_amd import _native
    lib = _native.load()
    fn = getattr(lib, "coup_debug_philox_counts" + ("_np" if a.players != 2 else ""), None)
    if fn is None:
        raise SystemExit("not a COUP_COUNT_PHILOX build (set COUP_LIB_PATH)")
    buf = (ctypes.c_ulonglong * 2)()
    env = BatchedCoupEnv(a.batch, seed=1, auto_reset=True, obs=False, device="cuda:0", num_players=a.players)
    env.rollout(256)
    waves = (a.batch + 63) // 64
    out = {"players": a.players, "batch": a.batch}
    for kind in ("step", "rollout"):
        torch.cuda.synchronize()
        fn(buf, 1)
        if kind == "step":
            for _ in range(a.steps):
                env.step()
        else:
            env.rollout(a.steps)
        torch.cuda.synchronize()
        fn(buf, 1)
        evals, lanes = buf[0], buf[1]
        out[kind] = {"evals_per_wave_step": round(evals / (waves * a.steps), 3),
                     "active_lanes_per_eval": round(lanes / max(evals, 1), 1)}
    # coup_step_many without tensors: one trajectory launch (c2 / c4's form)
    torch.cuda.synchronize()
    fn(buf, 1)
    env.step_many(a.steps)
    torch.cuda.synchronize()
    fn(buf, 1)
    evals, lanes = buf[0], buf[1]
    out["step_many"] = {"evals_per_wave_step": round(evals / (waves * a.steps), 3),
                        "active_lanes_per_eval": round(lanes / max(evals, 1), 1)}
    if a.players == 2:
        envo = BatchedCoupEnv(a.batch, seed=1, auto_reset=True, obs=True, device="cuda:0")
        envo.rollout(256)
        torch.cuda.synchronize()
        fn(buf, 1)
        envo.step_many(a.steps)
        torch.cuda.synchronize()
        fn(buf, 1)
        evals, lanes = buf[0], buf[1]
        out["step_many_obs"] = {"evals_per_wave_step": round(evals / (waves * a.steps), 3),
                                "active_lanes_per_eval": round(lanes / max(evals, 1), 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
