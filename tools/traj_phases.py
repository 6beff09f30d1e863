"""Where the 2-player rules trajectory's waves spend a step (measurement
build only).

    python -m open_spiel_coup_amd.build --out build/libab/phases.so --define COUP_TRAJ_PHASES
    COUP_LIB_PATH=build/libab/phases.so python tools/traj_phases.py [--batch B] [--steps K]

k_trajectory_sorted stamps the shader clock (s_memtime) at fixed points of
every step; coup_debug_traj_phases returns the cycles each phase took,
summed over waves, and the wave-steps (--players 6: np::k_trajectory_sorted,
coup_debug_np_traj_phases).  Prints, per form (c3's rules trajectory with
records; the bare trajectory of tensor-free steps), the
cycles per wave-step of each phase and its share.  The stamps cost a few
dozen cycles each, so the totals run above the product kernel's.
Measurement tool only.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ("count atomic + count barrier", "prefix + slot writes", "slot barrier",
          "slot read, unpack, FIRST / reset / rejected paths", "decision + deals",
          "outputs, legal mask, next draw")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--players", type=int, default=2, help="6: np::k_trajectory_sorted (c4's form)")
    a = ap.parse_args()
    import torch

    from open_spiel_coup_amd import BatchedCoupEnv, _native
    lib = _native.load()
    fn = getattr(lib, "coup_debug_traj_phases" if a.players == 2 else "coup_debug_np_traj_phases", None)
    if fn is None:
        raise SystemExit("not a COUP_TRAJ_PHASES build (set COUP_LIB_PATH)")
    buf = (ctypes.c_ulonglong * (len(PHASES) + 1))()
    forms = ((("c3 rules trajectory (records)", True), ("bare trajectory", False)) if a.players == 2 else
             (("bare trajectory (%d players)" % a.players, False),))
    for form, obs in forms:
        env = BatchedCoupEnv(a.batch, seed=1, auto_reset=True, obs=obs, device="cuda:0", num_players=a.players)
        env.rollout(256)
        env.step_many(a.steps)  # warm
        torch.cuda.synchronize()
        fn(buf, 1)
        env.step_many(a.steps)
        torch.cuda.synchronize()
        fn(buf, 1)
        ws = max(buf[len(PHASES)], 1)
        cyc = [buf[k] / ws for k in range(len(PHASES))]
        tot = sum(cyc)
        print(json.dumps({"form": form, "batch": a.batch, "steps": a.steps, "wave_steps": ws,
                          "cycles_per_wave_step": round(tot, 1),
                          "phases": {p: {"cycles": round(c, 1), "share": round(c / tot, 3)} for p, c in zip(PHASES, cyc)}}),
              flush=True)
        env.close()


if __name__ == "__main__":
    main()
