"""Does the Infinity Cache absorb part of a split writer's stores when the
same tensor buffer is rewritten every step?  (Measurement tool; DESIGN.md
section 5)

    python tools/mall_probe.py [--batch B] [--steps K] [--rounds R] [--info]

The c3 split step (the rules step, then k_obs_sweep_rows writing
[B][2][98] fp32) runs K eager steps into ONE observation buffer, and K steps
alternating between TWO buffers of the same size, interleaved over R rounds
(--info: c3i's InformationStateTensor step, 2^18 lanes).  The rules and the
writer are the same kernels in both; only the buffer a step rewrites
differs.  With one buffer the 256 MB Infinity Cache may still hold the dirty
tail of the previous step's stores when the next step rewrites it, and then
those lines never reach HBM; alternating two buffers of 822 MB (or 5.2 GB)
removes that reuse.  Prints the median us per step of both forms.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--info", action="store_true")
    a = ap.parse_args()
    import torch

    from open_spiel_coup_amd import BatchedCoupEnv
    B = a.batch or ((1 << 18) if a.info else (1 << 20))
    name = "info_state" if a.info else "obs"
    env = (BatchedCoupEnv(B, seed=1, obs=False, info_state=True, history=True, device="cuda:0") if a.info else
           BatchedCoupEnv(B, seed=1, obs=True, device="cuda:0"))
    bufs = [getattr(env, name), torch.empty_like(getattr(env, name))]
    stream = torch.cuda.current_stream()
    for _ in range(10):  # warm: both buffers touched, clocks up
        for b in bufs:
            env.set_output(name, b)
            env.step()
    torch.cuda.synchronize()

    def run(alternate):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        env.set_output(name, bufs[0])
        env.step()  # the form's first buffer written once before the window
        ev[0].record(stream)
        for k in range(a.steps):
            env.set_output(name, bufs[k & 1] if alternate else bufs[0])
            env.step()
        ev[1].record(stream)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) * 1e3 / a.steps

    res = {"one buffer": [], "two buffers": []}
    for _ in range(a.rounds):
        res["one buffer"].append(run(False))
        res["two buffers"].append(run(True))
    out = {"form": "c3i info-state split step" if a.info else "c3 obs split step", "batch": B, "steps": a.steps,
           "rounds": a.rounds, "buffer_mb": round(bufs[0].numel() * 4 / 2 ** 20, 1)}
    out.update({k: {"median_us": round(statistics.median(v), 2), "min_us": round(min(v), 2)} for k, v in res.items()})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
