"""Per-wave phase timeline of the 6-player regrouped step (c4; measurement
builds only).

    python -m open_spiel_coup_amd.build --out ab/trace.so --define COUP_WAVE_TRACE
    COUP_LIB_PATH=ab/trace.so python tools/np_wave_trace.py [--batch B] [--steps K]

The trace build stamps s_memrealtime (100 MHz) per wave of
np::k_step_sorted at the phase edges (coup_nplayer.hip NP_TRACE): entry (0),
record load returned (1), phase 1 done (2), after the sort barrier (3),
phase 2 (rules) done (4), after its barrier (5), auto-resets done (6), after
their barrier (7), stores issued (8), stores drained (9).  Prints the
percentiles of each phase's duration per wave and of the barrier waits, and
how many waves were resident at once.  The stamps' waits (vmcnt(0) at 1 and
9) serialise what the kernel otherwise overlaps, so the sum is a little
above the untraced step.  Measurement tool only.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = (("load", 0, 1), ("phase1", 1, 2), ("sort_barriers", 2, 3), ("rules", 3, 4), ("rules_barrier", 4, 5),
          ("resets", 5, 6), ("reset_barrier", 6, 7), ("store_issue", 7, 8), ("store_drain", 8, 9))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--players", type=int, default=6)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "np_wave_trace.json"))
    a = ap.parse_args()
    import torch

    from open_spiel_coup_amd import BatchedCoupEnv
    from open_spiel_coup_amd import _native
    lib = _native.load()
    if not hasattr(lib, "coup_debug_set_trace"):
        raise SystemExit("not a COUP_WAVE_TRACE build (set COUP_LIB_PATH)")
    lib.coup_debug_set_trace.argtypes = [ctypes.c_void_p]
    env = BatchedCoupEnv(a.batch, seed=1, auto_reset=True, obs=False, device="cuda:0", num_players=a.players,
                         episode_stats=True)
    env.rollout(256)
    for _ in range(5):
        env.step()
    waves = (a.batch + 255) // 256 * 4
    buf = torch.zeros(waves * 10, dtype=torch.int64, device="cuda:0")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    lib.coup_debug_set_trace(ctypes.c_void_p(buf.data_ptr()))
    for _ in range(a.steps):
        e0.record()
        env.step()
        e1.record()
    torch.cuda.synchronize()
    lib.coup_debug_set_trace(None)
    tr = buf.view(waves, 10).cpu().numpy().astype(np.float64)
    tr = tr[tr[:, 0] != 0]
    t = (tr - tr[:, 0].min()) / 100.0  # us
    q = lambda x: [round(float(v), 2) for v in np.percentile(x, [5, 50, 95])]  # noqa: E731
    phases = {name: q(t[:, k1] - t[:, k0]) for name, k0, k1 in PHASES}
    total = t[:, 9] - t[:, 0]
    # resident waves over time: mean number of waves between entry and drain
    span = float(t[:, 9].max())
    grid = np.linspace(0.0, span, 200)
    resident = [int(np.sum((t[:, 0] <= g) & (t[:, 9] > g))) for g in grid]
    summary = {"event_us": round(e0.elapsed_time(e1) * 1e3, 2), "span_us": round(span, 2), "waves": int(len(t)),
               "wave_lifetime_us_p5_50_95": q(total), "phases_us_p5_50_95": phases,
               "phase_share_of_median_lifetime": {name: round(float(np.median(t[:, k1] - t[:, k0]) /
                                                                    max(np.median(total), 1e-9)), 3)
                                                  for name, k0, k1 in PHASES},
               "resident_waves_p50_max": [int(np.median(resident)), int(max(resident))],
               "last_entry_us": round(float(t[:, 0].max()), 2)}
    print(json.dumps(summary))
    # timeline: per 2 us bin, waves resident / in the rules phase / waiting
    # at a barrier, and waves that entered
    rows = []
    for lo in np.arange(0.0, span, 2.0):
        mid = lo + 1.0
        res = int(np.sum((t[:, 0] <= mid) & (t[:, 9] > mid)))
        rules = int(np.sum((t[:, 3] <= mid) & (t[:, 4] > mid)))
        wait = int(np.sum(((t[:, 2] <= mid) & (t[:, 3] > mid)) | ((t[:, 4] <= mid) & (t[:, 5] > mid)) |
                          ((t[:, 6] <= mid) & (t[:, 7] > mid))))
        entered = int(np.sum((t[:, 0] >= lo) & (t[:, 0] < lo + 2.0)))
        rows.append({"t_us": float(lo), "resident": res, "rules": rules, "barrier": wait, "entered": entered})
        print(f"{lo:6.1f}  resident {res:5d}  rules {rules:5d}  barrier {wait:5d}  entered {entered:5d}")
    summary["timeline_2us"] = rows
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(summary, f)


if __name__ == "__main__":
    main()
