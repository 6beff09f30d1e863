"""Per-wave timeline of one c3 step, or with --obs 0 one c2 step (measurement
builds only).

    python -m open_spiel_coup_amd.build --out ab/trace.so --define COUP_WAVE_TRACE
    COUP_LIB_PATH=ab/trace.so python tools/wave_trace.py [--batch B] [--steps K]

The trace build stamps s_memrealtime (100 MHz) per wave at kernel entry (t0),
end of the step compute (t1), end of the obs store issue (t2), after
s_waitcnt vmcnt(0) (t3), and when the lane records' load has returned.  Prints a JSON summary and a timeline: per 4 us bin,
how many waves are computing / issuing stores / draining, and the obs bytes
whose store issue falls in the bin (each wave's 50 KiB spread evenly over its
issue window).  Measurement tool only.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--bin-us", type=float, default=4.0)
    ap.add_argument("--mode", default=None, help="COUP_OBS_MODE for the traced steps")
    ap.add_argument("--quiet", action="store_true", help="summary only")
    ap.add_argument("--obs", type=int, default=1, help="0: the c2 step (no observation writer)")
    a = ap.parse_args()
    if a.mode:
        os.environ["COUP_OBS_MODE"] = a.mode
    import torch

    from open_spiel_coup_amd import BatchedCoupEnv
    from open_spiel_coup_amd import _native
    lib = _native.load()
    if not hasattr(lib, "coup_debug_set_trace"):
        raise SystemExit("not a COUP_WAVE_TRACE build (set COUP_LIB_PATH)")
    lib.coup_debug_set_trace.argtypes = [ctypes.c_void_p]
    env = BatchedCoupEnv(a.batch, seed=1, auto_reset=True, obs=bool(a.obs), device="cuda:0")
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
    tr = buf.view(waves, 10).cpu().numpy()
    tr = tr[tr[:, 0] != 0]  # a persistent grid has fewer waves than groups
    waves = len(tr)
    t = (tr[:, :4] - tr[:, 0].min()).astype(np.float64) / 100.0  # us
    hw = tr[:, 4]
    xcc = (hw & 0xFFFFFFFF).astype(np.int64) & 0xF
    span = t[:, 3].max()
    comp, issue, drain = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    load = (tr[:, 5] - tr[:, 0]).astype(np.float64) / 100.0  # state load latency (us)
    late = t[:, 0] > 0.75 * t[:, 0].max()
    # step segments (stamps 5..9: record loaded, action drawn, decision applied,
    # deals resolved, end of the step incl. the reset of finished lanes)
    seg = {}
    for name, k0, k1 in (("mask_and_draw", 5, 6), ("apply_decision", 6, 7), ("deals", 7, 8), ("reset", 8, 9),
                         ("outputs_and_obs_bits", 9, None)):
        a0 = tr[:, k0].astype(np.float64)
        a1 = (tr[:, k1] if k1 is not None else tr[:, 0] + (t[:, 1] * 100.0).astype(np.int64)).astype(np.float64)
        ok = (tr[:, k0] != 0) & ((tr[:, k1] != 0) if k1 is not None else True)
        if ok.any():
            seg[name] = [round(float(v), 2) for v in np.percentile((a1[ok] - a0[ok]) / 100.0, [5, 50, 95])]
    q = lambda x: [round(float(v), 2) for v in np.percentile(x, [5, 50, 95])]
    summary = {"mode": a.mode, "obs": a.obs, "batch": a.batch, "event_us": round(e0.elapsed_time(e1) * 1e3, 2), "span_us": round(float(span), 2), "waves": int(waves),
               "compute_us_p5_50_95": q(comp), "issue_us_p5_50_95": q(issue), "drain_us_p5_50_95": q(drain),
               "load_us_p5_50_95": q(load), "late_waves_load_us_p5_50_95": q(load[late]),
               "late_waves_compute_us_p5_50_95": q(comp[late]),
               "first_store_issue_us": round(float(t[:, 1].min()), 2),
               "last_entry_us": round(float(t[:, 0].max()), 2),
               "xcc_counts": np.bincount(xcc, minlength=8).tolist(),
               "segments_us_p5_50_95": seg}
    print(json.dumps(summary))
    nb = int(np.ceil(span / a.bin_us))
    rows = []
    bytes_per_wave = 64 * 784
    for b in range(nb):
        lo, hi = b * a.bin_us, (b + 1) * a.bin_us
        c = int(np.sum((t[:, 0] < hi) & (t[:, 1] > lo)))
        i = int(np.sum((t[:, 1] < hi) & (t[:, 2] > lo)))
        d = int(np.sum((t[:, 2] < hi) & (t[:, 3] > lo)))
        w = np.clip(np.minimum(t[:, 2], hi) - np.maximum(t[:, 1], lo), 0, None) / np.maximum(issue, 1e-3)
        gbs = float(np.sum(w) * bytes_per_wave / (a.bin_us * 1e-6) / 1e9)
        rows.append({"t_us": lo, "computing": c, "issuing": i, "draining": d, "issue_GBps": round(gbs)})
        if not a.quiet:
            print(f"{lo:7.1f}  comp {c:6d}  issue {i:6d}  drain {d:6d}  issue-rate {gbs:8.0f} GB/s")
    with open(os.path.join(ROOT, "gpurun_out", f"wave_trace_m{a.mode or 'default'}_obs{a.obs}_b{a.batch}.json"), "w") as f:
        json.dump({"summary": summary, "timeline": rows}, f)


if __name__ == "__main__":
    main()
