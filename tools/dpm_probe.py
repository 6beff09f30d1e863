"""Power-state dependence of the c3 step on the GPU box: why the same graph
runs at ~133 us per step in a sustained A/B loop (tools/pipe_ab.py) and at
~145-155 us as bench.py's timed replay (VERDICT r4 item 2's "profile within
2 %" needs the two to agree).  Measurement tool only; reads the GPU's
metrics (amdsmi, read-only: clocks, socket power, temperatures, throttle
residency counters) from a sampling thread while the process replays:

  A  the bench's sequence (settle rollout, W eager steps, capture K steps),
     then R replays of the K-step graph each after an idle gap;
  B  R replays back to back (no host sync in between);
  C  R x K store-only sweeps of the same [B][2][98] buffer back to back.

One JSON line per replay (us per step, the metrics sampled during it) and
one per phase with the means.

    python tools/dpm_probe.py [--batch B] [--steps K] [--replays R] [--idle-ms MS]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KEYS = ("current_gfxclk", "average_gfxclk_frequency", "current_uclk", "average_uclk_frequency", "current_socket_power",
        "average_socket_power", "temperature_hotspot", "temperature_mem", "average_umc_activity",
        "average_gfx_activity", "throttle_status", "ppt_residency_acc", "socket_thm_residency_acc",
        "hbm_thm_residency_acc", "prochot_residency_acc", "accumulation_counter")


class Sampler:
    def __init__(self, bdf, period_s=0.002):
        self.samples, self.ok, self.err = [], False, None
        self.period = period_s
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self.h = amdsmi.amdsmi_get_processor_handle_from_bdf(bdf)
            self.get = amdsmi.amdsmi_get_gpu_metrics_info
            self.get(self.h)
            self.ok = True
        except Exception as e:  # metrics are best effort
            self.err = repr(e)
        self.stop = threading.Event()
        self.t = threading.Thread(target=self.run, daemon=True)

    def run(self):
        while not self.stop.is_set():
            try:
                m = self.get(self.h)
                self.samples.append((time.perf_counter(), {k: m.get(k) for k in KEYS}))
            except Exception as e:
                self.err = repr(e)
            time.sleep(self.period)

    def window(self, t0, t1):
        w = [m for t, m in self.samples if t0 <= t <= t1]
        out = {"n": len(w)}
        for k in KEYS:
            vals = [v for v in (m.get(k) for m in w) if isinstance(v, (int, float))]
            if vals:
                out[k] = round(sum(vals) / len(vals), 1) if "acc" not in k else [vals[0], vals[-1]]
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--replays", type=int, default=30)
    ap.add_argument("--idle-ms", type=float, default=20.0)
    ap.add_argument("--settle", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    import ctypes

    import torch

    import bench
    from open_spiel_coup_amd import BatchedCoupEnv, _native
    box = bench._box_identity(0)
    sampler = Sampler(box.get("pci", ""))
    print(json.dumps({"box": box, "metrics": sampler.ok, "metrics_error": sampler.err}), flush=True)
    if sampler.ok:
        sampler.t.start()
    env = BatchedCoupEnv(a.batch, seed=1, auto_reset=True, obs=True, device="cuda:0",
                         episode_stats=bench.episode_stats_mode(bench.payload_width(2, a.steps, a.batch)))
    stream = torch.cuda.current_stream()
    env.rollout(a.settle)
    for _ in range(a.warmup):
        env.step()
    env.clear_episode_stats()
    g = env.capture_steps(a.steps)
    lib = _native.load()
    obs = env.obs
    sweep = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(stream)
    with torch.cuda.graph(sweep, stream=side):
        for _ in range(a.steps):
            _native.check(lib.coup_measure_store_sweep(ctypes.c_void_p(obs.data_ptr()), obs.numel() // 4, 512, 2, 0,
                                                       ctypes.c_void_p(side.cuda_stream)))
    stream.wait_stream(side)
    torch.cuda.synchronize()

    def run_phase(name, graph, idle):
        evs = []
        walls = []
        for r in range(a.replays):
            if idle:
                torch.cuda.synchronize()
                time.sleep(a.idle_ms * 1e-3)
            env.clear_episode_stats()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            graph.replay()
            e1.record(stream)
            evs.append((e0, e1))
            if idle:
                t0 = time.perf_counter()
                e1.synchronize()
                walls.append((t0, time.perf_counter()))
        torch.cuda.synchronize()
        t_end = time.perf_counter()
        us = [e0.elapsed_time(e1) * 1e3 / a.steps for e0, e1 in evs]
        for r, u in enumerate(us):
            line = {"phase": name, "replay": r, "us_per_step": round(u, 2)}
            if idle and sampler.ok:
                line["metrics"] = sampler.window(walls[r][0] - u * a.steps * 1e-6, walls[r][1])
            print(json.dumps(line), flush=True)
        return us, t_end

    res = {}
    for name, graph, idle in (("A_idle_gaps", g, True), ("B_back_to_back", g, False), ("C_sweep_back_to_back", sweep, False),
                              ("D_back_to_back_again", g, False)):
        t0 = time.perf_counter()
        us, t1 = run_phase(name, graph, idle)
        summ = {"phase": name, "mean_us": round(sum(us) / len(us), 2), "first5": [round(x, 1) for x in us[:5]],
                "last5": [round(x, 1) for x in us[-5:]]}
        if sampler.ok:
            summ["metrics"] = sampler.window(t0, t1)
        res[name] = summ
        print(json.dumps(summ), flush=True)
    if sampler.ok:
        sampler.stop.set()
        sampler.t.join()
    assert env.error_count() == 0


if __name__ == "__main__":
    main()
