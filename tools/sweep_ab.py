"""Store-only ceilings of the split writers' buffers on this box, shape by
shape, interleaved in ONE process (measurement build: COUP_LIB_PATH=
build/variants/libcoup_mi355x.so for shapes other than 512 x 2 / 1024 x 2
and for the resident grid-stride form).

    COUP_LIB_PATH=build/variants/libcoup_mi355x.so python tools/sweep_ab.py [--rounds R]

Buffers: c3's [2^20][2][98] fp32 (822 MB) and c3i's [2^18][2][2492] fp32
(5.23 GB).  Each shape, with the tensor-like data (0.0, a 1.0 in one float
of 32) and with index bits in every float (COUP_SWEEP_INDEX_BITS): K
launches of coup_measure_store_sweep replayed from one HIP graph, the mean
per launch; one JSON line per (buffer, shape, data) with the median over
rounds and the rate.  With --gap-sleep an idle kernel separates the sweeps,
so the rate printed here includes it; read the sweep's own duration from a
rocprofv3 --kernel-trace --stats run of the same command.  Measurement tool only.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

R, BITS = 1, 2  # _native.SWEEP_RESIDENT, _native.SWEEP_INDEX_BITS


def PACE(n):  # measurement builds: a dependent chain of n integer ops ahead of each store
    return n << 8


WRITERLIKE = 1 << 16  # measurement builds: load -> LDS -> barrier -> stores, no decode


def DENS(d):  # measurement builds: a 1.0 per 2^(d-1) float4s, all zeros at 31 (share of all-zero lines)
    return d << 17


SHAPES = [(512, 2, 0), (1024, 2, 0), (512, 2, BITS), (1024, 2, BITS), (256, 2, 0), (512, 4, 0), (1024, 4, 0),
          (1024, 8, 0), (512, 2, R), (1024, 2, R), (1024, 8, R), (512, 2, PACE(8)), (512, 2, PACE(24)),
          (512, 2, PACE(64)), (1024, 2, PACE(24)), (1024, 2, PACE(64)), (512, 2, WRITERLIKE), (1024, 2, WRITERLIKE),
          (512, 2, DENS(1)), (512, 2, DENS(4)), (512, 2, DENS(5)), (512, 2, DENS(6)), (512, 2, DENS(8)),
          (512, 2, DENS(31)), (1024, 2, DENS(1)), (1024, 2, DENS(6)), (1024, 2, DENS(31))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--gap-sleep", type=int, default=0,
                    help="cycles of an idle kernel between sweeps (per-kernel durations then from rocprofv3)")
    ap.add_argument("--only", default=None, help="comma list of shape indices into SHAPES")
    a = ap.parse_args()
    import torch
    from open_spiel_coup_amd import _native
    lib = _native.load()
    ab = bool(lib.coup_build_flags() & _native.BUILD_AB_VARIANTS)
    shapes = SHAPES if ab else [s for s in SHAPES if not s[2] & (R | 0x3FFF00) and s[:2] in ((512, 2), (1024, 2))]
    if a.only:
        shapes = [shapes[int(i)] for i in a.only.split(",")]
    bufs = {"c3_obs": (1 << 20) * 2 * 98, "c3i_info": (1 << 18) * 2 * 2492}
    stream = torch.cuda.current_stream()
    graphs = {}
    for name, nfloat in bufs.items():
        buf = torch.empty(nfloat, dtype=torch.float32, device="cuda")
        for (t, s, r) in shapes:
            def launch(sv, buf=buf, t=t, s=s, r=r):
                _native.check(lib.coup_measure_store_sweep(ctypes.c_void_p(buf.data_ptr()), buf.numel() // 4, t, s,
                                                           r, ctypes.c_void_p(sv)))
            for _ in range(2):
                launch(stream.cuda_stream)
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(stream)
            with torch.cuda.graph(g, stream=side):
                for _ in range(a.steps):
                    launch(side.cuda_stream)
                    if a.gap_sleep:
                        torch.cuda._sleep(a.gap_sleep)
            stream.wait_stream(side)
            graphs[(name, t, s, r)] = (g, buf)
    times = {k: [] for k in graphs}
    for _ in range(a.rounds):
        for k, (g, _) in graphs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            g.replay()
            e1.record(stream)
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3 / a.steps)
    for (name, t, s, r), ts in times.items():
        med = statistics.median(ts)
        nbytes = bufs[name] * 4
        print(json.dumps({"buffer": name, "bytes": nbytes, "threads": t, "passes": s, "resident": bool(r & R),
                          "data": "index bits" if r & BITS else "tensor-like", "pace_ops": (r >> 8) & 0xFF, "writerlike": bool(r & WRITERLIKE),
                          "dens": (r >> 17) & 0x1F,
                          "median_us": round(med, 2), "min_us": round(min(ts), 2),
                          "tb_per_s": round(nbytes / (med * 1e-6) / 1e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
