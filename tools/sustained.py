"""Step time under sustained load: the c3 step run back to back for a while,
one line per ~second with the mean step time and the GPU's reported clocks
and power (measurement tool; shows how the step slows as the GPU heats).

    python tools/sustained.py [--seconds 60] [--config c3]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def smi():
    try:
        out = subprocess.run(["rocm-smi", "--showpower", "--showtemp", "--showclocks"], capture_output=True,
                             text=True, timeout=10).stdout
    except Exception:
        return {}
    keep = {}
    for line in out.splitlines():
        low = line.lower()
        for key in ("power", "sclk", "mclk", "fclk", "temperature (sensor edge)", "temperature (sensor junction)",
                    "temperature (sensor memory)"):
            if key in low and ":" in line:
                keep[key] = line.split(":", 2)[-1].strip()
    return keep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--batch", type=int, default=1 << 20)
    a = ap.parse_args()
    import torch

    from open_spiel_coup_amd import BatchedCoupEnv
    env = BatchedCoupEnv(a.batch, seed=1, auto_reset=True, obs=True, device="cuda:0")
    env.rollout(256)
    t_start = time.time()
    while time.time() - t_start < a.seconds:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        n = 0
        t0 = time.time()
        while time.time() - t0 < 1.0:
            for _ in range(50):
                env.step()
            n += 50
            torch.cuda.synchronize()
        e1.record()
        e1.synchronize()
        line = {"t_s": round(time.time() - t_start, 1), "step_us": round(e0.elapsed_time(e1) * 1e3 / n, 1)}
        line.update(smi())
        print(json.dumps(line), flush=True)
    assert env.error_count() == 0


if __name__ == "__main__":
    main()
