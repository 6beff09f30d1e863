"""Build libcoup_mi355x.so in-tree with hipcc for gfx950.

    python -m open_spiel_coup_amd.build [--force] [--verbose]

The .so is git-ignored but travels to the GPU box with the gpurun snapshot.
"""
import argparse
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SOURCES = [os.path.join(CSRC, "coup_kernels.hip"), os.path.join(CSRC, "coup_nplayer.hip")]
DEPS = SOURCES + [os.path.join(CSRC, h) for h in ("coup_lane.h", "coup_nlane.h", "coup_np.h", "coup_regroup.h")] + [
    os.path.join(ROOT, "include", "coup_mi355x.h")]
OUT = os.path.join(HERE, "libcoup_mi355x.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("COUP_OFFLOAD_ARCH", "gfx950")


def command(resource_usage=False, out=OUT, defines=()):
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-I", os.path.join(ROOT, "include"), "-o", out] + [f"-D{d}" for d in defines] + SOURCES
    if resource_usage:
        cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
    return cmd


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(p) <= t for p in DEPS)


def build(force=False, verbose=False):
    if not force and up_to_date():
        return OUT
    cmd = command(resource_usage=verbose)
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    return OUT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--out", default=None, help="measurement builds: write the library elsewhere")
    ap.add_argument("--define", action="append", default=[], help="measurement builds: e.g. COUP_WAVE_TRACE")
    a = ap.parse_args()
    if a.out or a.define:
        out = os.path.abspath(a.out or OUT)
        subprocess.check_call(command(a.verbose, out, a.define))
        print(out)
        return
    print(build(force=a.force, verbose=a.verbose))


if __name__ == "__main__":
    main()
