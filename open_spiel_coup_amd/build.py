"""Build the libraries in-tree.

    python -m open_spiel_coup_amd.build [--force] [--verbose]

  libcoup_mi355x.so   the kernels and the C ABI (include/coup_mi355x.h), hipcc
                      for gfx950: the shipped kernels only;
  build/variants/libcoup_mi355x.so
                      the same with -DCOUP_AB_VARIANTS: every measured and
                      rejected kernel variant too, chosen by environment
                      variables at coup_create (csrc/coup_knobs.h) -- A/B
                      runs and their equality tests (COUP_LIB_PATH);
  librust_spiel.so    the reference's per-state C ABI (rust_open_spiel.h,
                      include/coup_rust_abi.h) over it, host C++ (g++), so the
                      reference's Rust crate links it as `dylib=rust_spiel`.

The .so files are git-ignored but travel to the GPU box with the gpurun
snapshot.
"""
import argparse
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SOURCES = [os.path.join(CSRC, "coup_kernels.hip"), os.path.join(CSRC, "coup_nplayer.hip")]
# the per-game State ops on the host (same rules header, g++), linked into the
# same library (csrc/coup_host.cpp)
HOST_SRC = os.path.join(CSRC, "coup_host.cpp")
HOST_INC = os.path.join(CSRC, "host")
DEPS = SOURCES + [os.path.join(CSRC, h) for h in ("coup_lane.h", "coup_nlane.h", "coup_np.h", "coup_regroup.h", "coup_episodes.h",
                                                 "coup_tensor.h", "coup_knobs.h", "coup_launch_log.h")] + [
    os.path.join(ROOT, "include", "coup_mi355x.h"), HOST_SRC, os.path.join(HOST_INC, "hip", "hip_runtime.h")]
OUT = os.path.join(HERE, "libcoup_mi355x.so")
OBJ_DIR = os.path.join(ROOT, "build", "obj")  # git-ignored (build/)
# the measurement build (every A/B variant; csrc/coup_knobs.h)
VARIANTS_OUT = os.path.join(ROOT, "build", "variants", "libcoup_mi355x.so")
VARIANTS_OBJ_DIR = os.path.join(OBJ_DIR, "variants")
VARIANTS_DEFINE = "COUP_AB_VARIANTS"
RUST_SRC = os.path.join(CSRC, "rust_spiel.cpp")
RUST_DEPS = [RUST_SRC, os.path.join(ROOT, "include", "coup_rust_abi.h"), os.path.join(ROOT, "include", "coup_mi355x.hpp"),
             os.path.join(ROOT, "include", "coup_mi355x.h")]
RUST_OUT = os.path.join(HERE, "librust_spiel.so")
# _coup_host: the CPython binding of the library's host State ops (pyspiel)
EXT_SRC = os.path.join(CSRC, "host_ext.c")


def ext_out():
    import sysconfig
    return os.path.join(HERE, "_coup_host" + sysconfig.get_config_var("EXT_SUFFIX"))


def ext_command(out=None):
    """_coup_host: C over the CPython API, linked to libcoup_mi355x.so (found
    next to it through $ORIGIN)."""
    import sysconfig
    return [os.environ.get("CC", "gcc"), "-O2", "-fPIC", "-shared", "-Wall", "-I", sysconfig.get_paths()["include"],
            "-I", os.path.join(ROOT, "include"), EXT_SRC, "-o", out or ext_out(), "-L", HERE, "-lcoup_mi355x",
            "-Wl,-rpath,$ORIGIN"]
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("COUP_OFFLOAD_ARCH", "gfx950")


# LLVM's SLP vectorizer is off for every device build: on the packed-record
# rules it is the pass that triggers the ROCm 7.2 defect of DESIGN.md
# section 12 (record word 3 after NextPlayerMove paths) -- an opt-bisect over
# the IR passes puts the first failing limit exactly at slp-vectorizer on the
# reproducer's k_min<0>, and without it every reproducer variant and the
# run-time-branch step that failed in round 3 come out right.  The kernels
# are 0.7-1% faster without it (profiles/r03/codegen/).
NO_SLP = "-fno-slp-vectorize"

# Optimisation level per source.  -O2 measured 1% faster than -O3 for the
# 6-player step (33.7-34.0 against 33.9-34.5 us) but 6% slower for its
# trajectory kernel (26.3-26.5 against 24.7-24.9 us per step) and 0.5-1 us
# slower for the headline c3 step (alternating processes,
# profiles/r03/ab/compiler_flags.txt, o2_vs_o3_np_trajectory.txt): -O3 for both.
OPT = {"coup_kernels.hip": "-O3", "coup_nplayer.hip": "-O3"}


def host_command(obj):
    """coup_host.cpp -> obj: host C++ (g++), the lane rules through the
    csrc/host stand-in of the few HIP names they use."""
    return [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-Wall", "-Wno-unknown-pragmas", "-I", HOST_INC,
            "-I", CSRC, "-I",
            os.path.join(ROOT, "include"), "-c", HOST_SRC, "-o", obj]


HOST_OBJ = os.path.join(OBJ_DIR, "coup_host.o")


def command(resource_usage=False, out=OUT, defines=()):
    """Measurement builds: one hipcc command over the HIP sources and the
    host object (build it first with host_command(HOST_OBJ))."""
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", NO_SLP, "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-I", os.path.join(ROOT, "include"), "-o", out] + [f"-D{d}" for d in defines] + SOURCES + [HOST_OBJ]
    if resource_usage:
        cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
    return cmd


def rust_command(out=RUST_OUT):
    """librust_spiel.so: host-only C++ over libcoup_mi355x.so (found next to it
    through $ORIGIN) and the HIP runtime."""
    return [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-D__HIP_PLATFORM_AMD__",
            "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROCM, "include"), RUST_SRC, "-o", out,
            "-L", HERE, "-lcoup_mi355x", "-L", os.path.join(ROCM, "lib"), "-lamdhip64",
            "-Wl,-rpath,$ORIGIN:" + os.path.join(ROCM, "lib")]


REPRO_SRC = os.path.join(ROOT, "tools", "slot_inline_repro.hip")
REPRO_OUT = os.path.join(ROOT, "build", "slot_inline_repro")


INFO_REPRO_SRC = os.path.join(ROOT, "tools", "info_prefix_repro.hip")
INFO_REPRO_OUT = os.path.join(ROOT, "build", "info_prefix_repro")


def info_repro_command():
    """The uint2-prefix reproducer of round 4's k_info_sweep sighting
    (tests/test_gpu_codegen_hazard.py), with the product's device flags."""
    return [HIPCC, f"--offload-arch={ARCH}", "-O3", NO_SLP, "-std=c++17", "-I", os.path.join(ROOT, "include"),
            "-I", CSRC, INFO_REPRO_SRC, "-o", INFO_REPRO_OUT]


def build_repro(force=False):
    """The k_slot miscompile reproducer (investigation tool, DESIGN.md
    section 12; tests/test_gpu_codegen_hazard.py runs it on the GPU)."""
    deps = [REPRO_SRC] + DEPS
    if not force and up_to_date(REPRO_OUT, deps):
        return REPRO_OUT
    os.makedirs(os.path.dirname(REPRO_OUT), exist_ok=True)
    subprocess.check_call(repro_command())
    return REPRO_OUT


def repro_command():
    # COUP_RULES_V1: the branch-form decision transition, the form the inlined
    # k_slot miscompiles (the effect form, default since round 2, happens to
    # compile correctly inline: DESIGN.md section 12)
    return [HIPCC, f"--offload-arch={ARCH}", "-O3", NO_SLP, "-std=c++17", "-DCOUP_RULES_V1", "-I", os.path.join(ROOT, "include"),
            "-I", CSRC, REPRO_SRC, os.path.join(CSRC, "coup_nplayer.hip"), "-o", REPRO_OUT]


def up_to_date(out=OUT, deps=DEPS):
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(p) <= t for p in deps)


def _run_all(cmds, verbose=False):
    """Run compiler commands concurrently (one process each); raise if any fails."""
    procs = []
    for cmd in cmds:
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((cmd, subprocess.Popen(cmd)))
    failed = [cmd for cmd, p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])


def build(force=False, verbose=False, repro=False, variants=True):
    """libcoup_mi355x.so (its two HIP sources compiled concurrently, then
    linked), with `variants` the measurement build beside it
    (build/variants/), librust_spiel.so, and with `repro` the section-12
    reproducer, in one batch of compiler processes."""
    jobs, links = [], []
    lib_stale = force or not up_to_date()
    var_stale = variants and (force or not up_to_date(VARIANTS_OUT))
    if lib_stale or var_stale:
        jobs.append(host_command(HOST_OBJ))
    for stale, odir, out, defines in ((lib_stale, OBJ_DIR, OUT, ()),
                                      (var_stale, VARIANTS_OBJ_DIR, VARIANTS_OUT, (VARIANTS_DEFINE,))):
        if not stale:
            continue
        os.makedirs(odir, exist_ok=True)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        objs = []
        for src in SOURCES:
            obj = os.path.join(odir, os.path.basename(src) + ".o")
            objs.append(obj)
            cmd = [HIPCC, f"--offload-arch={ARCH}", OPT[os.path.basename(src)], NO_SLP, "-std=c++17", "-fPIC", "-Wall", "-I",
                   os.path.join(ROOT, "include"), "-c", src, "-o", obj] + [f"-D{d}" for d in defines]
            if verbose:
                cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
            jobs.append(cmd)
        links.append([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + [HOST_OBJ])
    if repro and (force or not up_to_date(REPRO_OUT, [REPRO_SRC] + DEPS)):
        os.makedirs(os.path.dirname(REPRO_OUT), exist_ok=True)
        jobs.append(repro_command())
    if repro and (force or not up_to_date(INFO_REPRO_OUT, [INFO_REPRO_SRC] + DEPS)):
        os.makedirs(os.path.dirname(INFO_REPRO_OUT), exist_ok=True)
        jobs.append(info_repro_command())
    _run_all(jobs, verbose)
    if links:
        _run_all(links, verbose)
    if force or not up_to_date(RUST_OUT, RUST_DEPS + [OUT]):
        cmd = rust_command()
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
    if force or not up_to_date(ext_out(), [EXT_SRC, os.path.join(ROOT, "include", "coup_mi355x.h"), OUT]):
        cmd = ext_command()
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
    ap.add_argument("--no-variants", action="store_true", help="skip the A/B-variant measurement build")
    a = ap.parse_args()
    if a.out or a.define:
        # a measurement build: objects per source under build/obj/m_<defines>/
        # (hipcc would take the host object for a HIP source in one command)
        out = os.path.abspath(a.out or OUT)
        odir = os.path.join(OBJ_DIR, "m_" + ("_".join(a.define) or "plain"))
        os.makedirs(odir, exist_ok=True)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        host_obj = os.path.join(odir, "coup_host.o")
        jobs, objs = [host_command(host_obj)], []
        for src in SOURCES:
            obj = os.path.join(odir, os.path.basename(src) + ".o")
            objs.append(obj)
            jobs.append([HIPCC, f"--offload-arch={ARCH}", OPT[os.path.basename(src)], NO_SLP, "-std=c++17", "-fPIC",
                         "-Wall", "-I", os.path.join(ROOT, "include"), "-c", src, "-o", obj] +
                        [f"-D{d}" for d in a.define])
        _run_all(jobs, a.verbose)
        _run_all([[HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + [host_obj]], a.verbose)
        print(out)
        return
    print(build(force=a.force, verbose=a.verbose, variants=not a.no_variants))


if __name__ == "__main__":
    main()
