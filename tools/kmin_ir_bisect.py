"""Round 4's k_min<0> defect: which IR pass of llc's pipeline puts a poison
value on a path to the kernel's store?  The committed SLP IR
(profiles/r04/codegen/kmin_slp.ll) runs through llc's IR passes up to and
including pass P with its <2 x i32> vectors (-stop-after=P), is scalarized
there (opt's scalarizer, semantics-preserving), and continues from P
(-start-after=P) to instruction selection; tools/mir_emu.py runs the
machine IR right after amdgpu-isel on oracle cases and counts records
stored with an undefined word.  Scalarized from the start: none; vectors
to the end: the defect.  The first P after which the count is non-zero
made the poison path.  Investigation tool (the oracle is the checker, as
in tests/).

    python tools/kmin_ir_bisect.py [cases]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import mir_emu  # noqa: E402
from test_kmin_isa_emulation import cases, DST  # noqa: E402

B = "/opt/rocm/llvm/bin"
T = ["-mtriple=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-O3"]
SRC = os.path.join(ROOT, "profiles", "r04", "codegen", "kmin_slp.ll")
OUT = os.path.join(ROOT, "build", "w3phi", "irbisect")
PASSES = ["early-cse", "amdgpu-codegenprepare", "codegenprepare", "load-store-vectorizer", "amdgpu-lower-intrinsics",
          "lowerswitch", "flattencfg", "sink", "amdgpu-late-codegenprepare", "amdgpu-unify-divergent-exit-nodes",
          "fix-irreducible", "unify-loop-exits", "structurizecfg", "amdgpu-annotate-uniform",
          "si-annotate-control-flow", "amdgpu-rewrite-undef-for-phi", "lcssa"]


def unwrap(mir, ll):
    lines = open(mir).read().split("\n")
    if not lines[0].startswith("--- |"):
        open(ll, "w").write("\n".join(lines))
        return
    out = []
    for ln in lines[1:]:
        if ln.startswith("...") or ln.startswith("---"):
            break
        out.append(ln[2:] if ln.startswith("  ") else ln)
    open(ll, "w").write("\n".join(out) + "\n")


def isel_mir(ll, start_after=None):
    args = [B + "/llc"] + T + (["-start-after=" + start_after] if start_after else []) + \
        ["-print-after=amdgpu-isel", "-stop-after=amdgpu-isel", ll, "-o", os.devnull]
    r = subprocess.run(args, capture_output=True, text=True, check=True)
    return r.stderr.split("# Machine code for function", 1)[1]


def undefined_stores(body, cs):
    mach = mir_emu.Machine(mir_emu.Function(body))
    n = 0
    for rec, a, _ in cs:
        mem = {DST + 4 * k: rec[k] for k in range(4)}
        mach.run({0: DST, 0x20: a}, mem)
        n += any(mem.get(DST + 4 * k) is None for k in range(4))
    return n


def main():
    ncases = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    os.makedirs(OUT, exist_ok=True)
    cs = cases(ncases)
    scal0 = os.path.join(OUT, "scal_from_start.ll")
    subprocess.run([B + "/opt", "-passes=scalarizer<load-store>", SRC, "-S", "-o", scal0], check=True)
    print("scalarized from the start: %d of %d records with an undefined word" % (undefined_stores(isel_mir(scal0), cs),
                                                                                len(cs)), flush=True)
    print("vectors to the end:        %d" % undefined_stores(isel_mir(SRC), cs), flush=True)
    for p in PASSES:
        mir, ll, sc = (os.path.join(OUT, x % p) for x in ("after_%s.mir", "after_%s.ll", "after_%s_scal.ll"))
        subprocess.run([B + "/llc"] + T + ["-stop-after=" + p, SRC, "-o", mir], check=True)
        unwrap(mir, ll)
        subprocess.run([B + "/opt", "-passes=scalarizer<load-store>", ll, "-S", "-o", sc], check=True)
        print("vectors through %-34s then scalar: %d" % (p, undefined_stores(isel_mir(sc, p), cs)), flush=True)


if __name__ == "__main__":
    main()
