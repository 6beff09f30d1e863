"""Round 4's k_min<0> defect on the CPU: the
committed llc -O3 assembly of the reproducer's SLP IR
(profiles/r04/codegen/kmin_slp_O3.s) and of the same IR after opt's
scalarizer (kmin_slpscal_O3.s), executed instruction by instruction by a
one-lane emulator of the instructions they use (tools/salu_emu.py), on
records and actions from the oracle's random play.  The scalarized code
matches the oracle on every case; the vector code's wrong records are
reproduced without a GPU, so they are in the instructions llc emitted, not
in how the hardware runs them.  Test infrastructure: the oracle is the
checker.
"""
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)

import salu_emu  # noqa: E402
from oracle import oracle  # noqa: E402

CODEGEN = os.path.join(ROOT, "profiles", "r04", "codegen")
DST = 0x2000


def cases(n, seed=5):
    rng = random.Random(seed)
    out = []
    while len(out) < n:
        st = oracle.OracleState()
        for _ in range(rng.randrange(64)):
            acts = st.legal_actions()
            if not acts:
                break
            nxt = st.clone()
            nxt.apply_action(rng.choice(acts))
            if nxt.is_terminal():
                break
            st = nxt
        acts = st.legal_actions()
        if st.is_terminal() or not acts:
            continue
        a = rng.choice(acts)
        after = st.clone()
        after.apply_action(a)
        out.append((st.pack(), a, after.pack()))
    return out


def run(prog, rec, action):
    mem = salu_emu.Memory()
    for k in range(4):
        mem.store32(DST + 4 * k, rec[k])
    prog.run({0: DST, 0x20: action}, mem)
    return [mem.load32(DST + 4 * k) for k in range(4)]


@pytest.fixture(scope="module")
def programs():
    return {v: salu_emu.Program(open(os.path.join(CODEGEN, f"kmin_{v}_O3.s")).read()) for v in ("slp", "slpscal")}


def test_kmin_isa_emulation(programs):
    cs = cases(1500)
    bad = {"slp": 0, "slpscal": 0}
    words = [0, 0, 0, 0]
    for rec, a, want in cs:
        for v, prog in programs.items():
            got = run(prog, rec, a)
            if got != want:
                bad[v] += 1
                if v == "slp":
                    for k in range(4):
                        words[k] += got[k] != want[k]
    print("mismatches of", len(cs), bad, "slp words", words)
    assert bad["slpscal"] == 0
    assert bad["slp"] > 0  # the defect, reproduced from the instructions alone


LLC = "/opt/rocm/llvm/bin/llc"


@pytest.mark.skipif(not os.path.exists(LLC), reason="needs the ROCm llc")
def test_structurizecfg_routes_poison_to_the_store(tmp_path):
    """tools/kmin_ir_bisect.py in small: the SLP IR's <2 x i32> values carried
    through llc's IR passes up to unify-loop-exits and scalarized there give
    machine code (right after amdgpu-isel) that stores no undefined word;
    carried one pass further, through structurizecfg, it stores undefined
    words 2 and 3 on the failing cases."""
    import kmin_ir_bisect as kb
    kb.OUT = str(tmp_path)
    cs = cases(120)
    got = {}
    for p in ("unify-loop-exits", "structurizecfg"):
        mir, ll, sc = (str(tmp_path / (x % p)) for x in ("after_%s.mir", "after_%s.ll", "after_%s_scal.ll"))
        import subprocess
        subprocess.run([LLC] + kb.T + ["-stop-after=" + p, kb.SRC, "-o", mir], check=True)
        kb.unwrap(mir, ll)
        subprocess.run([kb.B + "/opt", "-passes=scalarizer<load-store>", ll, "-S", "-o", sc], check=True)
        got[p] = kb.undefined_stores(kb.isel_mir(sc, p), cs)
    print(got)
    assert got["unify-loop-exits"] == 0
    assert got["structurizecfg"] > 0
