"""The code-generation hazard of DESIGN.md section 12, kept under watch.

build/slot_inline_repro (tools/slot_inline_repro.hip, built by build()) draws
200,000 random (record, legal action) cases and applies each one four ways:
per lane (every batched kernel's form; the expected result), on a
wave-uniform record with the rules inlined, on a wave-uniform record with
the rules behind __noinline__ functions (the shipped k_slot's form), and
through copies of k_slot built with the rules inlined (COUP_SLOT_INLINE).
The reproducer is built with the branch-form rules (-DCOUP_RULES_V1) and the
product's flags, which turn LLVM's SLP vectorizer off: with it, ROCm 7.2 at
-O2/-O3 gets word 3 of the record wrong after Tax / Exchange / Steal / Block
announcements in every inlined copy (an opt-bisect pins the first failing
pass to slp-vectorizer); without it every form must
agree with the per-lane rules, inlined copies and round 1's k_apply with the
history byte stored from inside the rules (apply_bytehist_*) included."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "slot_inline_repro")


def test_shipped_slot_form_matches_per_lane_rules():
    if not os.path.exists(EXE):
        pytest.fail("build/slot_inline_repro missing: run __graft_entry__.build()")
    out = subprocess.run([EXE, "200000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    variants = lines[0]["slot_variants"]
    summary = lines[-1]
    assert summary["cases"] == 200000
    assert summary["uniform_call_mismatch"] == 0  # the shipped k_slot form
    assert summary["uniform_inline_mismatch"] == 0
    # every action id was exercised
    assert all(v[0] > 0 for v in summary["by_action"].values())
    counts = {k: v["mismatch"] for k, v in variants.items()}
    print("\ninlined k_slot copies, mismatching records of 20000:", counts)
    # built without the SLP vectorizer, the inlined shapes compile right too
    assert all(c == 0 for c in counts.values()), counts


INFO_EXE = os.path.join(ROOT, "build", "info_prefix_repro")


def test_info_prefix_forms_against_the_reference_writer():
    """Round 4's second sighting: the split
    InformationStateTensor writer with its prefix words stored as uint2
    (<2 x i32>) LDS stores gave a few lanes in 1000 wrong observer bits.
    build/info_prefix_repro (tools/info_prefix_repro.hip) writes 100,000
    generated states' tensors with that first form (k_sweep_uint2, three
    block shapes) and with the shipped one (k_sweep_rows, 32-bit stores),
    against a one-thread-per-float4 reference (k_info_elems' decode).  The
    shipped form must match on every lane; the uint2 form's count is
    printed (it is not shipped: info_prefix_to_lds stores 32-bit words)."""
    if not os.path.exists(INFO_EXE):
        pytest.fail("build/info_prefix_repro missing: run __graft_entry__.build()")
    out = subprocess.run([INFO_EXE, "100000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = {d["kernel"]: d for d in (json.loads(x) for x in out.stdout.splitlines() if x.startswith("{"))}
    print("\n" + "\n".join(json.dumps(v) for v in lines.values()))
    shipped = [v for k, v in lines.items() if k.startswith("k_sweep_rows")]
    assert shipped and all(v["mismatching_lanes"] == 0 for v in shipped), shipped
    assert all(v["terminal_lanes"] > 0 for v in lines.values())  # finished games are in the sample
