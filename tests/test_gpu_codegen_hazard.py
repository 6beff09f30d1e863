"""The code-generation hazard of DESIGN.md section 12, kept under watch.

build/slot_inline_repro (tools/slot_inline_repro.hip, built by build()) draws
200,000 random (record, legal action) cases and applies each one four ways:
per lane (every batched kernel's form; the expected result), on a
wave-uniform record with the rules inlined, on a wave-uniform record with
the rules behind __noinline__ functions (the shipped k_slot's form), and
through copies of k_slot built with the rules inlined (COUP_SLOT_INLINE).
The shipped form must agree with the per-lane form on every case; the
inlined k_slot copies are reported (ROCm 7.2 at -O2/-O3 gets word 3 of the
record wrong after Tax / Exchange / Steal / Block announcements).  The
reproducer is built with the branch-form rules (-DCOUP_RULES_V1), the form
that triggers it; it also reports round 1's k_apply with the history byte
stored from inside the rules (apply_bytehist_*)."""
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
    print("\ninlined k_slot copies, mismatching records of 20000:",
          {k: v["mismatch"] for k, v in variants.items()})
