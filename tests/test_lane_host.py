"""The 2-player device rules (open_spiel_coup_amd/csrc/coup_lane.h) compiled
for the host with g++ under UBSan (tools/hoststub stands in for
hip_runtime.h) and walked against the oracle: random legal actions,
decisions and chance outcomes, every record compared after every action
(tools/lane_ubsan_walk.cpp).  Both forms of the decision transition: the
effect form the rules-bound kernels use (apply_decision_v2, default) and the
reference-shaped branches the store-bound kernels use (-DCOUP_RULES_V1).
The unchecked walk applies any action id through apply_action_unchecked (the
per-game ops' path: pyspiel's apply_action has no legality check) against
oc_apply_action_unchecked: accepted / rejected and every record agree."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("form", ["effect", "branches", "unchecked"])
def test_lane_rules_walk_matches_oracle_under_ubsan(tmp_path, form):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "walk")
    cmd = ["g++", "-O1", "-g", "-fsanitize=undefined", "-fno-sanitize-recover=all", "-I",
           os.path.join(ROOT, "tools", "hoststub"), "-I", os.path.join(ROOT, "open_spiel_coup_amd", "csrc"), "-I",
           os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools", "lane_ubsan_walk.cpp"),
           os.path.join(ROOT, "oracle", "coup_oracle.c"), "-o", exe]
    if form == "branches":
        cmd.insert(1, "-DCOUP_RULES_V1")
    subprocess.check_call(cmd)
    out = subprocess.run([exe, "4000"] + (["unchecked"] if form == "unchecked" else []), capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok 4000 games")
