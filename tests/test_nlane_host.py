"""Host build of the N-player device rules (csrc/coup_nlane.h) against the
N-player specification (oracle/coup_nplayer.c), on the CPU.

tools/nlane_host_check.cpp compiles the same header the gfx950 kernels use
with g++ (tools/hoststub stands in for hip_runtime.h) and replays uniform
rollouts step for step: actions, step types, rewards, legal masks, every
ObservationTensor element and the final 32-byte records.  The GPU tests
then check the compiled kernels themselves (tests/test_gpu_nplayer.py)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("nlane") / "nlane_host_check")
    subprocess.check_call(
        ["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas", "-I", os.path.join(ROOT, "tools", "hoststub"),
         "-I", os.path.join(ROOT, "open_spiel_coup_amd", "csrc"), "-I", os.path.join(ROOT, "oracle"),
         os.path.join(ROOT, "tools", "nlane_host_check.cpp"), "-x", "c",
         os.path.join(ROOT, "oracle", "coup_oracle.c"), os.path.join(ROOT, "oracle", "coup_nplayer.c"),
         "-o", exe])
    return exe


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6])
@pytest.mark.parametrize("auto_reset", [0, 1])
def test_device_rules_match_spec_on_host(checker, n, auto_reset):
    out = subprocess.run([checker, str(n), str(100 + n), "64", "400", str(auto_reset)],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("OK")
