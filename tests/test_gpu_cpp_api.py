"""The C++ host layer (include/coup_mi355x.hpp: CoupGame / CoupState /
BatchedEnv over the C ABI) against the reference's golden transcript.

tests/cpp/state_driver.cpp replays coup.txt's history through
coup_amd::LoadGame("coup")->NewInitialState() and prints every State
accessor; the CPU test only builds it, the GPU test runs it."""
import json
import os
import shutil
import subprocess

import pytest

from tests import golden_util as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PT = G.load_playthrough()["states"]


def build_driver(out_dir):
    from open_spiel_coup_amd import build
    lib = build.build()
    exe = os.path.join(out_dir, "state_driver")
    cxx = shutil.which("g++")
    subprocess.check_call(
        [cxx, "-O2", "-std=c++17", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROOT, "include"),
         "-I", "/opt/rocm/include", os.path.join(ROOT, "tests", "cpp", "state_driver.cpp"), "-o", exe,
         "-L", os.path.dirname(lib), "-lcoup_mi355x", "-L", "/opt/rocm/lib", "-lamdhip64",
         "-Wl,-rpath," + os.path.dirname(lib) + ":/opt/rocm/lib"])
    return exe


@pytest.fixture(autouse=True, params=["host", "device"])
def state_mode(request, monkeypatch):
    """The C++ layer's States host-resident (default) or on device lanes
    (COUP_STATE_DEVICE=1), for the driver processes this module starts."""
    monkeypatch.setenv("COUP_STATE_DEVICE", "1" if request.param == "device" else "0")
    return request.param


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"):
        pytest.skip("g++ / ROCm headers not available")
    return build_driver(str(tmp_path_factory.mktemp("cppapi")))


def test_cpp_layer_builds(driver):
    assert os.path.exists(driver)


@pytest.mark.gpu
def test_cpp_state_playthrough(driver):
    hist = PT[-1]["history"]
    out = subprocess.run([driver] + [str(a) for a in hist], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    got = [json.loads(line) for line in out.stdout.splitlines()]
    assert len(got) == len(PT)
    for rec, g in zip(PT, got):
        assert g["history"] == rec["history"]
        assert g["serialize"] == "".join(f"{a}\n" for a in rec["history"])
        if "to_string" in rec:
            assert G.rstrip_lines(g["to_string"]) == rec["to_string"]
        if "current_player" not in rec:
            continue
        assert g["current_player"] == rec["current_player"]
        assert g["is_terminal"] == rec["is_terminal"] and g["is_chance"] == rec["is_chance"]
        if not rec["is_terminal"]:
            assert g["legal_actions"] == rec["legal_actions"]
        if rec["is_chance"]:
            assert [tuple(x) for x in g["chance_outcomes"]] == [tuple(x) for x in rec["chance_outcomes"]]
        else:
            assert g["rewards"] == [int(x) for x in rec["rewards"]]
            assert g["returns"] == [int(x) for x in rec["returns"]]
        for p in ("0", "1"):
            assert g["obs" + p] == [[int(k), int(v)] for k, v in rec["ObservationTensor"][p]]
            assert g["info" + p] == [[int(k), int(v)] for k, v in rec["InformationStateTensor"][p]]
            assert g["obs_str" + p] == rec["ObservationString"][p]
            assert g["info_str" + p] == rec["InformationStateString"][p]


@pytest.mark.gpu
def test_cpp_state_errors_clone_child(driver):
    out = subprocess.run([driver, "--illegal"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    r = json.loads(out.stdout)
    assert r["illegal"] == "rejected"
    assert r["history"] == [4, 3, 2, 0] and r["clone"] == [4, 3, 2, 0]
    assert r["child"] == [4, 3, 2, 0, 0] and r["roundtrip"] == [4, 3, 2, 0, 0]


@pytest.mark.gpu
def test_cpp_unchecked_apply_action(driver):
    """ApplyAction has the reference's semantics (no legality check,
    spiel.cc:322-331): the Tax answered by Block of policy_analysis.py
    applies, ApplyActionWithLegalityCheck refuses it; equal to the oracle."""
    from oracle import oracle
    out = subprocess.run([driver, "--unchecked"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    r = json.loads(out.stdout)
    st = oracle.OracleState()
    for a in [1, 1, 3, 3, 3, 10, 9]:
        st.apply_action_unchecked(a)
    assert r["checked_threw"] is True
    assert r["history"] == [1, 1, 3, 3, 3, 10] and r["child"] == [1, 1, 3, 3, 3, 10, 9]
    assert r["child_player"] == st.current_player() and r["child_legal"] == st.legal_actions()


@pytest.mark.gpu
def test_cpp_batched_children_equal_child(driver):
    """coup_amd::CoupState::Children (one coup_slot_ops launch for all legal
    actions) == Child(a) one by one, along six random games."""
    out = subprocess.run([driver, "--children"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert json.loads(out.stdout)["children_checked"] > 100
