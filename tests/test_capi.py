"""CPU-side checks of the C-ABI boundary: the library builds, loads and
exports every entry point include/coup_mi355x.h declares; host-side format
helpers agree with the oracle's canonical packing."""
import ctypes
import os
import re

import numpy as np
import pytest

from open_spiel_coup_amd import _native, build, packed
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    with open(os.path.join(ROOT, "include", "coup_mi355x.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|size_t|const char\*)\s+(coup_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    build.build()
    lib = ctypes.CDLL(_native.LIB_PATH)
    declared = _declared_functions()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(_native.SYMBOLS) == declared


def test_abi_version_and_error_plumbing():
    L = _native.load()
    assert L.coup_abi_version() == _native.ABI_VERSION
    rc = L.coup_create(-5, 0, 0, 1, ctypes.byref(ctypes.c_void_p()))
    assert rc == _native.COUP_E_INVALID
    assert b"batch" in L.coup_last_error()
    assert L.coup_destroy(None) == _native.COUP_E_INVALID
    with pytest.raises(_native.CoupError):
        _native.check(rc)


def test_create_ex_validates_players_and_flags():
    """Argument errors are reported before any HIP call (no GPU needed)."""
    L = _native.load()
    h = ctypes.c_void_p()
    for players in (0, 1, 7):
        assert L.coup_create_ex(16, 0, 0, 1, players, ctypes.byref(h)) == _native.COUP_E_INVALID
        assert b"num_players" in L.coup_last_error()
    # no N-player history / InformationStateTensor
    assert L.coup_create_ex(16, 0, 0, _native.FLAG_HISTORY, 3, ctypes.byref(h)) == _native.COUP_E_INVALID
    assert L.coup_create_ex(16, 0, 0, _native.FLAG_HISTORY | _native.FLAG_GENERIC, 2,
                            ctypes.byref(h)) == _native.COUP_E_INVALID
    assert L.coup_create_ex(16, 0, 0, 64, 2, ctypes.byref(h)) == _native.COUP_E_INVALID
    # the reference's unchecked ApplyAction is the 2-player engine's
    assert L.coup_create_ex(16, 0, 0, _native.FLAG_UNCHECKED, 3, ctypes.byref(h)) == _native.COUP_E_INVALID
    assert b"UNCHECKED" in L.coup_last_error()
    assert L.coup_create_ex(16, 0, 0, _native.FLAG_UNCHECKED | _native.FLAG_GENERIC, 2,
                            ctypes.byref(h)) == _native.COUP_E_INVALID
    assert not h.value
    assert L.coup_num_players(None) == -1 and L.coup_state_bytes(None) == -1


def test_store_sweep_validates_before_launching():
    """coup_measure_store_sweep refuses unknown mode bits, a product build's
    resident form and shapes outside the build before any HIP call."""
    L = _native.load()
    fake = ctypes.c_void_p(4096)  # never dereferenced: every call below fails first
    assert L.coup_measure_store_sweep(fake, 64, 512, 2, 4, None) == _native.COUP_E_INVALID
    assert b"mode" in L.coup_last_error()
    assert L.coup_measure_store_sweep(None, 64, 512, 2, 0, None) == _native.COUP_E_INVALID
    assert L.coup_measure_store_sweep(fake, 64, 384, 2, 0, None) == _native.COUP_E_INVALID
    assert b"shape" in L.coup_last_error()
    assert L.coup_measure_store_sweep(fake, 0, 512, 2, _native.SWEEP_INDEX_BITS, None) == _native.COUP_OK
    if not L.coup_build_flags() & _native.BUILD_AB_VARIANTS:
        assert L.coup_measure_store_sweep(fake, 64, 512, 2, _native.SWEEP_RESIDENT, None) == _native.COUP_E_INVALID
        assert b"measurement build" in L.coup_last_error()


def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    L = _native.load()
    h = ctypes.c_void_p()
    rc = L.coup_create(16, 0, 0, 1, ctypes.byref(h))
    assert rc == _native.COUP_E_HIP and not h.value


def test_packed_decode_matches_oracle_fields():
    out = oracle.rollout(seed=3, n=256, steps=37, auto_reset=True)
    words = out["final_state"]
    d = packed.decode(words)
    # replay lane 5 on the oracle object and compare decoded fields
    for lane in (0, 5, 255):
        r = packed.lane(words, lane)
        assert sum(r["deck"]) + len(r["cards"][0]) + len(r["cards"][1]) == 15
        assert r["move_player"] in (0, 1) and r["queue_len"] == 0
    assert np.all(d["coins"] <= 12)
    assert np.all(np.abs(d["reward0"]) <= 2)


def test_packed_roundtrip_of_initial_state():
    st = oracle.OracleState()
    w = np.array([st.pack()], np.uint32)
    r = packed.lane(w)
    assert r["cards"] == [[], []]
    assert r["deck"] == [3, 3, 3, 3, 3]
    assert r["coins"] == [1, 2]
    assert r["last_action"] == [-1, -1]
    assert r["queue"] == [0, 1, 0, 1]
    assert r["turn_begin"] == 1 and r["move_number"] == 0


def test_slot_result_layout_matches_header(tmp_path):
    """The Python view of coup_slot_result (pyspiel._SLOT_RESULT) has the C
    struct's field offsets and size (gcc offsetof on include/coup_mi355x.h)."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    from open_spiel_coup_amd import pyspiel
    src = tmp_path / "layout.c"
    fields = ["record", "history", "legal_mask", "cur_player", "terminal", "ok", "unrepresentable", "rewards", "returns",
              "pad"]
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "coup_mi355x.h"\nint main(void) {\n'
                   + "".join(f'  printf("{f} %zu\\n", offsetof(coup_slot_result, {f}));\n' for f in fields)
                   + '  printf("size %zu\\n", sizeof(coup_slot_result));\n  return 0;\n}\n')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = dict(line.split() for line in subprocess.check_output([str(exe)], text=True).splitlines())
    dt = pyspiel._SLOT_RESULT
    for f in fields:
        assert int(got[f]) == dt.fields[f][1], f
    assert int(got["size"]) == dt.itemsize == _native.SLOT_RESULT_BYTES


def test_episode_counter_is_28_bits_in_the_record():
    """The 2-player record keeps a 28-bit episode (w3 [31:7] + w2 [31:29]):
    the oracle's packing and the host decoder agree up to 2^28 - 1 and the
    other fields are untouched."""
    st = oracle.OracleState()
    for a in (0, 1, 2, 3, 0):
        st.apply_action(a)
    base = packed.lane(np.array([st.pack(0)], np.uint32))
    for ep in (1, (1 << 25) - 1, 1 << 25, (1 << 28) - 1):
        r = packed.lane(np.array([st.pack(ep)], np.uint32))
        assert r["episode"] == ep
        assert {k: v for k, v in r.items() if k != "episode"} == {k: v for k, v in base.items() if k != "episode"}


def test_device_builds_turn_the_slp_vectorizer_off(monkeypatch):
    """Every device compile of the product (and the section-12 reproducer the
    GPU suite runs) carries -fno-slp-vectorize: with LLVM's SLP vectorizer,
    ROCm 7.2 miscompiles the packed-record rules in several code shapes
    (DESIGN.md section 12).  The commands are inspected, nothing is built."""
    from open_spiel_coup_amd import build as b
    cmds = []
    monkeypatch.setattr(b, "_run_all", lambda jobs, verbose=False: cmds.extend(jobs))
    monkeypatch.setattr(b, "up_to_date", lambda *a, **k: False)
    monkeypatch.setattr(b.subprocess, "check_call", lambda cmd, *a, **k: cmds.append(cmd))
    b.build(force=True, repro=True)
    device = [c for c in cmds if c[0] == b.HIPCC and any(str(x).endswith(".hip") for x in c)]
    assert len(device) == 6  # the two product sources, their measurement build and the two reproducers
    assert all(b.NO_SLP in c for c in device)
    assert b.NO_SLP in b.command() and b.NO_SLP in b.repro_command() and b.NO_SLP in b.info_repro_command()


# The kernels the product library ships: the A/B
# variants measured and rejected in rounds 1-4 live in the measurement
# build only (build/variants/, -DCOUP_AB_VARIANTS; csrc/coup_knobs.h).
_SHIPPED_2P = """
coup::k_info_elems coup::k_measure_traffic coup::k_obs_lanes coup::k_reset coup::k_rollout coup::k_server
coup::k_step_trajectory coup::np::k_export coup::np::k_import |
void coup::k_apply<false> | void coup::k_apply<true> | void coup::k_info_sweep<1024, 2, 0> |
void coup::k_obs_sweep_rows<512, 2, 0, 0> | void coup::k_query<false, false> | void coup::k_query<false, true> |
void coup::k_query<true, false> | void coup::k_query<true, true> | void coup::k_rollout_sorted<1024> |
void coup::k_slot<false> | void coup::k_slot<true> | void coup::k_slot_batch<false> | void coup::k_slot_batch<true> |
void coup::k_step<false, 0, 256, 0, true> | void coup::k_step<false, 0, 256, 1, false> |
void coup::k_step<false, 0, 256, 1, true> | void coup::k_step<false, 0, 256, 2, false> |
void coup::k_step<false, 0, 256, 2, true> | void coup::k_step<false, 4, 256, 1, false> |
void coup::k_step<false, 4, 256, 1, true> | void coup::k_step<false, 4, 256, 2, false> |
void coup::k_step<false, 4, 256, 2, true> | void coup::k_step<false, 9, 256, 0, false> |
void coup::k_step<false, 9, 256, 0, true> | void coup::k_step<true, 0, 256, 1, false> |
void coup::k_step<true, 0, 256, 2, false> | void coup::k_step<true, 4, 256, 1, false> |
void coup::k_step<true, 4, 256, 2, false> | void coup::k_step<true, 9, 256, 0, false> |
void coup::k_step_group<1, false> | void coup::k_step_group<1, true> |
void coup::k_step_sorted<false, 512> | void coup::k_step_sorted<true, 512> |
void coup::k_trajectory_sorted<1024, false, false, 8, 0, false> |
void coup::k_trajectory_sorted<1024, true, false, 8, 0, false> |
void coup::k_trajectory_sorted<1024, true, false, 8, 0, true> |
void coup::k_store_sweep<512, 2> | void coup::k_store_sweep<1024, 2>
"""


def _shipped_kernels():
    words = _SHIPPED_2P.split("|")
    names = set()
    for w in words:
        w = " ".join(w.split())
        if w.startswith("coup::"):  # the plain (non-template) kernels
            names.update(w.split())
        elif w:
            names.add(w)
    for n in range(2, 7):
        tb = 1024 if n >= 6 else 512
        names.update(f"void coup::np::{k}<{n}>" for k in ("k_apply", "k_obs", "k_query", "k_reset", "k_rollout",
                                                          "k_step_trajectory"))
        names.update({f"void coup::np::k_step<{n}, false>", f"void coup::np::k_step<{n}, true>",
                      f"void coup::np::k_rollout_sorted<{n}, 1024, true>",
                      f"void coup::np::k_trajectory_sorted<{n}, 1024, 1>",
                      f"void coup::np::k_step_sorted<{n}, false, false, {tb}, false, 4>",
                      f"void coup::np::k_step_sorted<{n}, true, true, {tb}, false, 4>"})
    return names


def _kernel_handles(path):
    """Kernel handle symbols of a HIP library (the host-side stubs the
    runtime registers, one per instantiated __global__), demangled without
    their parameter lists."""
    import subprocess
    out = subprocess.run(["nm", path], capture_output=True, text=True, check=True).stdout
    mangled = [ln.split()[2] for ln in out.splitlines()
               if len(ln.split()) == 3 and ln.split()[1] in "DV" and re.match(r"_ZN4coup(2np)?\d+k_", ln.split()[2])]
    dem = subprocess.run(["c++filt"], input="\n".join(mangled), capture_output=True, text=True, check=True).stdout
    return {ln.split("(")[0] for ln in dem.splitlines() if ln}


def test_product_library_ships_only_the_shipped_kernels():
    build.build()
    got = _kernel_handles(_native.LIB_PATH)
    want = _shipped_kernels()
    assert got == want, {"unexpected": sorted(got - want), "missing": sorted(want - got)}
    lib = ctypes.CDLL(_native.LIB_PATH)
    # the product: no variants, the rules trajectories' outputs stored by the playing thread (0)
    assert lib.coup_build_flags() == 0


def test_measurement_build_holds_the_variants():
    """build() also writes the A/B-variant build; it holds every shipped
    kernel and the rejected ones (a sample named here)."""
    build.build()
    got = _kernel_handles(build.VARIANTS_OUT)
    assert _shipped_kernels() <= got
    for k in ("void coup::k_obs_sweep<1>", "void coup::k_obs_sweep_rows<256, 2, 0, 0>", "void coup::k_step_group<4, true>",
              "void coup::k_step<true, 1, 256, 0, false>", "void coup::k_step_sorted<true, 1024>",
              "void coup::k_info_sweep<512, 2, 0>", "void coup::k_step_obs_pipe<512, 2>",
              "void coup::k_trajectory_sorted<1024, false, true, 4, 0, false>",
              "void coup::k_trajectory_sorted<1024, true, false, 8, 1, false>", "void coup::k_obs_sweep_nib<512, 2>",
              "void coup::np::k_step_sorted<6, true, true, 1024, true, 4>",
              "void coup::np::k_rollout_sorted<6, 1024, false>", "void coup::np::k_trajectory_sorted<6, 1024, 0>"):
        assert k in got, k
    lib = ctypes.CDLL(build.VARIANTS_OUT)
    lib.coup_build_flags.restype = ctypes.c_int
    assert lib.coup_build_flags() == _native.BUILD_AB_VARIANTS
