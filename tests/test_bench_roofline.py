"""bench.py's roofline object on the CPU: the VALU issue
fraction of the tensor-free trajectory forms, the bound it selects, no field
named a ceiling, and the kernel-name mirror (expected_kernel) for every
config at its default batch."""
import json
import os

import pytest

import bench


def _fields(**kw):
    base = dict(kernel="k", launched="k", achieved=500.0, traffic=None, valu_insts=None, launch_ms=0.1,
                bytes_per_launch=50_000_000, box={"sclk": "1: 2400Mhz"}, sweep_ms=None, sweep_form=None,
                step_form="fused")
    base.update(kw)
    return bench.roofline_fields(**base)


def test_valu_issue_fraction_and_bound():
    # c4's profile (profiles/r05/c4/summary.json): 272.8e6 VALU instructions in a 510 us launch
    r = _fields(valu_insts=272.8e6, launch_ms=0.510, achieved=4440.0)
    assert r["valu_issue_frac"] == pytest.approx(272.8e6 * 4 / (1024 * 2.4e9 * 0.510e-3))
    assert 0.85 < r["valu_issue_frac"] < 0.9 and r["bound"] == "valu"
    # a tensor-writing step stays HBM-bound whatever its VALU share (call r06d)
    r = _fields(valu_insts=71.08e6, launch_ms=0.1331, achieved=6490.0, tensors=True)
    assert r["valu_issue_frac"] > r["frac"] and r["bound"] == "hbm"
    # without a profile of the same form: no VALU fraction, the HBM bound
    r = _fields(valu_insts=None, achieved=6400.0)
    assert r["valu_issue_frac"] is None and r["bound"] == "hbm" and r["frac"] == pytest.approx(0.8)
    # at the peak gfx clock, whatever the box's clock read afterwards
    r = _fields(valu_insts=1e6, launch_ms=1.0, box={"sclk": "1: 2000Mhz"})
    assert r["valu_issue_frac"] == pytest.approx(4e6 / (1024 * 2.4e9 * 1e-3))


def test_no_field_is_a_ceiling():
    """The store-only sweep runs slower than the split writers (DESIGN.md
    section 5): it is reported as a measurement, never as a ceiling, so no
    field named like one can exceed 1.0 of anything."""
    r = _fields(sweep_ms=0.1365, sweep_form="sweep", launch_ms=0.1347)
    assert not any("ceiling" in k for k in r)
    assert r["sweep_over_kernel"] > 1.0 and r["store_sweep_note"]
    # every fraction the object reports is a bound's fraction, <= 1 by construction for real inputs
    for k, v in r.items():
        if k.endswith("frac") and v is not None:
            assert 0.0 <= v


def test_traffic_table_carries_valu_for_the_trajectory_forms():
    with open(bench.TRAFFIC_FILE) as f:
        t = json.load(f)
    for cfg in ("c2", "c4"):
        assert t[cfg]["valu_insts_per_launch"] > 0 and t[cfg]["steps_per_launch"] == 20, cfg


@pytest.mark.parametrize("cfg,want", [
    ("c3", "coup::k_trajectory_sorted<1024, true, false, 8, 0, true> + coup::k_obs_sweep_rows<512, 2>"),
    ("c2", "coup::k_step_trajectory"),
    ("c4", "coup::np::k_trajectory_sorted<6, 1024>"),
    ("c2r", "coup::k_rollout"),
    ("c4r", "coup::np::k_rollout_sorted<6, 1024>"),
    ("c2t", "coup::k_step_trajectory"),
    ("c4t", "coup::np::k_trajectory_sorted<6, 1024>"),
])
def test_expected_kernel_names(monkeypatch, cfg, want):
    """The mirror of the library's dispatch at each config's default batch
    and graph setting (the driver's command); the GPU tests hold the
    library's own launch log to the same strings."""
    for k in ("COUP_PIPE", "COUP_REGROUP", "COUP_OBS_SPLIT", "COUP_MANY_STAGE", "COUP_AHEAD", "COUP_STEP_TPL",
              "COUP_TRAJ_CHUNK"):
        monkeypatch.delenv(k, raising=False)
    # obs_split_active / info_split_active ask the library (it only reads knobs; no GPU)
    if not os.path.exists(os.path.join(bench.ROOT, "open_spiel_coup_amd", "libcoup_mi355x.so")):
        pytest.skip("library not built")
    B = bench.CONFIGS[cfg][0]
    assert bench.expected_kernel(cfg, B, cfg in bench.GRAPH_AUTO) == want
