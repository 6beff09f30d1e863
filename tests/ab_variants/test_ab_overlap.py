"""Measurement build (tests/ab_variants/conftest.py): coup_step_many's
rejected forms -- the fused trajectory writing the observations itself
(COUP_PIPE=4, COUP_FUSED_SHAPE) and the overlapped rules-trajectory form (COUP_PIPE=3: the rules trajectory of chunk
c + 1 on a second stream beside chunk c's writers, records double-buffered,
fork / join events; measured slower than the one-stream form, DESIGN.md
section 5), through tests/test_gpu_step_many.py's checks: equal to
coup_step launched once per step, bit for bit.  (The CU-masked stream form,
COUP_OVERLAP_CUS, was deleted in round 6: DESIGN.md section 5.)"""
import pytest
import torch

from tests import test_gpu_step_many as M

pytestmark = pytest.mark.gpu

@pytest.mark.parametrize("B", [1000, (1 << 18) + 5])
def test_overlap_equals_stepping(monkeypatch, B):
    M.test_step_many_equals_stepping(monkeypatch, B, "3")


@pytest.mark.parametrize("chunk", [1, 3])
def test_overlap_chunk_length_invariant(monkeypatch, chunk):
    M.test_chunk_length_invariant(monkeypatch, chunk, "3", None)


def test_overlap_graph_capture(monkeypatch):
    M.test_graph_capture_and_packed_word(monkeypatch, "3", 2)


def test_overlap_trajectory_slices(monkeypatch):
    M.test_trajectory_slices_every_step(monkeypatch, 1 << 20, 21, "3", None)


def test_overlap_capture_without_resources_falls_back(monkeypatch):
    """COUP_PIPE=3 switched on after coup_create (coup_reload_knobs), so the
    env's first overlapped coup_step_many is inside a graph capture, where no
    stream or buffer can be made: the call runs on the env's stream alone,
    same results; the next eager call makes them and overlaps."""
    B, seed, K = 4096, 8, 6
    many, ref = M._env(monkeypatch, B, "1", seed), M._env(monkeypatch, B, False, seed)
    monkeypatch.setenv("COUP_PIPE", "3")
    many.reload_knobs()
    g = many.capture_steps(K)
    g.replay()
    torch.cuda.synchronize()
    for _ in range(K):
        ref.step()
    M._same(M._state(many), M._state(ref), "capture fallback")
    many.step_many(5)  # eager: now with the second stream
    for _ in range(5):
        ref.step()
    M._same(M._state(many), M._state(ref), "after")


@pytest.mark.parametrize("shape", ["1", "2", "3"])
def test_fused_trajectory_shapes(monkeypatch, shape):
    """kManyFused's block / register-budget variants (COUP_FUSED_SHAPE: 512
    lanes x 4 waves per SIMD, 1024 x 8, 512 x 8) equal stepping, and their
    trajectory slices equal one coup_step per slice."""
    monkeypatch.setenv("COUP_FUSED_SHAPE", shape)
    M.test_step_many_equals_stepping(monkeypatch, 65536 + 77, "4")
    M.test_chunk_length_invariant(monkeypatch, 8, "4", None)


@pytest.mark.parametrize("B,T", [(1000, 12), (1 << 20, 10)])
def test_fused_trajectory_default_shape(monkeypatch, B, T):
    """kManyFused's default shape (1024 lanes, 4 waves per SIMD): stepping,
    graph capture and trajectory slices."""
    M.test_step_many_equals_stepping(monkeypatch, 3, "4")
    M.test_graph_capture_and_packed_word(monkeypatch, "4", 8)
    M.test_trajectory_slices_every_step(monkeypatch, B, T, "4", None)


@pytest.mark.parametrize("chunk", [1, 8, 32])
def test_staged_rules_trajectory(monkeypatch, chunk):
    """The rules trajectory with its outputs staged by lane in LDS
    (COUP_MANY_STAGE; measured slower): stepping at every chunk length, and
    trajectory slices at the bench size."""
    M.test_chunk_length_invariant(monkeypatch, chunk, "1", "1")
    if chunk == 8:
        M.test_trajectory_slices_every_step(monkeypatch, 1 << 20, 21, "1", "1")


@pytest.mark.parametrize("shape", ["1", "2", "3", "4"])
def test_rules_trajectory_shapes(monkeypatch, shape):
    """The rules trajectory's block / register-budget variants
    (COUP_MANY_SHAPE) equal stepping."""
    monkeypatch.setenv("COUP_MANY_SHAPE", shape)
    M.test_chunk_length_invariant(monkeypatch, 8, "1", None)


@pytest.mark.parametrize("pol", ["1", "2", "3"])
def test_obs_writer_store_policies(monkeypatch, pol):
    """COUP_WRITER_POL: the rules-trajectory form's k_obs_sweep_rows<512, 2>
    with plain, sc1 or sc1 nt buffer stores equals stepping (ragged batch:
    the last block's range drops the stores past it)."""
    monkeypatch.setenv("COUP_WRITER_POL", pol)
    M.test_chunk_length_invariant(monkeypatch, 8, "1", None)


@pytest.mark.parametrize("knobs", [{"COUP_WRITER_PRIO": "2"}, {"COUP_OVERLAP_LDS": "98304", "COUP_WRITER_PRIO": "1"}])
def test_overlap_priority_and_occupancy(monkeypatch, knobs):
    """The overlapped form with the writer's waves at a higher issue priority
    and the rules' blocks capped per CU by dynamic LDS equals stepping."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    M.test_chunk_length_invariant(monkeypatch, 3, "3", None)
    M.test_chunk_length_invariant(monkeypatch, 8, "1", None)


@pytest.mark.parametrize("form", ["1", "2", "3", "4"])
def test_nibble_writer_shapes(monkeypatch, form):
    """COUP_WRITER_FORM: the nibble + table observation writer
    (k_obs_sweep_nib, round 6) in the rules-trajectory form equals stepping
    at every chunk length, and (512 x 2) its trajectory slices at the bench
    size."""
    monkeypatch.setenv("COUP_WRITER_FORM", form)
    M.test_chunk_length_invariant(monkeypatch, 8, "1", None)
    if form == "1":
        M.test_trajectory_slices_every_step(monkeypatch, 1 << 20, 21, "1", None)
