"""rl_environment._float_lists (the library's CPython binding,
_coup_host.float_lists): the time steps' per-player lists equal numpy's
tolist of the same float32 rows element by element -- one-hots, coin counts,
and any other value (fractions, negative zero, large values) -- each call
returns new lists the caller owns, and the lists of floats stay out of the
cyclic garbage collector (rl_environment.py:243-248 hands out fresh lists)."""
import gc
import math

import numpy as np
import pytest


def _lists():
    try:
        from open_spiel_coup_amd.rl_environment import _float_lists
        _float_lists(np.zeros((1, 1), np.float32))
    except (ImportError, OSError) as e:
        pytest.skip(f"library / binding not built: {e}")
    return _float_lists


def test_float_lists_equal_tolist():
    fl = _lists()
    rng = np.random.default_rng(7)
    for _ in range(50):
        rows = (rng.random((2, 2492)) < 0.02).astype(np.float32)
        rows[:, 60:62] = rng.integers(0, 16, size=(2, 2))
        got = fl(rows)
        assert got == rows.tolist()
        assert all(type(v) is float for v in got[0][:100])
    odd = np.array([[0.0, -0.0, 1.5, 15.0, 16.0, -1.0, 1e30, 3.0]], np.float32)
    got = fl(odd)[0]
    assert got == odd[0].tolist()
    assert math.copysign(1.0, got[1]) == -1.0  # -0.0 keeps its sign


def test_float_lists_are_fresh_and_untracked():
    fl = _lists()
    rows = np.eye(2, 98, dtype=np.float32)
    a, b = fl(rows), fl(rows)
    assert a == b and a[0] is not b[0]
    a[0][0] = "caller's"
    assert b[0][0] == 1.0 and fl(rows)[0][0] == 1.0
    assert not gc.is_tracked(b[0]) and gc.is_tracked(b)  # the outer list is an ordinary one


def test_state_tensor_rows_stay_tracked():
    """pyspiel State tensors are ordinary lists: untrack = 0
    keeps them in the cyclic collector, equal to tolist."""
    from open_spiel_coup_amd import _coup_host
    rows = np.eye(1, 98, dtype=np.float32)
    t = _coup_host.float_lists(rows, 1, 98, 0)[0]
    assert gc.is_tracked(t) and t == rows[0].tolist()


def test_float_lists_of_non_contiguous_input():
    fl = _lists()
    big = np.arange(4 * 10, dtype=np.float32).reshape(4, 10)
    assert fl(big[::2]) == big[::2].tolist()


def test_float_lists_reference_counts():
    """The shared zeros' references are counted in bulk (per column copy,
    added once per row): building then freeing lists leaves every shared
    float's count where it was, and a live list holds exactly one reference
    per element (columns 0, 8, 16, ... share copy 0)."""
    import sys
    fl = _lists()
    z = np.zeros((2, 1003), np.float32)
    z[1, 5] = 1.0
    probe_lists = fl(z)
    zero0, one5 = probe_lists[0][0], probe_lists[1][5]
    base0, base1 = sys.getrefcount(zero0), sys.getrefcount(one5)
    for _ in range(5):
        x = fl(z)
        del x
    assert sys.getrefcount(zero0) == base0 and sys.getrefcount(one5) == base1
    x = fl(z)
    assert sys.getrefcount(zero0) == base0 + 2 * len(range(0, 1003, 8))
    assert sys.getrefcount(one5) == base1 + 1
    del x
    assert sys.getrefcount(zero0) == base0
