"""The A/B-variant equality tests run against the measurement build
(build/variants/libcoup_mi355x.so, -DCOUP_AB_VARIANTS: every measured and
rejected kernel variant, selected by environment variables at coup_create).
tests/test_gpu_ab_variants.py runs this directory in a child process with
COUP_LIB_PATH at that build; against the product library (which instantiates
the shipped kernels only) every test here is skipped."""
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _measurement_build():
    try:
        from open_spiel_coup_amd import _native
        return bool(_native.load().coup_build_flags() & _native.BUILD_AB_VARIANTS)
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    mine = [it for it in items if str(it.fspath).startswith(HERE)]
    if mine and not _measurement_build():
        skip = pytest.mark.skip(reason="A/B variants: run by tests/test_gpu_ab_variants.py against the measurement "
                                       "build (COUP_LIB_PATH=build/variants/libcoup_mi355x.so)")
        for it in mine:
            it.add_marker(skip)
