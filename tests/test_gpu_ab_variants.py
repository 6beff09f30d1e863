"""The A/B-variant equality suite (tests/ab_variants/) against the
measurement build.  The product library instantiates the shipped kernels
only; every variant that was measured and rejected
 lives in build/variants/libcoup_mi355x.so
(-DCOUP_AB_VARIANTS), which build() writes beside it.  Its tests load that
library through COUP_LIB_PATH, so they run in ONE child pytest process --
the library is loaded once per process -- whose progress goes to
gpurun_out/ab_variants.log line by line."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_variant_suite_against_the_measurement_build():
    from open_spiel_coup_amd import build
    lib = build.VARIANTS_OUT
    assert os.path.exists(lib), f"{lib} missing: build() writes the measurement build"
    log_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(log_dir, exist_ok=True)
    log = os.path.join(log_dir, "ab_variants.log")
    env = dict(os.environ, COUP_LIB_PATH=lib)
    with open(log, "w") as f:
        r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-v", "-p", "no:cacheprovider", "-m", "gpu",
                            os.path.join(ROOT, "tests", "ab_variants")], env=env, cwd=ROOT, stdout=f,
                           stderr=subprocess.STDOUT, timeout=1800)
    with open(log) as f:
        text = f.read()
    assert r.returncode == 0, text[-6000:]
    assert " passed" in text and " skipped" not in text.splitlines()[-1], text[-2000:]
