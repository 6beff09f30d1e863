"""bench.py's own argument edges on the GPU (warm-up + K near the
packed int16 episode word's 63-step reserve; the power warm-up's and the
gate calibration's untimed steps cleared before the timed window): each run
prints one line with no lane errors and finished episodes, its power_warm
and gate fields as asked."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line(args):
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--no-cpu-baseline"] + args,
                       capture_output=True, text=True, timeout=170, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["lane_errors"] == 0 and rec["episodes"]["finished"] > 0
    return rec


@pytest.mark.parametrize("config,args", [
    ("c3", ["--batch", "65536", "--steps", "60", "--warmup", "12"]),   # int16 word, 60 of its 63 steps
    ("c3", ["--batch", "65536", "--steps", "70", "--warmup", "3"]),    # int32 word past 63
    ("c4", ["--batch", "16384", "--steps", "20", "--warmup", "20"]),
    ("c2", ["--batch", "16384", "--steps", "20", "--warmup", "5", "--gate-steps", "3"]),
    ("c3i", ["--batch", "4096", "--steps", "8", "--warmup", "2"]),
])
def test_bench_argument_edges(config, args):
    rec = _line(["--config", config] + args)
    assert rec["power_warm"]["steps"] > 0  # the default 40 ms warm-up ran
    if "--gate-steps" in args:
        assert rec["config"]["gate_steps"] == int(args[args.index("--gate-steps") + 1])


def test_bench_without_power_warm_or_gate():
    rec = _line(["--config", "c2", "--batch", "16384", "--power-warm-ms", "0", "--gate-steps", "0"])
    assert rec["power_warm"] == {"steps": 0, "ms": 0.0} and rec["config"]["gate_steps"] == 0
