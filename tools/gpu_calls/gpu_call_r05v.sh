# Round 5: the whole GPU suite on the current tree (the A/B-variant suite runs
# inside it against build/variants/), smoke(), the driver's default line, and
# the c3i profile (per-kernel steady-state numbers).
set -u
D=gpurun_out/r05v
mkdir -p $D
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_default.json')); r=d['roofline']; print('c3', d['value'], r['frac'], r['kernel_ms'], r.get('store_ceiling_ms'), d['power_warm'])"
timeout -k 10 900 bash tools/profile_gpu.sh r05 c3i > gpurun_out/profile_r05_c3i.log 2>&1 || { tail -30 gpurun_out/profile_r05_c3i.log; exit 1; }
tail -2 gpurun_out/profile_r05_c3i.log
