# Round 6: the shipped tree (packed-record carry, two barriers per step,
# playing-thread stores): the whole GPU suite, smoke(), the driver's default line.
set -u
. tools/gpu_calls/attempt.sh r06p
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_default.json')); r=d['roofline']; print('c3', d['value'], r['frac'], r['kernel_ms'], r['kernel'] == r['kernel_launched'])"
