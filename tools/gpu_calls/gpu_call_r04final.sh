# Round 4, final call: the tree as it ends the round -- the whole GPU suite,
# smoke(), and the driver's default bench line.
set -u
D=gpurun_out/r04final
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$D/bench.json').readline()); print(d['value'], d['roofline']['frac'], d['roofline']['kernel'], d['cpu_baseline']['value'])"
