# End-of-session check on the tree as committed (libraries rebuilt by build() in the container first):
# full GPU suite, smoke(), the driver's default bench line, the facade latency table.
set -u
D=gpurun_out/r02final4
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err || exit $?
cut -c1-400 $D/bench.json
timeout -k 10 400 python -u tools/facade_latency.py > $D/facade_latency.json 2> $D/facade.err || { tail -3 $D/facade.err; exit 1; }
