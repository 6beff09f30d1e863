# Session-2 re-entry check: the tree rebuilt in a fresh container by build(); full GPU suite, smoke(), default bench line.
set -u
mkdir -p gpurun_out/r02s2a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r02s2a/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r02s2a/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r02s2a/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02s2a/smoke.log 2>&1 || { tail -20 gpurun_out/r02s2a/smoke.log; exit 1; }
tail -1 gpurun_out/r02s2a/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r02s2a/bench.json 2> gpurun_out/r02s2a/bench.err || exit $?
cut -c1-400 gpurun_out/r02s2a/bench.json
