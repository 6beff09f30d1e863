# Round 4, twenty-third call: the split InformationStateTensor step as the
# default from 2^18 lanes -- the whole GPU suite, smoke(), the driver's
# default bench line, the c3i line and its profile.
set -u
D=gpurun_out/r04w
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
cut -c1-200 $D/bench.json
bash tools/profile_gpu.sh r04 c3i > $D/profile_c3i.log 2>&1 || { tail -30 $D/profile_c3i.log; exit 1; }
tail -3 $D/profile_c3i.log
