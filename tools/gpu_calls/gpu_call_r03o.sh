# Round 3, fresh container: the whole GPU suite and smoke() on the current
# tree, the driver's default bench line, then the c3 profile with the bench command.
set -u
D=gpurun_out/r03o
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { tail -5 $D/bench_default.err; exit 1; }
cut -c1-300 $D/bench_default.json
timeout -k 10 900 bash tools/profile_gpu.sh r03 c3 --gpus 1 --steps 20 --warmup 5 > $D/prof_c3.log 2>&1 || { tail -20 $D/prof_c3.log; exit 1; }
grep -E "kernel_ms|rocprof_minus|rocprof_mean|timed_kernel|fetch|write" $D/prof_c3.log | head
