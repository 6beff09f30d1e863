# Round 3: the whole GPU suite and smoke() on the current tree, then the c4 and
# c4t profiles with the bench commands (c4t outputs staged by lane).
set -u
D=gpurun_out/r03k
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 900 bash tools/profile_gpu.sh r03 c4 --gpus 1 --steps 20 --warmup 5 > $D/prof_c4.log 2>&1 || { tail -20 $D/prof_c4.log; exit 1; }
grep -E "kernel_ms|rocprof_minus|rocprof_mean|timed_kernel" $D/prof_c4.log | head
timeout -k 10 900 bash tools/profile_gpu.sh r03 c4t --gpus 1 --steps 100 --warmup 5 > $D/prof_c4t.log 2>&1 || { tail -20 $D/prof_c4t.log; exit 1; }
grep -E "kernel_ms|rocprof_minus|write_size|fetch_size|timed_kernel" $D/prof_c4t.log | head
