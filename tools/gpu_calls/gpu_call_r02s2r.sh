# Round 2, session 2: smoke() with the trajectory and skip checks, then the c3 profile of the final tree
# (trace + FETCH/WRITE/SQ passes of the driver's bench command, bench lines before/after on the same lease).
set -u
mkdir -p gpurun_out/r02s2r
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02s2r/smoke.log 2>&1 || { tail -20 gpurun_out/r02s2r/smoke.log; exit 1; }
tail -1 gpurun_out/r02s2r/smoke.log
bash tools/profile_gpu.sh r02 c3 --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof_r02_c3.log 2>&1 || { tail -5 gpurun_out/prof_r02_c3.log; exit 1; }
grep -h '"bench_vs_rocprof_kernel_ms"\|rocprof_minus_bench_pct' -A0 gpurun_out/prof_r02_c3.log | head -3
