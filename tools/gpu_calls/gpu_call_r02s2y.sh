# Round 2, session 2: final-tree profile of the c4 step (known decision nodes), driver-style K = 20.
set -u
bash tools/profile_gpu.sh r02 c4 --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof_r02_c4.log 2>&1 || { tail -5 gpurun_out/prof_r02_c4.log; exit 1; }
grep -h '"bench_vs_rocprof_kernel_ms"\|rocprof_minus_bench_pct' -A0 gpurun_out/prof_r02_c4.log | head -3
