# Final round-2 profiles, part A: c3 (the driver's exact command), c2, c2r (100 fused steps).
set -u
bash tools/profile_gpu.sh r02 c3 --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof_r02_c3.log 2>&1 || { tail -5 gpurun_out/prof_r02_c3.log; exit 1; }
bash tools/profile_gpu.sh r02 c2 --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof_r02_c2.log 2>&1 || { tail -5 gpurun_out/prof_r02_c2.log; exit 1; }
bash tools/profile_gpu.sh r02 c2r --gpus 1 --steps 100 --warmup 5 > gpurun_out/prof_r02_c2r.log 2>&1 || { tail -5 gpurun_out/prof_r02_c2r.log; exit 1; }
for c in c3 c2 c2r; do grep -h '"bench_vs_rocprof_kernel_ms"\|rocprof_minus_bench_pct' -A0 gpurun_out/prof_r02_$c.log | head -3; done
