# Final round-2 profiles, part B: c4, c4r (100 fused steps), c3i.
set -u
bash tools/profile_gpu.sh r02 c4 --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof_r02_c4.log 2>&1 || { tail -5 gpurun_out/prof_r02_c4.log; exit 1; }
bash tools/profile_gpu.sh r02 c3i --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof_r02_c3i.log 2>&1 || { tail -5 gpurun_out/prof_r02_c3i.log; exit 1; }
bash tools/profile_gpu.sh r02 c4r --gpus 1 --steps 100 --warmup 5 > gpurun_out/prof_r02_c4r.log 2>&1 || { tail -5 gpurun_out/prof_r02_c4r.log; exit 1; }
for c in c4 c3i c4r; do grep -h '"bench_vs_rocprof_kernel_ms"\|rocprof_minus_bench_pct' -A0 gpurun_out/prof_r02_$c.log | head -3; done
