# Round-2 profiles of the fused-trajectory configs (c4t, c2t: 100 steps per launch) with the bench line before/after.
set -u
bash tools/profile_gpu.sh r02 c4t --gpus 1 --steps 100 --warmup 5 > gpurun_out/prof_r02_c4t.log 2>&1 || { tail -5 gpurun_out/prof_r02_c4t.log; exit 1; }
bash tools/profile_gpu.sh r02 c2t --gpus 1 --steps 100 --warmup 5 > gpurun_out/prof_r02_c2t.log 2>&1 || { tail -5 gpurun_out/prof_r02_c2t.log; exit 1; }
for c in c4t c2t; do grep -h '"bench_vs_rocprof_kernel_ms"\|rocprof_minus_bench_pct' -A0 gpurun_out/prof_r02_$c.log | head -3; done
