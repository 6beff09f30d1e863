# Round 3, final build (no SLP): the c4 and c4t profiles with the bench commands.
set -u
D=gpurun_out/r03za
mkdir -p $D
timeout -k 10 900 bash tools/profile_gpu.sh r03 c4 --gpus 1 --steps 20 --warmup 5 > $D/prof_c4.log 2>&1 || { tail -20 $D/prof_c4.log; exit 1; }
grep -E "kernel_ms|rocprof_minus|timed_kernel" $D/prof_c4.log | head
timeout -k 10 900 bash tools/profile_gpu.sh r03 c4t --gpus 1 --steps 100 --warmup 5 > $D/prof_c4t.log 2>&1 || { tail -20 $D/prof_c4t.log; exit 1; }
grep -E "kernel_ms|rocprof_minus|write_size|timed_kernel" $D/prof_c4t.log | head
