# Round-2 profiles of every bench config: plain bench lines with the CPU
# baseline, then tools/profile_gpu.sh (trace + FETCH/WRITE/SQ passes).
set -u
mkdir -p gpurun_out/r02m
bash tools/profile_gpu.sh r02 c3 --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02m/profile_c3.log 2>&1 || { tail -5 gpurun_out/r02m/profile_c3.log; exit 1; }
grep -A3 '"bench_vs_rocprof_kernel_ms"' gpurun_out/r02m/profile_c3.log | head -5
for c in c2 c2r c4 c4r c3i; do
  timeout -k 10 300 python -u bench.py --config $c --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02m/bench_$c.json 2> gpurun_out/r02m/bench_$c.err || exit $?
  cut -c1-200 gpurun_out/r02m/bench_$c.json
  bash tools/profile_gpu.sh r02 $c --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02m/profile_$c.log 2>&1 || { tail -5 gpurun_out/r02m/profile_$c.log; exit 1; }
done
