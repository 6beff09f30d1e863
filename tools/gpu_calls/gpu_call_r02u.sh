# Default regroup blocks 512 (step) / 1024 (rollout): N-player parity, A/B against 256, c4 / c4r bench lines.
set -u
mkdir -p gpurun_out/r02u
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nplayer.py > gpurun_out/r02u/nplayer.log 2>&1 || { tail -20 gpurun_out/r02u/nplayer.log; exit 1; }
tail -1 gpurun_out/r02u/nplayer.log
timeout -k 10 300 python -u tools/ab_step.py --players 6 --obs 0 --rounds 7 COUP_NP_SORT_THREADS=256 COUP_NP_SORT_THREADS=512 COUP_NP_SORT_THREADS=1024 > gpurun_out/r02u/ab_step6.log 2>&1 || { tail gpurun_out/r02u/ab_step6.log; exit 1; }
grep variant gpurun_out/r02u/ab_step6.log
timeout -k 10 300 python -u tools/ab_step.py --players 6 --obs 0 --rounds 7 --fused 20 COUP_NP_SORT_THREADS=256 COUP_NP_SORT_THREADS=1024 > gpurun_out/r02u/ab_rollout6.log 2>&1 || { tail gpurun_out/r02u/ab_rollout6.log; exit 1; }
grep variant gpurun_out/r02u/ab_rollout6.log
for c in c4 c4r; do
  timeout -k 10 200 python -u bench.py --config $c --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02u/bench_$c.json 2> gpurun_out/r02u/bench_$c.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['kernel'])" gpurun_out/r02u/bench_$c.json
done
COUP_LIB_PATH=ab/trace.so timeout -k 10 120 python -u tools/np_wave_trace.py --out gpurun_out/r02u/np_wave_trace_512.json > gpurun_out/r02u/np_wave_trace_512.log || exit $?
