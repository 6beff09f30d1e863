# c4 phase timeline (COUP_WAVE_TRACE build) + fused-bench gate check + parity.
set -u
mkdir -p gpurun_out/r02n
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r02n/parity.log 2>&1 || { tail -20 gpurun_out/r02n/parity.log; exit 1; }
tail -2 gpurun_out/r02n/parity.log
COUP_LIB_PATH=ab/trace.so timeout -k 10 120 python -u tools/np_wave_trace.py --out gpurun_out/r02n/np_wave_trace.json || exit $?
for c in c2r c4r; do
  timeout -k 10 200 python -u bench.py --config $c --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02n/bench_$c.json 2> gpurun_out/r02n/bench_$c.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['roofline']['kernel_ms'])" gpurun_out/r02n/bench_$c.json
done
