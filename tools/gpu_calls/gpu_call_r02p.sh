# c4 phase timeline (COUP_WAVE_TRACE build) + fused-bench gate check.
set -u
mkdir -p gpurun_out/r02p
COUP_LIB_PATH=ab/trace.so timeout -k 10 120 python -u tools/np_wave_trace.py --out gpurun_out/r02p/np_wave_trace.json > gpurun_out/r02p/np_wave_trace.log || exit $?
for c in c2r c4r; do
  timeout -k 10 200 python -u bench.py --config $c --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02p/bench_$c.json 2> gpurun_out/r02p/bench_$c.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['gate_steps'])" gpurun_out/r02p/bench_$c.json
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r02p/prof_c2r -o run -- python3 bench.py --config c2r --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02p/prof_c2r.log 2>&1 || exit $?
find gpurun_out/r02p/prof_c2r -name '*kernel_stats.csv' -exec head -3 {} \;
