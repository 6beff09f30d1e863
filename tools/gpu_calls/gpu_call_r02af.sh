# Full GPU suite, then every bench config with its CPU baseline.
set -u
mkdir -p gpurun_out/r02af
bash tools/gpu_call_suite.sh r02af || exit $?
for c in c2 c2r c4 c4r c3i; do
  timeout -k 10 300 python -u bench.py --config $c --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02af/bench_$c.json 2> gpurun_out/r02af/bench_$c.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], '%.3e'%d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d['cpu_baseline']['value'])" gpurun_out/r02af/bench_$c.json
done
