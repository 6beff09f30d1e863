# Graph replay vs K eager launches (one event span, gated) per config.
set -u
mkdir -p gpurun_out/r02w
for c in c4 c3 c2 c3i; do for g in on off; do
  timeout -k 10 200 python -u bench.py --config $c --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --graph $g > gpurun_out/r02w/bench_${c}_$g.json 2> gpurun_out/r02w/bench_${c}_$g.err || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['gate_steps'])" gpurun_out/r02w/bench_${c}_$g.json
done; done
