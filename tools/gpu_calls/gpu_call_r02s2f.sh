# Round 2, session 2: regrouped N-player coup_step_trajectory -- parity tests, then c4t / c4 / c4r bench lines.
set -u
D=gpurun_out/r02s2f
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_trajectory.py -x -v --timeout 150 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
for c in c4t c4 c4r c2t; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $D/bench_$c.json 2> $D/bench_$c.err || { tail $D/bench_$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$D/bench_$c.json')); print('$c', '%.3e' % d['value'], round(d['roofline']['kernel_ms']*1e3/ (d['config']['fused_steps_per_launch']), 2), 'us/step', d['roofline']['kernel'])"
done
