# Round 2, session 2: regrouped N-player trajectory with decision_mask at known decision nodes -- parity, A/B, c4t.
set -u
D=gpurun_out/r02s2h
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_trajectory.py -x -v --timeout 150 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python -u tools/traj_ab.py --players 6 > $D/traj_ab.jsonl 2>$D/err.log || { tail $D/err.log; exit 1; }
cat $D/traj_ab.jsonl
timeout -k 10 300 python -u bench.py --config c4t --no-cpu-baseline > $D/bench_c4t.json 2> $D/bench_c4t.err || { tail $D/bench_c4t.err; exit 1; }
python -c "import json,sys; d=json.load(open('$D/bench_c4t.json')); print('c4t', '%.3e' % d['value'], round(d['roofline']['kernel_ms']*1e3/ (d['config']['fused_steps_per_launch']), 2), 'us/step', d['roofline']['kernel'])"
