# Round 2, session 2: coup_step_trajectory and the 6-player reset-store step -- parity tests, same-process A/B of
# the reset store, bench lines of c2 / c2t / c4 / c4t.
set -u
D=gpurun_out/r02s2e
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_trajectory.py tests/test_gpu_nplayer.py -x -v --timeout 150 --timeout-method thread -k "trajectory or reset_store or regrouped_step_equals" > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python -u tools/ab_step.py --players 6 --obs 0 --rounds 9 --steps 20 COUP_NP_RESET_STORE=0 COUP_NP_RESET_STORE=1 COUP_NP_RESET_STORE=0,COUP_NP_SORT_THREADS=1024 COUP_NP_RESET_STORE=1,COUP_NP_SORT_THREADS=1024 > $D/ab_c4_reset_store.jsonl 2>$D/ab.err || { tail $D/ab.err; exit 1; }
cat $D/ab_c4_reset_store.jsonl
for c in c2 c2t c4 c4t; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $D/bench_$c.json 2> $D/bench_$c.err || { tail $D/bench_$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$D/bench_$c.json')); print('$c', '%.3e' % d['value'], round(d['roofline']['kernel_ms']*1e3/ (d['config']['fused_steps_per_launch']), 2), 'us/step', d['roofline']['kernel'])"
done
