# Round 6: balanced rules-trajectory chunks of up to 10 steps (the new
# default; K = 20 runs as 10 + 10): the step_many / every-lane / headline /
# trajectory tests, then alternating processes against COUP_TRAJ_CHUNK=8
# (now balanced: 7 + 7 + 6), then the driver's default line.
set -u
. tools/gpu_calls/attempt.sh r06x
timeout -k 10 700 python -u -m pytest tests/test_gpu_every_lane.py tests/test_gpu_step_many.py tests/test_gpu_trajectory.py \
  tests/test_gpu_headline.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
P=open_spiel_coup_amd/libcoup_mi355x.so
timeout -k 10 700 python -u tools/bench_ab.py --rounds 5 $P $P:COUP_TRAJ_CHUNK=8 -- --config c3 --steps 20 --warmup 5 > $D/ab_c3.jsonl 2> $D/ab_c3.err || { tail -20 $D/ab_c3.err; exit 1; }
grep median $D/ab_c3.jsonl
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_default.json 2> $D/bench_default.err || { tail -20 $D/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$D/bench_default.json')); r=d['roofline']; print('c3', d['value'], r['frac'], r['kernel_ms'], r['kernel'] == r['kernel_launched'])"
