# Round 3: N-player kernels at -O2 -- the N-player and trajectory suites, then
# the c4 and c4t bench lines.
set -u
D=gpurun_out/r03x
mkdir -p $D
timeout -k 10 800 python -u -m pytest tests/test_gpu_nplayer.py tests/test_gpu_trajectory.py tests/test_gpu_vector_env.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
for c in c4 c4t; do
  st=20; [ $c = c4t ] && st=100
  timeout -k 10 300 python -u bench.py --gpus 1 --config $c --steps $st --warmup 5 --no-cpu-baseline > $D/bench_$c.json 2> $D/bench_$c.err || { tail -5 $D/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$D/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
