# Round 2, session 2: 6-player step defaulting to 1024-lane blocks -- N-player suite, smoke, c4 bench line.
set -u
D=gpurun_out/r02s3a
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_nplayer.py tests/test_gpu_trajectory.py tests/test_gpu_vector_env.py -x -q --timeout 150 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline > $D/bench_c4.json 2>$D/bench_c4.err || { tail $D/bench_c4.err; exit 1; }
python -c "import json; d=json.load(open('$D/bench_c4.json')); print('c4', '%.3e' % d['value'], round(d['roofline']['kernel_ms']*1e3, 2), 'us/step')"
