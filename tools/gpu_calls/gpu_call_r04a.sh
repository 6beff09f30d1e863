# Round 4, first call: the packed episode word (new tests first), the
# bench.py --gpus launcher and the config-5 rehearsal, the c4 bench-path pin,
# then the whole GPU suite and the c3 / c2 lines.
set -u
D=gpurun_out/r04a
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_episode_word.py tests/test_gpu_headline.py tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread > $D/pytest_new.log 2>&1 || { tail -60 $D/pytest_new.log; exit 1; }
tail -3 $D/pytest_new.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $D/bench_c3.json 2> $D/bench_c3.err || { tail -5 $D/bench_c3.err; exit 1; }
cut -c1-400 $D/bench_c3.json
timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 5 > $D/bench_c2.json 2> $D/bench_c2.err || { tail -5 $D/bench_c2.err; exit 1; }
cut -c1-400 $D/bench_c2.json
