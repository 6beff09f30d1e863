# Round 3: rl_environment get_time_step and 1-2 env vector envs as lane ops;
# the facade, vector env and server suites, then the facade latency rows.
set -u
D=gpurun_out/r03l
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_vector_env.py tests/test_gpu_server.py tests/test_gpu_facade.py tests/test_gpu_slot_pool.py -m gpu -x -v --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 400 python -u tools/facade_latency.py --rounds 3 --ops 600 > $D/facade_latency.json 2> $D/facade.err || { tail -20 $D/facade.err; exit 1; }
echo done
