# Round 4, tenth call: rl_environment.Environment host-resident (its game a
# host state; reset / step through coup_host_state_step): the facade, server,
# unchecked and vector-env tests, the whole GPU suite, then the facade
# latency rows (host env step beside the device-lane env step).
set -u
D=gpurun_out/r04j
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_facade.py tests/test_gpu_server.py tests/test_gpu_unchecked.py tests/test_gpu_vector_env.py tests/test_host_state.py -x -q --timeout 120 --timeout-method thread > $D/pytest_env.log 2>&1 || { tail -40 $D/pytest_env.log; exit 1; }
tail -2 $D/pytest_env.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python -u tools/facade_latency.py > $D/facade.json 2> $D/facade.err || { tail -20 $D/facade.err; exit 1; }
cat $D/facade.json
