# Round 2, session 2: coup_step_host (one launch into mapped host memory) for Environment / SyncVectorEnv --
# facade and vector-env suites, then the facade latency table.
set -u
D=gpurun_out/r02s2w
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_vector_env.py tests/test_gpu_facade.py tests/test_gpu_slot_pool.py tests/test_capi.py -x -v --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 400 python -u tools/facade_latency.py > $D/facade_latency.json 2> $D/facade.err || { tail -3 $D/facade.err; exit 1; }
python -c "import json; d=json.load(open('$D/facade_latency.json')); print({k: v for k, v in d.items() if k.startswith(('pool_child', 'rl_', 'vector'))})"
