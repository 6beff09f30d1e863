# Round 3: the op server with two ring polls in flight -- the per-game suites
# through the server, then the facade latency table.
set -u
D=gpurun_out/r03v
mkdir -p $D
timeout -k 10 800 python -u -m pytest tests/test_gpu_server.py tests/test_gpu_slot_pool.py tests/test_gpu_facade.py tests/test_gpu_unchecked.py tests/test_rust_abi.py tests/test_gpu_cpp_api.py tests/test_policy_prefixes.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 400 python -u tools/facade_latency.py --rounds 5 > $D/facade_latency.json 2> $D/facade.err || { tail -20 $D/facade.err; exit 1; }
python -c "import json; d=json.load(open('$D/facade_latency.json')); [print(k, v) for k, v in d['rows_us'].items() if 'server' in k or 'rl_env' in k or 'children' in k]"
