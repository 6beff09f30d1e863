# Round 3: rl_environment reset/step as op-server lane ops (COUP_SLOT_RESET /
# COUP_SLOT_DEAL), info tensors via plain stores + one write-back; facade
# suites, then the facade latency table.
set -u
D=gpurun_out/r03h
mkdir -p $D
timeout -k 10 800 python -u -m pytest tests/test_gpu_server.py tests/test_gpu_slot_pool.py tests/test_gpu_facade.py tests/test_rust_abi.py tests/test_gpu_cpp_api.py tests/test_gpu_vector_env.py tests/test_gpu_trajectory.py -x -v -s --timeout 150 --timeout-method thread > $D/pytest.log 2>&1 || { tail -60 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 400 python -u tools/facade_latency.py --rounds 5 > $D/facade_latency.json 2> $D/facade.err || { tail -20 $D/facade.err; exit 1; }
python -c "import json; d=json.load(open('$D/facade_latency.json')); print(d['server_stats']); [print(k, v) for k, v in d['rows_us'].items()]"
