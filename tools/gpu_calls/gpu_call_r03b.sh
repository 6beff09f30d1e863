# Round 3: the device-resident op server (coup_server_*): its own tests, the
# per-game facade suites that now run through it, then the facade latency
# table as interleaved repeats (server vs per-op launches).
set -u
D=gpurun_out/r03b
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_server.py tests/test_gpu_slot_pool.py tests/test_gpu_facade.py tests/test_rust_abi.py tests/test_gpu_cpp_api.py tests/test_gpu_vector_env.py -x -v -s --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { tail -60 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 400 python -u tools/facade_latency.py --rounds 5 > $D/facade_latency.json 2> $D/facade.err || { tail -20 $D/facade.err; exit 1; }
python -c "import json; d=json.load(open('$D/facade_latency.json')); print(d['server_stats']); [print(k, v) for k, v in d['rows_us'].items() if not k.startswith('vector')]"
