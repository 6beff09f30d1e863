# Round 4, seventh call: the CPython binding of the host State ops and the
# C-built time-step lists -- facade tests (both State modes), the whole GPU
# suite, the facade latencies, the vector-env profile; then the c4 profile
# (the r04f chain stopped before it).
set -u
D=gpurun_out/r04g
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_facade.py tests/test_gpu_slot_pool.py tests/test_gpu_unchecked.py tests/test_gpu_server.py tests/test_gpu_vector_env.py -x -q --timeout 200 --timeout-method thread > $D/pytest_facade.log 2>&1 || { tail -60 $D/pytest_facade.log; exit 1; }
tail -2 $D/pytest_facade.log
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 200 python -u tools/facade_latency.py --rounds 3 --ops 500 > $D/facade_latency.json 2> $D/facade_latency.err || { tail -5 $D/facade_latency.err; exit 1; }
python -c "import json;d=json.load(open('$D/facade_latency.json'));[print(k,v['median']) for k,v in d['rows_us'].items() if k.startswith(('host','vector','server_child','server_mccfr','rl_'))]"
timeout -k 10 240 python -u tools/vector_env_profile.py --steps 30 --top 15 > $D/vector_env_profile.txt 2>&1 || { tail -20 $D/vector_env_profile.txt; exit 1; }
grep "===" $D/vector_env_profile.txt
bash tools/profile_gpu.sh r04 c4
