# Round 4, eleventh call: SyncVectorEnv keeps host-resident games on the host
# (vector_env.HOST_UPTO): the vector-env / unchecked / server tests in both
# state modes, then the facade latency rows (kept / adopted / loop forms).
set -u
D=gpurun_out/r04k
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_vector_env.py tests/test_gpu_unchecked.py tests/test_gpu_server.py tests/test_gpu_facade.py -x -q --timeout 120 --timeout-method thread > $D/pytest_env.log 2>&1 || { tail -40 $D/pytest_env.log; exit 1; }
tail -2 $D/pytest_env.log
timeout -k 10 400 python -u tools/facade_latency.py > $D/facade.json 2> $D/facade.err || { tail -20 $D/facade.err; exit 1; }
python -c "
import json; d=json.load(open('$D/facade.json'))['rows_us']
for k,v in d.items():
    if k.startswith(('vector','rl_env')): print(k, v['median'])"
