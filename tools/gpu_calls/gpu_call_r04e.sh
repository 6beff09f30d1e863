# Round 4, fifth call: host-resident per-game States (default) next to the
# device-lane ones -- the facade tests in both modes, the whole GPU suite,
# smoke(), and the facade latencies (host / server / launch rows, MCCFR-shaped
# node, SyncVectorEnv).
set -u
D=gpurun_out/r04e
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_facade.py tests/test_gpu_slot_pool.py tests/test_gpu_unchecked.py tests/test_gpu_server.py -x -q --timeout 200 --timeout-method thread > $D/pytest_facade.log 2>&1 || { tail -60 $D/pytest_facade.log; exit 1; }
tail -2 $D/pytest_facade.log
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -60 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 200 python -u tools/facade_latency.py --rounds 3 --ops 500 > $D/facade_latency.json 2> $D/facade_latency.err || { tail -5 $D/facade_latency.err; exit 1; }
python -c "import json;d=json.load(open('$D/facade_latency.json'));[print(k,v['median']) for k,v in d['rows_us'].items()]"
