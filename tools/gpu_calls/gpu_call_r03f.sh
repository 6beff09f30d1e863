# Round 3: fence-free op server; c4t outputs staged by lane and stored as whole
# words per block; their tests, A/B, the c4t profile, the facade latency table.
set -u
D=gpurun_out/r03f
mkdir -p $D
timeout -k 10 700 python -u -m pytest tests/test_gpu_server.py tests/test_gpu_slot_pool.py tests/test_gpu_facade.py tests/test_rust_abi.py tests/test_gpu_cpp_api.py tests/test_gpu_trajectory.py -x -v -s --timeout 150 --timeout-method thread > $D/pytest.log 2>&1 || { tail -60 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 300 python -u tools/traj_ab.py --players 6 --steps 100 --rounds 7 > $D/traj_ab_6p.jsonl 2> $D/traj_ab.err || { tail -20 $D/traj_ab.err; exit 1; }
cat $D/traj_ab_6p.jsonl
timeout -k 10 400 python -u tools/facade_latency.py --rounds 5 --no-vector > $D/facade_latency.json 2> $D/facade.err || { tail -20 $D/facade.err; exit 1; }
python -c "import json; d=json.load(open('$D/facade_latency.json')); print(d['server_stats']); [print(k, v) for k, v in d['rows_us'].items() if not k.startswith('vector')]"
timeout -k 10 900 bash tools/profile_gpu.sh r03 c4t --gpus 1 --steps 100 --warmup 5 > $D/prof_c4t.log 2>&1 || { tail -20 $D/prof_c4t.log; exit 1; }
grep -E "kernel_ms|write_size|fetch_size|rocprof_minus|timed_kernel" $D/prof_c4t.log | head
