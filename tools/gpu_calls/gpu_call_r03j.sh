# Round 3: r03h (Environment lane ops: tests + facade table) and r03i (measurement set) in one lease.
D=gpurun_out/r03j
mkdir -p $D
timeout -k 10 800 python -u -m pytest tests/test_gpu_server.py tests/test_gpu_slot_pool.py tests/test_gpu_facade.py tests/test_rust_abi.py tests/test_gpu_cpp_api.py tests/test_gpu_vector_env.py tests/test_gpu_trajectory.py -x -v -s --timeout 150 --timeout-method thread > $D/pytest.log 2>&1 || { tail -60 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 400 python -u tools/facade_latency.py --rounds 5 > $D/facade_latency.json 2> $D/facade.err || { tail -20 $D/facade.err; exit 1; }
python -c "import json; d=json.load(open('$D/facade_latency.json')); print(d['server_stats']); [print(k, v) for k, v in d['rows_us'].items()]"
bash tools/boxinfo.sh > $D/box.txt 2>&1 || true
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_c3.json 2> $D/bench_c3.err || { tail -5 $D/bench_c3.err; exit 1; }
cut -c1-300 $D/bench_c3.json
timeout -k 10 200 ./build/store_probe > $D/store_probe.jsonl 2> $D/store_probe.err || { tail -5 $D/store_probe.err; exit 1; }
tail -4 $D/store_probe.jsonl
for c in c4 c4t c2; do
  st=20; [ $c = c4t ] && st=100
  timeout -k 10 300 python -u bench.py --gpus 1 --config $c --steps $st --warmup 5 > $D/bench_$c.json 2> $D/bench_$c.err || { tail -5 $D/bench_$c.err; exit 1; }
  cut -c1-200 $D/bench_$c.json
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $D/bench_c3_again.json 2> $D/bench_c3b.err || { tail -5 $D/bench_c3b.err; exit 1; }
cut -c1-200 $D/bench_c3_again.json
timeout -k 10 900 bash tools/profile_gpu.sh r03 c4 --gpus 1 --steps 20 --warmup 5 > $D/prof_c4.log 2>&1 || { tail -20 $D/prof_c4.log; exit 1; }
grep -E "kernel_ms|rocprof_minus|timed_kernel" $D/prof_c4.log | head
