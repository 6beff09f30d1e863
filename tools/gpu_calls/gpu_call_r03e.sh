# Round 3: the device-resident op server (coup_server_*) with the per-game
# facade suites that now run through it; the c4t trajectory with outputs staged
# by lane; the 6-player step with inline resets (kKeyEnding); A/B of both, the
# c4t profile, then the facade latency table (interleaved repeats).
set -u
D=gpurun_out/r03e
mkdir -p $D
timeout -k 10 700 python -u -m pytest tests/test_gpu_server.py tests/test_gpu_slot_pool.py tests/test_gpu_facade.py tests/test_rust_abi.py tests/test_gpu_cpp_api.py tests/test_gpu_vector_env.py tests/test_gpu_trajectory.py tests/test_gpu_nplayer.py -x -v -s --timeout 150 --timeout-method thread > $D/pytest.log 2>&1 || { tail -60 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 300 python -u tools/ab_step.py --players 6 --obs 0 --rounds 9 --steps 20 COUP_NP_RESET_INLINE=1 COUP_NP_RESET_INLINE=0 > $D/ab_np_reset_inline.jsonl 2> $D/ab_np.err || { tail -20 $D/ab_np.err; exit 1; }
cat $D/ab_np_reset_inline.jsonl
timeout -k 10 300 python -u tools/traj_ab.py --players 6 --steps 100 --rounds 7 > $D/traj_ab_6p.jsonl 2> $D/traj_ab.err || { tail -20 $D/traj_ab.err; exit 1; }
cat $D/traj_ab_6p.jsonl
timeout -k 10 400 python -u tools/facade_latency.py --rounds 5 > $D/facade_latency.json 2> $D/facade.err || { tail -20 $D/facade.err; exit 1; }
python -c "import json; d=json.load(open('$D/facade_latency.json')); print(d['server_stats']); [print(k, v) for k, v in d['rows_us'].items() if not k.startswith('vector')]"
timeout -k 10 900 bash tools/profile_gpu.sh r03 c4t --gpus 1 --steps 100 --warmup 5 > $D/prof_c4t.log 2>&1 || { tail -20 $D/prof_c4t.log; exit 1; }
grep -E "kernel_ms|write_size|fetch_size|rocprof_minus" $D/prof_c4t.log | head
