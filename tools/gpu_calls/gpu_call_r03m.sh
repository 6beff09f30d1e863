# Round 3: the 6-player step's reset phase dealt by 4-thread groups (Philox
# blocks shared by shuffles); N-player parity, the facade / vector env / server
# suites (get_time_step and 1-2 env vector envs as lane ops), then the A/B of
# the reset forms and the facade latency rows.
set -u
D=gpurun_out/r03m
mkdir -p $D
timeout -k 10 700 python -u -m pytest tests/test_gpu_nplayer.py tests/test_gpu_vector_env.py tests/test_gpu_server.py tests/test_gpu_facade.py tests/test_gpu_slot_pool.py -m gpu -x -v --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python -u tools/ab_step.py --players 6 --obs 0 --rounds 9 --steps 20 COUP_NP_RESET_GROUP=1 COUP_NP_RESET_GROUP=4 > $D/ab_np_reset_group.jsonl 2> $D/ab_np.err || { tail -20 $D/ab_np.err; exit 1; }
cat $D/ab_np_reset_group.jsonl
timeout -k 10 400 python -u tools/facade_latency.py --rounds 3 --ops 600 > $D/facade_latency.json 2> $D/facade.err || { tail -20 $D/facade.err; exit 1; }
echo done
