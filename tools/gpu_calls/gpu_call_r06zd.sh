# Round 6: the rules trajectory storing each step's records as 8-byte
# obs_word (half the bytes; k_obs_sweep_words reads them) -- the step_many /
# every-lane / headline / trajectory / obs-split tests on the product, then
# alternating processes of c3: words at chunks of 10 (the product default)
# and 20 (one launch for K = 20: 160 MB of words at 2^20), against 16-byte
# records at 10 (measurement build, COUP_TRAJ_REC16=1).
set -u
. tools/gpu_calls/attempt.sh r06zd
timeout -k 10 700 python -u -m pytest tests/test_gpu_every_lane.py tests/test_gpu_step_many.py tests/test_gpu_trajectory.py \
  tests/test_gpu_headline.py tests/test_gpu_obs_split.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
P=open_spiel_coup_amd/libcoup_mi355x.so
V=build/variants/libcoup_mi355x.so
timeout -k 10 800 python -u tools/bench_ab.py --rounds 4 $P $P:COUP_TRAJ_CHUNK=20 $V:COUP_TRAJ_REC16=1 -- --config c3 --steps 20 --warmup 5 > $D/ab_c3.jsonl 2> $D/ab_c3.err || { tail -20 $D/ab_c3.err; exit 1; }
grep median $D/ab_c3.jsonl
