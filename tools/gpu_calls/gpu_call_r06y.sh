# Round 6: the lanes that finished on a chunk's last step dealt by a group
# gathered through LDS after the loop (product) instead of in place by every
# wave (fininplace.so, -DCOUP_TRAJ_FIN_INPLACE): the step_many / every-lane /
# headline / trajectory tests, then alternating processes, c3 and the bare
# trajectory at 2^20.
set -u
. tools/gpu_calls/attempt.sh r06y
timeout -k 10 700 python -u -m pytest tests/test_gpu_every_lane.py tests/test_gpu_step_many.py tests/test_gpu_trajectory.py \
  tests/test_gpu_headline.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
L="open_spiel_coup_amd/libcoup_mi355x.so build/libab/fininplace.so"
for c in "c3" "c2 --batch 1048576"; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 600 python -u tools/bench_ab.py --rounds 5 $L -- --config $c --steps 20 --warmup 5 > $D/ab_$n.jsonl 2> $D/ab_$n.err || { tail -20 $D/ab_$n.err; exit 1; }
  echo "== $c"; grep median $D/ab_$n.jsonl
done
