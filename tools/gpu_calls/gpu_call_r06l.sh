# Round 6: the rules trajectories' step outputs staged by lane and stored by
# each lane's home thread behind the next step's count barrier (STAGE 2, the
# product) against the playing thread's scattered stores (stage0.so,
# -DCOUP_TRAJ_OUT_STAGE=0): the trajectory / step_many / every-lane / headline
# tests on the product, alternating-process bench lines (c3, the bare rules
# trajectory at 2^20), the phase timing of the STAGE 2 build.
set -u
. tools/gpu_calls/attempt.sh r06l
timeout -k 10 700 python -u -m pytest tests/test_gpu_every_lane.py tests/test_gpu_step_many.py tests/test_gpu_trajectory.py \
  tests/test_gpu_headline.py tests/test_gpu_vector_env.py tests/test_gpu_obs_split.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
L="build/libab/stage0.so open_spiel_coup_amd/libcoup_mi355x.so"
for c in "c3" "c2 --batch 1048576"; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 600 python -u tools/bench_ab.py --rounds 4 $L -- --config $c --steps 20 --warmup 5 > $D/ab_$n.jsonl 2> $D/ab_$n.err || { tail -20 $D/ab_$n.err; exit 1; }
  echo "== $c"; grep median $D/ab_$n.jsonl
done
COUP_LIB_PATH=build/libab/phases.so timeout -k 10 120 python -u tools/traj_phases.py > $D/traj_phases.jsonl 2> $D/traj_phases.err || { tail -20 $D/traj_phases.err; exit 1; }
cat $D/traj_phases.jsonl
