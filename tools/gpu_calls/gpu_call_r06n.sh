# Round 6: (1) the shipped tree (STAGE 0 again) on the trajectory / step_many /
# every-lane / headline tests; (2) the stores' share of the rules trajectory:
# measurement builds that skip the small outputs (abl1) and also the records
# (abl2), alternating processes against the product, c3 and the bare
# trajectory at 2^20; (3) the phase timing of the shipped form; (4) the
# writers' rate against their buffer's size (tools/gpu_calls/gpu_call_r06m.sh).
set -u
. tools/gpu_calls/attempt.sh r06n
timeout -k 10 700 python -u -m pytest tests/test_gpu_every_lane.py tests/test_gpu_step_many.py tests/test_gpu_trajectory.py \
  tests/test_gpu_headline.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
L="open_spiel_coup_amd/libcoup_mi355x.so build/libab/abl1.so build/libab/abl2.so"
for c in "c3" "c2 --batch 1048576"; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 600 python -u tools/bench_ab.py --rounds 3 $L -- --config $c --steps 20 --warmup 5 > $D/ab_$n.jsonl 2> $D/ab_$n.err || { tail -20 $D/ab_$n.err; exit 1; }
  echo "== $c"; grep median $D/ab_$n.jsonl
done
COUP_LIB_PATH=build/libab/phases.so timeout -k 10 120 python -u tools/traj_phases.py > $D/traj_phases.jsonl 2> $D/traj_phases.err || { tail -20 $D/traj_phases.err; exit 1; }
cat $D/traj_phases.jsonl
bash tools/gpu_calls/gpu_call_r06m.sh
