# Round 6: the sorted kernels with two barriers per step (product) against the
# same code with the third, top-of-step barrier (v1, -DCOUP_TRAJ_TOP_BARRIER:
# the packed-record carry only) and the round's previous product build (base):
# the whole GPU suite on the product build,
# then alternating-process bench lines: c3, the bare rules trajectory at 2^20,
# c4, c2r, c4r.
set -u
. tools/gpu_calls/attempt.sh r06k
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
L="build/libab/base.so build/libab/v1.so open_spiel_coup_amd/libcoup_mi355x.so"
for c in "c3" "c2 --batch 1048576" "c4" "c2r" "c4r"; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 600 python -u tools/bench_ab.py --rounds 3 $L -- --config $c --steps 20 --warmup 5 > $D/ab_$n.jsonl 2> $D/ab_$n.err || { tail -20 $D/ab_$n.err; exit 1; }
  echo "== $c"; grep median $D/ab_$n.jsonl
done
# where the rules trajectory's waves spend a step (COUP_TRAJ_PHASES build)
COUP_LIB_PATH=build/libab/phases.so timeout -k 10 120 python -u tools/traj_phases.py > $D/traj_phases.jsonl 2> $D/traj_phases.err || { tail -20 $D/traj_phases.err; exit 1; }
cat $D/traj_phases.jsonl
