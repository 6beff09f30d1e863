# Round 6: two more cuts of the 2-player rules trajectory's work, as
# measurement builds against the product (alternating processes, c3 and the
# bare trajectory at 2^20): refined regroup keys (-DCOUP_REFINE_KEYS: a Pass
# by what it completes, a Challenge by its outcome, so the deal waves sort
# apart) and the loop-free policy draw (-DCOUP_TRAJ_SELECT_DRAW).
set -u
. tools/gpu_calls/attempt.sh r06o
L="open_spiel_coup_amd/libcoup_mi355x.so build/libab/refine.so build/libab/select.so"
for c in "c3" "c2 --batch 1048576"; do
  n=$(echo $c | tr -d ' -')
  timeout -k 10 600 python -u tools/bench_ab.py --rounds 3 $L -- --config $c --steps 20 --warmup 5 > $D/ab_$n.jsonl 2> $D/ab_$n.err || { tail -20 $D/ab_$n.err; exit 1; }
  echo "== $c"; grep median $D/ab_$n.jsonl
done
